#!/bin/bash
# dev: recompile only p2pmg_dqn.hip (with $EXTRA flags, e.g. -DP2PMG_TRACE=1) and relink libp2pmg.so
# from build/obj/main's other objects to OUT (default: in-tree)
R=/root/repo; O=$R/build/obj/main; OUT=${1:-$R/p2pmicrogrid_amd/libp2pmg.so}
DO=$O/p2pmg_dqn.o; [ -n "$EXTRA" ] && DO=$O/p2pmg_dqn_extra.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wall -Wno-unused-function -Wno-pass-failed \
  -I$R/include -I$R/p2pmicrogrid_amd/csrc $EXTRA -c $R/p2pmicrogrid_amd/csrc/p2pmg_dqn.hip -o $DO || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $O/kernels_*.o $DO $O/p2pmg_runtime.o -o $OUT.tmp && mv $OUT.tmp $OUT
