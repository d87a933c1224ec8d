#!/bin/bash
# dev: recompile only p2pmg_dqn.hip into build/obj/main and relink libp2pmg.so to OUT (default: in-tree)
R=/root/repo; O=$R/build/obj/main; OUT=${1:-$R/p2pmicrogrid_amd/libp2pmg.so}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wall -Wno-unused-function -Wno-pass-failed \
  -I$R/include -I$R/p2pmicrogrid_amd/csrc $EXTRA -c $R/p2pmicrogrid_amd/csrc/p2pmg_dqn.hip -o $O/p2pmg_dqn.o || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $O/kernels_*.o $O/p2pmg_dqn.o $O/p2pmg_runtime.o -o $OUT.tmp && mv $OUT.tmp $OUT
