"""Dev probe: first mismatches of the fast kernel vs the reference loop fixture (prints hex)."""
import sys
import numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
from conftest import load_golden
from test_gpu_parity import _engine_from_fixture, REC
from p2pmicrogrid_amd.engine import unpack_index

d = load_golden(sys.argv[1] if len(sys.argv) > 1 else "loop_thesis_T96")
for kernel in ("general", "auto"):
    eng = _engine_from_fixture(d)
    e = 0
    eng.set_temperatures(d["t_in0"][e][None], d["t_m0"][e][None])
    eng.set_replay_codes(d["codes"][e])
    eng.run_episode("train", "replay", episode=e, epsilon=float(d["eps"][e]), record=REC, kernel=kernel)
    rec = eng.get_records(REC)
    print("==", kernel)
    for k in ("reward", "cost", "grid", "p2p", "t_in"):
        g, w = rec[k][:, 0], d[f"train_{k}"][e]
        bad = np.argwhere(g != w)
        if len(bad):
            t, a = bad[0]
            print(k, "n_bad", len(bad), "first", (t, a), g[t, a], w[t, a], hex(g[t, a].view(np.uint32)), hex(w[t, a].view(np.uint32)))
    ga, wa = rec["action"][:, :, 0], d["train_action"][e]
    bad = np.argwhere(ga != wa)
    print("action n_bad", len(bad), bad[:3].tolist())
    gi, wi = unpack_index(rec["index"][:, :, 0]), d["train_idx"][e]
    bad = np.argwhere(gi != wi)
    print("index n_bad", len(bad), bad[:3].tolist(), gi[tuple(bad[0][:3])] if len(bad) else "", wi[tuple(bad[0][:3])] if len(bad) else "")
