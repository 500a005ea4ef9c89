"""Capture the problems the conditioned select kernel hands over inside the
device outer loop (quadrotor, tools/bench_forward.py's batch; VERDICT r03
item 2).  Each select is run once more with HOP_OPT_NO_RERUN (HOP_ST_HANDOVER
left in status); the trajectory-form inputs of every handed-over problem are
saved to an npz fixture with the select's parameters.

    python tools/handover_capture.py [B] [out.npz]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from time_opt_ilqr_amd import _lib, engine, solver, systems  # noqa: E402
from oracle import ilqr_oracle as io  # noqa: E402

Bn = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
out = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/handover_capture.npz"
N, iters = 100, 5
F, x0, xg, u_ref, Q, R, alpha, w, _, _, _, wrap, _ = systems.make_quadrotor(N=N)
rng = np.random.default_rng(9)
X0 = x0 + 0.2 * rng.standard_normal((Bn, F.n))
Qf = io.orc.terminal_weight(alpha, F.n)
orig = engine.propagate_traj
caps = {}
log = []


def probe(*a, **k):
    with _lib.options(no_rerun=True):
        r = orig(*a, **k)
    st = r.status.cpu().numpy()
    flagged = np.nonzero(st & _lib.ST_HANDOVER)[0]
    sel = len(log)
    full = orig(*a, **k)
    log.append((len(st), flagged.tolist(), full.status.cpu().numpy()[flagged].tolist(),
                [(int(st[i]) >> 5) & 255 for i in flagged], [int(st[i]) >> 13 for i in flagged]))
    names = ("A", "B", "a_res", "X", "U", "xg", "u_ref", "Q", "R_inv", "P", "w")
    for i in flagged.tolist():
        for nm, t in zip(names, a):
            v = t.detach().cpu().numpy()
            caps[f"s{sel}_p{i}_{nm}"] = v[i] if v.ndim >= 1 and v.shape[0] == len(st) and \
                nm in ("A", "B", "a_res", "X", "U") else v
        caps[f"s{sel}_p{i}_J"] = full.J.cpu().numpy()[i]
        caps[f"s{sel}_p{i}_tstar"] = int(full.t_star.cpu().numpy()[i])
        caps[f"s{sel}_p{i}_status"] = int(full.status.cpu().numpy()[i])
        caps[f"s{sel}_p{i}_kw"] = np.array([k.get("t_min", 0), k.get("t_max", 0),
                                            k.get("n_use") or 0])
        caps[f"s{sel}_p{i}_wrap"] = np.array(k.get("wrap_idx") or [], dtype=np.int64)
    return full


engine.propagate_traj = probe
solver.engine.propagate_traj = probe
res = solver.ilqr_timeopt_batch(2, X0, xg, u_ref, Q, R, Qf, w, N, max(1, N // 5), N, dt=F.dt,
                                max_iter=iters, wrap_idx=wrap, use_central_diff=False)
for i, (b, idx, sts, why, at) in enumerate(log):
    print(f"select {i}: batch {b}, handed over {len(idx)}: {idx[:12]} final status {sts[:12]}"
          f" reason bits {why[:12]} (developer builds) at horizon {at[:12]}")
print("crashed", int(res["crashed"].sum().item()))
os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
np.savez_compressed(out, **caps)
print("saved", len(caps), "arrays to", out)
