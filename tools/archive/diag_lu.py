import os, sys
import numpy as np
sys.path.insert(0, os.getcwd())
import torch
from oracle import hop_oracle as orc
from time_opt_ilqr_amd import _lib, engine
dev = torch.device("cuda", 0)
_lib.check(_lib.load().hop_set_options(_lib.OPT_FORCE_GENERIC, 0))  # the generic kernel
for s, m in ((4, 2), (4, 1), (3, 1), (5, 1), (5, 2)):
    Bn, N = 131, 40
    A, Bm, Q, R, Ri, z0, QT = orc.synth_lft_batch(900 + s, Bn, s, m, N)
    Q = Q.copy()
    Q[7, 3] = Q[7, 3] - np.eye(s) * (np.linalg.eigvalsh(Q[7, 3]).min() + 5e-7)
    sl = slice(7, 8)
    t = lambda x: torch.as_tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev)
    r = engine.propagate(t(A[sl]), t(Bm[sl]), t(Q[sl]), t(Ri[sl]), t(z0[0]), t(QT[sl]),
                         return_efg=True, return_prefix=True)
    o = orc.lft_sweep(A[7], Bm[7], Q[7], Ri[7], z0[0], QT[7], want_efg=True, want_prefix=True)
    st = int(r.status[0])
    efg = r.efg[0].cpu().numpy()
    msg = []
    for key, idx in (("E", 0), ("F", 1), ("G", 2)):
        ref = o[key][:N]
        got = efg[:, idx]
        msg.append(f"{key} rel {np.max(np.abs(got - ref)) / np.max(np.abs(ref)):.1e}")
    Jr = r.J[0].cpu().numpy()
    print(s, m, "status", st, "oracle", o.get("status"), " ".join(msg),
          "J rel", f"{np.max(np.abs(Jr - o['J']) / np.abs(o['J'])):.1e}", flush=True)
