"""Bitwise check of the s <= 5 rerun paths on blocks with many LU steps: real cart-pole
augmented blocks (fp64, s = 5, N = 200) with Q_aug[k][0][0] - 1 at every odd k, so
chol_inv's ladder ends in the LU slot there; one to four hand-overs per workgroup
through the pipelined rerun (default), the one-lane rerun (HOP_OPT_RERUN_LANE) and the
reference association alone (HOP_OPT_REFERENCE_ASSOC).  Prints status, T* and the J
mismatch counts.  The same case is tests/test_gpu_small_rowgroup.py::
test_pipelined_small_rerun_many_lu_steps_bitwise; this script found that a side-by-side
jitter ladder differed in the last bits.

    python tools/dbg_handover.py     (HOP_LIB=<path> for another library)
"""
import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from time_opt_ilqr_amd import _lib, engine, systems
from time_opt_ilqr_amd.utils import as_terminal_weight
dev = torch.device("cuda", 0)
N, Bn = 200, 64
F, x0, xg, u_ref, Q, R, alpha, w, _, _, _, wrap, _ = systems.make_cartpole_swingup(N=N)
g = torch.Generator(device=dev); g.manual_seed(29)
kw = dict(device=dev, dtype=torch.float64, generator=g)
U = torch.as_tensor(u_ref, device=dev) + 2.0 * torch.randn((Bn, N, F.m), **kw)
X = engine.rollout(F.system_id, torch.as_tensor(x0, device=dev) + 0.3 * torch.randn((Bn, F.n), **kw), U, F.dt)
t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float64), device=dev)
P = t(as_terminal_weight(alpha, F.n)); Ri = torch.linalg.inv(t(R)).contiguous()
lin = engine.linearize(F.system_id, X, U, F.dt, central=True)
blk = engine.augment(lin.A, lin.B, lin.a_res, X, U, t(xg), t(u_ref), t(Q), P, w, wrap_idx=wrap)
for nb in (1, 2, 3, 4):
    h = slice(0, nb)
    Qh = blk.Q[h].clone(); Qh[:, 1::2, 0, 0] -= 1.0
    hargs = (blk.A[h].contiguous(), blk.B[h].contiguous(), Qh, Ri, blk.z0, blk.QT[h].contiguous())
    a = engine.propagate(*hargs, t_min=50, t_max=N)
    with _lib.options(rerun_lane=True):
        b = engine.propagate(*hargs, t_min=50, t_max=N)
    with _lib.options(reference_assoc=True):
        c = engine.propagate(*hargs, t_min=50, t_max=N)
    torch.cuda.synchronize()
    Ja, Jb, Jc = a.J.cpu().numpy(), b.J.cpu().numpy(), c.J.cpu().numpy()
    print(nb, "status", a.status.tolist(), b.status.tolist(), c.status.tolist(), "tstar", a.t_star.tolist(), b.t_star.tolist())
    d = ~((Ja == Jb) | (np.isnan(Ja) & np.isnan(Jb)))
    print("  J mismatches pipe vs lane:", int(d.sum()), "first", np.argwhere(d)[:3].tolist(), "lane vs ref", int((~((Jb == Jc) | (np.isnan(Jb) & np.isnan(Jc)))).sum()))
    if d.any():
        i, k = np.argwhere(d)[0]
        print("  values", Ja[i, k-1:k+2], Jb[i, k-1:k+2])
