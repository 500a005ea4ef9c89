"""Drop-ins for the reference's linearization.py on the device.

  linearize_forward_diff_traj(F, X, U, epsx, epsu, relx, relu)   linearization.py:216-262
  linearize_central_diff_traj(F, X, U, epsx, epsu, relx, relu)   linearization.py:177-211
  compute_affine_residuals(F, X, U)                              linearization.py:269-270

Same names, arguments and return shapes (lists of per-step NumPy blocks) for one
trajectory; ``linearize_batch`` is the batched device form (torch tensors in
HBM, the layout engine.propagate_traj / engine.riccati read).  ``F`` must be a
:class:`~time_opt_ilqr_amd.systems.DeviceDynamics` (a system the kernel knows):
an arbitrary Python callable is refused with TypeError rather than evaluated on
the CPU.
"""
from __future__ import annotations

import numpy as np

from . import engine
from .systems import DeviceDynamics


def _check_F(F):
    if not isinstance(F, DeviceDynamics):
        raise TypeError("F must be a time_opt_ilqr_amd.systems DeviceDynamics (the device "
                        "linearisation has no path for arbitrary Python dynamics)")
    return F


def _run(F, X, U, central, epsx, epsu, relx, relu):
    import torch
    F = _check_F(F)
    X = np.asarray(X, dtype=float)
    U = np.asarray(U, dtype=float)
    if U.ndim == 1:
        U = U.reshape(-1, F.m)
    N = len(U)
    dev = torch.device("cuda", torch.cuda.current_device())
    Xt = torch.as_tensor(np.ascontiguousarray(X[:N + 1]), device=dev)
    if Xt.shape[0] < N + 1:  # the linearisations only read X[:N]
        Xt = torch.cat([Xt, Xt[-1:].expand(N + 1 - Xt.shape[0], -1)], 0)
    Ut = torch.as_tensor(np.ascontiguousarray(U), device=dev)
    return engine.linearize(F.system_id, Xt[None], Ut[None], F.dt, central=central,
                            epsx=epsx, epsu=epsu, relx=relx, relu=relu)


def linearize_forward_diff_traj(F, X, U, epsx: float = 1e-5, epsu: float = 1e-5,
                                relx: float = 1e-6, relu: float = 1e-6):
    """Forward differences with h = max(eps, rel * max(1, |v|)); an all-NaN
    (A_k, B_k) where F(x_k, u_k) is not finite.  Returns (A_list, B_list)."""
    if len(U) == 0:
        return [], []
    r = _run(F, X, U, False, epsx, epsu, relx, relu)
    return list(r.A[0].cpu().numpy()), list(r.B[0].cpu().numpy())


def linearize_central_diff_traj(F, X, U, epsx: float = 1e-5, epsu: float = 1e-5,
                                relx: float = 1e-6, relu: float = 1e-6):
    """Central differences (F(v + h e) - F(v - h e)) / 2h.  Returns (A_list, B_list)."""
    if len(U) == 0:
        return [], []
    r = _run(F, X, U, True, epsx, epsu, relx, relu)
    return list(r.A[0].cpu().numpy()), list(r.B[0].cpu().numpy())


def compute_affine_residuals(F, X, U):
    """[F(x_k, u_k) - x_{k+1}] as (n, 1) columns, k < len(U)."""
    if len(U) == 0:
        return []
    r = _run(F, X, U, False, 1e-5, 1e-5, 1e-6, 1e-6)
    return [a.reshape(-1, 1) for a in r.a_res[0].cpu().numpy()]


def linearize_batch(F, X, U, *, central: bool = False, n_use=None, epsx: float = 1e-5,
                    epsu: float = 1e-5, relx: float = 1e-6, relu: float = 1e-6,
                    want_fx: bool = False) -> "engine.Linearization":
    """Batched form: X [B, N+1, n], U [B, N, m] fp64 device tensors ->
    engine.Linearization(A [B, N, n, n], B [B, N, n, m], a_res [B, N, n])."""
    F = _check_F(F)
    return engine.linearize(F.system_id, X, U, F.dt, central=central, n_use=n_use, epsx=epsx,
                            epsu=epsu, relx=relx, relu=relu, want_fx=want_fx)
