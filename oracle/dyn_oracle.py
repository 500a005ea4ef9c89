"""CPU restatement of the batched dynamics + finite-difference linearisation
(SURVEY.md section 8(f) rank 2).  TEST INFRASTRUCTURE ONLY: imported by tests/,
``__graft_entry__.smoke()`` and the CPU-baseline leg of tools/bench_linearize.py,
never by the product path (time_opt_ilqr_amd calls hop_linearize_f64 and fails
loudly without the HIP library).

Restates, in NumPy:
  F of the five benchmark systems ........... systems.py:28-349
      double integrator 30-33, cart-pole 72-95, quadrotor 170-210 (guards
      175-191), point mass 239-249, segway 321-333; angle_normalize utils.py:127-128
  linearize_forward_diff_traj ............... linearization.py:216-262
  linearize_central_diff_traj ............... linearization.py:177-211
  compute_affine_residuals .................. linearization.py:269-270

``dynamics`` / ``linearize`` are vectorised over any leading batch shape (the
checker for large GPU runs); ``linearize_loop`` keeps the reference's per-step,
per-column loop with one F call at a time (the CPU baseline).

Parity pinning: tests/golden/lin_*.npz hold F, both linearisations and the
residuals computed by the reference itself (tests/golden/make_golden.py --lin);
tests/test_oracle_golden.py checks this module against them.
"""
from __future__ import annotations

import math

import numpy as np

SYSTEMS = {"di": 0, "cartpole": 1, "quadrotor": 2, "pointmass": 3, "segway": 4}
DIMS = {0: (2, 1), 1: (4, 1), 2: (12, 4), 3: (4, 2), 4: (4, 1)}
DEFAULT_DT = {0: 0.05, 1: 0.02, 2: 0.05, 3: 0.05, 4: 0.02}  # the makers' defaults


def angle_normalize(a):
    """utils.py:127-128: (a + pi) % (2 pi) - pi (floor-mod semantics)."""
    return np.remainder(a + np.pi, 2.0 * np.pi) - np.pi


def _f_di(x, u, dt):  # systems.py:30-33
    return np.stack([x[..., 0] + dt * x[..., 1], x[..., 1] + dt * u[..., 0]], -1)


def _f_cartpole(x, u, dt):  # systems.py:72-95
    g, m_cart, m_pole, length = 9.81, 1.0, 0.1, 0.5
    total_mass = m_cart + m_pole
    polemass_length = m_pole * length
    x_pos, x_dot, th, th_dot = (x[..., i] for i in range(4))
    force = u[..., 0]
    th_u = th - math.pi
    costh, sinth = np.cos(th_u), np.sin(th_u)
    temp = (force + polemass_length * th_dot * th_dot * sinth) / total_mass
    denom = length * (4.0 / 3.0 - m_pole * costh * costh / total_mass)
    th_acc = (g * sinth - costh * temp) / denom
    x_acc = temp - polemass_length * th_acc * costh / total_mass
    return np.stack([x_pos + dt * x_dot, x_dot + dt * x_acc,
                     angle_normalize(th + dt * th_dot), th_dot + dt * th_acc], -1)


def _f_quadrotor(x, u, dt):  # systems.py:138-210
    m, g = 1.0, 9.81
    Ix, Iy, Iz = 0.02, 0.02, 0.04
    kv, kw = 0.05, 0.01
    with np.errstate(all="ignore"):
        bad = ~(np.isfinite(x).all(-1) & np.isfinite(u).all(-1))
        bad |= np.sqrt((x * x).sum(-1)) > 1e6
        phi, th, psi = x[..., 6], x[..., 7], x[..., 8]
        omg = x[..., 9:12]
        bad |= np.abs(np.cos(th)) < 1e-3
        bad |= (np.abs(omg) > 1e3).any(-1)
        s, c = np.sin, np.cos
        z, o = np.zeros_like(phi), np.ones_like(phi)
        Rz = np.stack([np.stack([c(psi), -s(psi), z], -1), np.stack([s(psi), c(psi), z], -1),
                       np.stack([z, z, o], -1)], -2)
        Ry = np.stack([np.stack([c(th), z, s(th)], -1), np.stack([z, o, z], -1),
                       np.stack([-s(th), z, c(th)], -1)], -2)
        Rx = np.stack([np.stack([o, z, z], -1), np.stack([z, c(phi), -s(phi)], -1),
                       np.stack([z, s(phi), c(phi)], -1)], -2)
        Rb = Rz @ Ry @ Rx
        thrust = u[..., 0]
        e3t = np.stack([z * thrust, z * thrust, o * thrust], -1)
        acc = (Rb @ e3t[..., None])[..., 0] / m - np.array([0.0, 0.0, g]) - kv * x[..., 3:6]
        t, sec = np.tan(th), 1.0 / np.cos(th)
        Tm = np.stack([np.stack([o, s(phi) * t, c(phi) * t], -1),
                       np.stack([z, c(phi), -s(phi)], -1),
                       np.stack([z, s(phi) * sec, c(phi) * sec], -1)], -2)
        eulerdot = (Tm @ omg[..., None])[..., 0]
        Iw = omg * np.array([Ix, Iy, Iz])
        omgdot = (u[..., 1:4] - np.cross(omg, Iw)) * np.array([1.0 / Ix, 1.0 / Iy, 1.0 / Iz]) \
            - kw * omg
        xdot = np.concatenate([x[..., 3:6], acc, eulerdot, omgdot], -1)
        xn = x + dt * xdot
    return np.where(bad[..., None], np.nan, xn)


def _f_pointmass(x, u, dt):  # systems.py:239-249
    return np.stack([x[..., 0] + dt * x[..., 2], x[..., 1] + dt * x[..., 3],
                     x[..., 2] + dt * u[..., 0], x[..., 3] + dt * u[..., 1]], -1)


_SEG = {}


def _segway_consts():  # systems.py:305-319
    if not _SEG:
        g, r, M, m, l = 9.81, 0.15, 1.0, 2.0, 0.5
        I = (1.0 / 3.0) * m * l * l  # noqa: E741
        a1, a2, a3 = M + m, m * l, I + m * l * l
        Den = a1 * a3 - a2 * a2
        _SEG.update(A_tau=a3 / (r * Den) - a2 / Den, A_th=-(a2 * m * g * l) / Den,
                    B_tau=-a2 / (r * Den) + a1 / Den, B_th=(a1 * m * g * l) / Den)
    return _SEG


def _f_segway(x, u, dt):  # systems.py:321-333
    c = _segway_consts()
    tau, th = u[..., 0], x[..., 2]
    xdd = c["A_tau"] * tau + c["A_th"] * th
    thdd = c["B_tau"] * tau + c["B_th"] * th
    return np.stack([x[..., 0] + dt * x[..., 1], x[..., 1] + dt * xdd,
                     angle_normalize(th + dt * x[..., 3]), x[..., 3] + dt * thdd], -1)


_F = {0: _f_di, 1: _f_cartpole, 2: _f_quadrotor, 3: _f_pointmass, 4: _f_segway}


def dynamics(sys_id, X, U, dt):
    """x' = F(x, u) over any leading batch shape."""
    X = np.asarray(X, dtype=np.float64)
    U = np.asarray(U, dtype=np.float64)
    return _F[sys_id](X, U, dt)


def _fd_step(v, eps, rel):
    # max(eps, rel * max(1.0, |v|)) with Python's max (a NaN |v| keeps 1.0)
    av = np.abs(v)
    inner = np.where(av > 1.0, av, 1.0)
    rh = rel * inner
    return np.where(rh > eps, rh, eps)


def linearize(sys_id, X, U, dt, central=False, epsx=1e-5, epsu=1e-5, relx=1e-6, relu=1e-6):
    """A [..., N, n, n], B [..., N, n, m], a_res [..., N, n] for X [..., N+1, n],
    U [..., N, m]: linearization.py:177-211 (central) / 216-262 (forward) and
    compute_affine_residuals 269-270, vectorised over steps and batch."""
    X = np.asarray(X, dtype=np.float64)
    U = np.asarray(U, dtype=np.float64)
    n, m = DIMS[sys_id]
    N = U.shape[-2]
    x, u = X[..., :N, :], U
    with np.errstate(all="ignore"):
        f0 = dynamics(sys_id, x, u, dt)
        A = np.zeros(x.shape[:-1] + (n, n))
        B = np.zeros(x.shape[:-1] + (n, m))
        for j in range(n + m):
            onx = j < n
            v = x[..., j] if onx else u[..., j - n]
            h = _fd_step(v, epsx, relx) if onx else _fd_step(v, epsu, relu)
            e = np.zeros(n if onx else m)
            e[j if onx else j - n] = 1.0
            if not central:
                # x + hi * I_n[i] (linearization.py:254, 258)
                xp = x + h[..., None] * e if onx else x
                up = u if onx else u + h[..., None] * e
                col = (dynamics(sys_id, xp, up, dt) - f0) / h[..., None]
            else:
                xp, xm, up, um = x.copy(), x.copy(), u.copy(), u.copy()
                if onx:
                    xp[..., j] += h
                    xm[..., j] -= h
                else:
                    up[..., j - n] += h
                    um[..., j - n] -= h
                col = (dynamics(sys_id, xp, up, dt) - dynamics(sys_id, xm, um, dt)) \
                    / (2.0 * h[..., None])
            if onx:
                A[..., :, j] = col
            else:
                B[..., :, j - n] = col
        if not central:
            bad = ~np.isfinite(f0).all(-1)
            A[bad] = np.nan
            B[bad] = np.nan
        a_res = f0 - X[..., 1:N + 1, :]
    return A, B, a_res


def _scalar_F(sys_id, dt):
    f = _F[sys_id]
    return lambda x, u: f(np.asarray(x, float), np.asarray(u, float), dt)


def linearize_loop(sys_id, X, U, dt, central=False, epsx=1e-5, epsu=1e-5, relx=1e-6, relu=1e-6):
    """The reference's loop structure for one trajectory: per step, per column,
    one F call at a time (linearization.py:238-262 / 190-211, 269-270)."""
    with np.errstate(all="ignore"):
        return _linearize_loop(_scalar_F(sys_id, dt), X, U, central, epsx, epsu, relx, relu)


def _linearize_loop(F, X, U, central, epsx, epsu, relx, relu):
    N, n, m = len(U), X.shape[1], U.shape[1]
    A_list, B_list = [], []
    I_n, I_m = np.eye(n), np.eye(m)
    for k in range(N):
        x, u = X[k], U[k]
        A, B = np.zeros((n, n)), np.zeros((n, m))
        if not central:
            f0 = F(x, u)
            if not np.all(np.isfinite(f0)):
                A[:] = np.nan
                B[:] = np.nan
            else:
                for i in range(n):
                    hi = max(float(epsx), float(relx) * max(1.0, abs(float(x[i]))))
                    A[:, i] = (F(x + hi * I_n[i], u) - f0) / hi
                for j in range(m):
                    hj = max(float(epsu), float(relu) * max(1.0, abs(float(u[j]))))
                    B[:, j] = (F(x, u + hj * I_m[j]) - f0) / hj
        else:
            for i in range(n):
                hi = max(epsx, relx * max(1.0, abs(float(x[i]))))
                xp, xm = x.copy(), x.copy()
                xp[i] += hi
                xm[i] -= hi
                A[:, i] = (F(xp, u) - F(xm, u)) / (2.0 * hi)
            for j in range(m):
                hj = max(epsu, relu * max(1.0, abs(float(u[j]))))
                up, um = u.copy(), u.copy()
                up[j] += hj
                um[j] -= hj
                B[:, j] = (F(x, up) - F(x, um)) / (2.0 * hj)
        A_list.append(A)
        B_list.append(B)
    a_res = [F(X[k], U[k]) - X[k + 1] for k in range(N)]
    return np.array(A_list), np.array(B_list), np.array(a_res)
