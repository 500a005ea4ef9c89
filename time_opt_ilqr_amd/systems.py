"""The reference's benchmark systems (systems.py) with their dynamics on the device.

Each ``make_*`` returns the reference's 13-tuple
``(F, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max, wrap_idx, extra)`` with the
same problem data (systems.py:28-349); ``F`` is a :class:`DeviceDynamics`, whose
evaluations run in libhop_amd.so (hop_dynamics_f64 / hop_linearize_f64,
csrc/dynamics.hpp).  ``F(x, u)`` keeps the reference's single-step call
signature; the batched forms are ``F.batch`` and the linearisation drop-ins in
:mod:`time_opt_ilqr_amd.linearization`.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

from . import engine


@dataclass(frozen=True)
class DeviceDynamics:
    """x_{k+1} = F(x_k, u_k) of system ``system_id`` with step ``dt``."""
    system_id: int
    dt: float
    n: int
    m: int
    name: str = ""

    def __call__(self, x, u):
        """One step for one (x, u) pair, NumPy in / NumPy out (reference call form)."""
        import torch
        dev = torch.device("cuda", torch.cuda.current_device())
        xt = torch.as_tensor(np.asarray(x, dtype=float).reshape(self.n), device=dev)
        ut = torch.as_tensor(np.asarray(u, dtype=float).reshape(self.m), device=dev)
        return engine.dynamics(self.system_id, xt, ut, self.dt).cpu().numpy()

    def batch(self, X, U):
        """x' for device tensors X [..., n], U [..., m]."""
        return engine.dynamics(self.system_id, X, U, self.dt)


def _F(sid, dt, name):
    n, m = {0: (2, 1), 1: (4, 1), 2: (12, 4), 3: (4, 2), 4: (4, 1)}[sid]
    return DeviceDynamics(sid, float(dt), n, m, name)


def make_double_integrator(dt: float = 0.05, N: int = 120):
    """systems.py:28-50: x = [pos, vel], u = [acc]."""
    F = _F(0, dt, "double_integrator")
    return (F, np.array([1.0, 0.0]), np.array([2.0, 0.0]), np.array([0.0]),
            np.diag([1.0, 0.1]), np.array([[1e-2]]), 50.0, 0.02, N, 10, 80, [], None)


def make_cartpole_swingup(dt: float = 0.02, N: int = 360):
    """systems.py:57-112: x = [cart_pos, cart_vel, theta (0 = down), theta_dot]."""
    F = _F(1, dt, "cartpole")
    return (F, np.zeros(4), np.array([0.0, 0.0, math.pi, 0.0]), np.array([0.0]),
            np.diag([0.01, 0.2, 0.0, 0.2]), np.array([[0.02]]), np.diag([5.0, 5.0, 800.0, 40.0]),
            0.03, N, 40, 320, [2], None)


def make_quadrotor(dt: float = 0.05, N: int = 160):
    """systems.py:119-230: x = [pos, vel, euler (phi, th, psi), omega], u = [thrust, tau];
    F returns all-NaN past its guards (non-finite input, ||x|| > 1e6,
    |cos(pitch)| < 1e-3, |omega| > 1e3)."""
    F = _F(2, dt, "quadrotor")
    x0 = np.zeros(12)
    x0[0:3] = 2.0
    return (F, x0, np.zeros(12), np.array([9.81, 0.0, 0.0, 0.0]),
            np.diag([5, 5, 5, 1, 1, 1, 20, 20, 10, 1, 1, 1]).astype(float),
            np.diag([1e-3, 1e-2, 1e-2, 1e-2]), 300.0, 0.005, N, 40, 160, [6, 7, 8], None)


OBSTACLES = ((np.array([-1.0, -0.5]), 0.65, 6.0), (np.array([0.0, 0.2]), 0.70, 6.0),
             (np.array([1.0, 1.0]), 0.65, 6.0))


def obstacle_stage_cost(x, u=None):
    """The point-mass maker's extra_stage_cost (systems.py:271-293): soft Gaussian
    obstacle penalties -> (c, cx [4], cxx [4, 4]) at one state."""
    p = np.asarray(x[:2], dtype=float)
    c, cx, cxx = 0.0, np.zeros(4), np.zeros((4, 4))
    for o, r, wt in OBSTACLES:
        d = p - o
        ci = wt * math.exp(-float(d @ d) / (2.0 * r * r))
        c += ci
        cx[:2] += -(ci / (r * r)) * d
        cxx[:2, :2] += ci * (np.outer(d, d) / (r ** 4) - np.eye(2) / (r * r))
    return c, cx, cxx


def make_pointmass_navigation(dt: float = 0.05, N: int = 240):
    """systems.py:237-296: 2-D double integrator with obstacle penalties (extra)."""
    F = _F(3, dt, "pointmass")
    extra = dict(obstacles=[dict(center=o, radius=r, weight=wt) for o, r, wt in OBSTACLES],
                 extra_stage_cost=obstacle_stage_cost)
    return (F, np.array([-2.0, -2.0, 0.0, 0.0]), np.array([2.0, 2.0, 0.0, 0.0]), np.zeros(2),
            np.diag([0.0, 0.0, 0.15, 0.15]), np.diag([0.05, 0.05]),
            np.diag([250.0, 250.0, 30.0, 30.0]), 0.06, N, 30, 220, [], extra)


def make_segway_balance(dt: float = 0.02, N: int = 240):
    """systems.py:303-349: linearised wheel-pendulum, x = [x, x_dot, th, th_dot]."""
    F = _F(4, dt, "segway")
    return (F, np.array([0.05, 0.0, 0.08, 0.0]), np.zeros(4), np.array([0.0]),
            np.diag([1.0, 0.1, 25.0, 1.0]), np.array([[0.25]]),
            np.diag([20.0, 2.0, 250.0, 10.0]), 1e-4, N, 40, 200, [2], None)


MAKERS = {"double_integrator": make_double_integrator, "cartpole": make_cartpole_swingup,
          "quadrotor": make_quadrotor, "pointmass": make_pointmass_navigation,
          "segway": make_segway_balance}
