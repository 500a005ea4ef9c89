"""The time-optimal iLQR outer loop on the device.

``ilqr_timeopt_batch`` runs ``ilqr_timeopt(method="propagator")``
(/root/reference/solver.py:449-765) for a batch of independent problems of one
system: every stage is a batched HIP launch of libhop_amd.so --
linearisation (hop_linearize_f64), the select block (hop_lft_sweep_traj_f64:
augmented builders + propagator + argmin), the truncated Riccati pass at T*
(hop_riccati_f64 mode 0), the forward line search (hop_forward_linesearch_f64)
and the accept / LM / stop-rule bookkeeping (hop_ilqr_accept_f64).  The host
only sequences launches; it reads one flag per iteration (all problems done)
to stop early.

The reference-shaped single-problem drop-ins (same names and arguments as
solver.py) are ``rollout``, ``cost_timeopt_true``, ``forward_linesearch_fixedT``
and ``ilqr_timeopt`` / ``ilqr_timeopt_ourmethod``.  F is a
:class:`time_opt_ilqr_amd.systems.DeviceDynamics` (the make_* makers of
:mod:`time_opt_ilqr_amd.systems` return one: everything on the device) or any
Python callable F(x, u) -> x_next, and ``extra_stage_cost`` None, the point-mass
obstacle cost of those makers, or any callable (x, u) -> (c, cx, cxx).  A callable
the device has no kernel for is evaluated on the host per problem (rollouts, FD
linearisation, line search: host_dynamics.py, the reference's own call form) while
the select, the Riccati pass and the accept / LM / stop step stay on the device.
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from types import SimpleNamespace
from typing import Any, Dict, List, Optional, Sequence

import numpy as np

from . import _lib, engine, host_dynamics
from .utils import _sym, as_terminal_weight, chol_inv

ALPHAS = engine.ALPHAS


def _torch():
    import torch
    return torch


@dataclass
class IlqrState:
    """Per-problem outer-loop state (device tensors)."""
    X: "object"        # [B, N+1, n]
    U: "object"        # [B, N, m]
    lm: "object"       # [B] f64
    T_bar: "object"    # [B] i32
    J_hist: "object"   # [B, H] f64
    T_hist: "object"   # [B, H] i32
    n_hist: "object"   # [B] i32
    done: "object"     # [B] i32 (stop rule met, or the select block raised)
    crashed: "object"  # [B] i32 (the reference would have raised in the select block)


def _obstacle_rows(extra_stage_cost):
    """The obstacle table of the point-mass extra_stage_cost, or None."""
    if extra_stage_cost is None:
        return None
    from . import systems
    if extra_stage_cost is systems.obstacle_stage_cost:
        return np.array([[o[0], o[1], r, wt] for o, r, wt in systems.OBSTACLES])
    obs = getattr(extra_stage_cost, "obstacles", None)
    if obs is not None:
        return np.asarray(obs, dtype=float).reshape(-1, 4)
    raise NotImplementedError("extra_stage_cost must be None or the point-mass obstacle cost "
                              "(systems.obstacle_stage_cost): arbitrary Python callables "
                              "cannot run on the device")


def ilqr_timeopt_batch(system, x0, xg, u_ref, Q, R, Qf, w, N: int, T_min: int, T_max: int, *,
                       dt: float = 0.0, U_init=None, max_iter: int = 15, lm_init: float = 1e-3,
                       wrap_idx: Optional[Sequence[int]] = None, use_central_diff: bool = True,
                       obstacles=None, alphas=ALPHAS, device=None,
                       stage_timers: bool = True, method: str = "propagator",
                       extra_stage_cost=None) -> Dict[str, Any]:
    """Batched ilqr_timeopt(method="propagator" | "bruteforce") (solver.py:449-765).

    The select step is the LFT sweep of the augmented system (propagator) or the
    brute-force J curve of T_max value-expansion sweeps (bruteforce, solver.py:293-358,
    one hop_bruteforce_jcurve launch); everything after it is shared.

    x0 [n] or [B, n] (torch or NumPy); U_init [B, N, m] or None (u_ref tiled);
    xg/u_ref/Q/R shared or per problem; Qf = as_terminal_weight(alpha) [n, n];
    w scalar.  Returns device tensors X, U, J_hist [B, H], T_hist, n_hist, T_star,
    crashed, plus per-stage wall times in ``timers`` (the reference's timers dict;
    each stage is synchronised for it -- stage_timers=False skips those syncs and
    leaves the host waiting only on the once-per-iteration "all done" flag).

    ``system`` is a device system (id, name or systems.DeviceDynamics, with ``dt``) or
    a host_dynamics.HostDynamics wrapping a Python callable F(x, u): then the rollouts,
    the FD linearisation and the line search evaluate F on the host per problem (the
    reference's own call form, host_dynamics.py) and the select, Riccati and accept
    steps stay on the device.  ``extra_stage_cost``: a Python callable (x, u) ->
    (c, cx, cxx) evaluated on the host the same way (host systems only; the device
    systems take the point-mass ``obstacles`` table).
    """
    torch = _torch()
    if method not in ("propagator", "bruteforce"):
        raise NotImplementedError(f"method={method!r}: the device outer loop implements "
                                  "'propagator' and 'bruteforce'")
    host = isinstance(system, host_dynamics.HostDynamics)
    if host:
        sid, n, m = None, int(system.n), int(system.m)
        if obstacles is not None and len(obstacles) > 0:
            raise ValueError("host dynamics: pass the stage cost as extra_stage_cost")
    else:
        if extra_stage_cost is not None:
            raise ValueError("device dynamics take the point-mass obstacles table; a "
                             "Python extra_stage_cost needs host dynamics")
        sid = engine.system_id(system)
        n, m = engine.system_dims(sid)
    dev = device or torch.device("cuda", torch.cuda.current_device())
    f64 = torch.float64
    tt = lambda a: torch.as_tensor(np.asarray(a, dtype=float) if not isinstance(  # noqa: E731
        a, torch.Tensor) else a, dtype=f64, device=dev).contiguous()
    N, T_min, T_max = int(N), int(T_min), int(T_max)
    if not 1 <= T_min <= T_max <= N:
        raise IndexError("need 1 <= T_min <= T_max <= N (the reference indexes lists of N)")
    x0 = tt(x0)
    Bn = x0.shape[0] if x0.dim() == 2 else 1
    xg_t, ur_t, Q_t, R_t, Qf_t = tt(xg), tt(np.atleast_1d(u_ref) if not isinstance(
        u_ref, torch.Tensor) else u_ref), tt(Q), tt(R), tt(Qf)
    R_np = R_t.cpu().numpy() if R_t.dim() == 2 else None
    if R_np is None:
        raise ValueError("R must be one [m, m] matrix shared by the batch")
    R_inv = tt(chol_inv(_sym(R_np)))
    if Qf_t.dim() != 2:
        raise ValueError("Qf must be one [n, n] terminal weight shared by the batch "
                         "(as_terminal_weight(alpha))")
    P = 0.5 * (Qf_t + Qf_t.transpose(-1, -2))  # _sym on the device
    obs = None if obstacles is None or len(obstacles) == 0 else tt(obstacles)
    # w as a device scalar made once (a Python float would cost a fill launch per call)
    w_t = torch.full((1,), float(w), dtype=f64, device=dev)
    w_f = float(w)
    bits = torch.tensor([1 << i for i in range(8)], dtype=torch.int32, device=dev)
    cost = engine.CostParams(xg_t, ur_t, Q_t, R_t, Qf_t, w_t, obs, wrap_idx)
    if U_init is None:
        U = ur_t.reshape(-1, m).expand(Bn, m)[:, None, :].expand(Bn, N, m).contiguous()
    else:
        U = tt(U_init)
        if U.dim() == 1:  # solver.py:484-485: a 1-D U_init is one control per step
            U = U.reshape(-1, 1)
        if U.dim() == 2:
            U = U[None]
        if U.dim() != 3 or U.shape[-1] != m or U.shape[0] not in (1, Bn):
            raise ValueError(f"U_init must be [N', {m}] or [B or 1, N', {m}]")
        U = U.expand(Bn, -1, -1)
        if U.shape[1] < N:  # pad with the last control, as the reference does
            U = torch.cat([U, U[:, -1:].expand(Bn, N - U.shape[1], m)], 1)
        U = U[:, :N].contiguous()
    # the reference's four timers (solver.py:497); its initial rollout is untimed and
    # is reported separately here.  Without stage_timers the stages are not
    # synchronised, so their times are unknown: NaN, not 0.
    nan = float("nan")
    timers = {k: (0.0 if stage_timers else nan)
              for k in ("linearize", "select", "backward", "forward")}
    t_rollout = 0.0 if stage_timers else nan

    def clock(key, t0):
        if stage_timers:
            torch.cuda.synchronize(dev)
            timers[key] += time.perf_counter() - t0

    if host:
        if not all(t.dim() == d for t, d in ((xg_t, 1), (ur_t, 1), (Q_t, 2), (Qf_t, 2))):
            raise ValueError("host dynamics: xg, u_ref, Q and Qf shared by the batch")
        # the host line search's cost arguments (solver.py:65-102 with Qf expanded)
        cost_np = (xg_t.cpu().numpy(), ur_t.cpu().numpy().reshape(-1), Q_t.cpu().numpy(),
                   R_np, Qf_t.cpu().numpy(), float(w), wrap_idx)
    t0 = time.perf_counter()
    if host:
        x0h = x0.reshape(-1, n).expand(Bn, n).cpu().numpy()
        Uh = U.cpu().numpy()
        X = tt(host_dynamics.rollout_batch(system, x0h, Uh))
    else:
        X = engine.rollout(sid, x0, U, dt)
    if stage_timers:
        torch.cuda.synchronize(dev)
        t_rollout = time.perf_counter() - t0
    H = int(max_iter) + 1
    st = IlqrState(X, U, torch.full((Bn,), float(lm_init), dtype=f64, device=dev),
                   torch.zeros((Bn,), dtype=torch.int32, device=dev),
                   torch.zeros((Bn, H), dtype=f64, device=dev),
                   torch.zeros((Bn, H), dtype=torch.int32, device=dev),
                   torch.zeros((Bn,), dtype=torch.int32, device=dev),
                   torch.zeros((Bn,), dtype=torch.int32, device=dev),
                   torch.zeros((Bn,), dtype=torch.int32, device=dev))
    bad = _lib.ST_FAIL | _lib.ST_NONFINITE
    # the last select's J curve of every problem (solver.py:751-762 returns it)
    J_curve = torch.full((Bn, T_max), float("nan"), dtype=f64, device=dev)
    # A problem whose initial trajectory is not finite on the rows the select block
    # reads (X[:T_max+1], U[:T_max]) raises in the reference's first select: its
    # augmented blocks are NaN and chol_inv's _assert_finite (utils.py:77) refuses
    # them.  Such problems are marked crashed here and never enter the batch, so
    # they cannot cost the select block's rerun launch (one reference-association
    # sweep of latency, 0.83 ms at N = 100, for a handful of problems).  The
    # line search only ever accepts finite rollouts, so later trajectories stay
    # finite and the check is needed once.
    pre_bad = ~(torch.isfinite(X[:, :T_max + 1]).flatten(1).all(1)
                & torch.isfinite(U[:, :T_max]).flatten(1).all(1))

    def iterate(s, warm):
        """one update (solver.py:541-553 when warm, else 578-752) of the problems in s"""
        t0 = time.perf_counter()
        if host:
            Xh, Uh = s.X.cpu().numpy(), s.U.cpu().numpy()
            A, Bm, a_res = host_dynamics.linearize_batch(system, Xh, Uh, central=use_central_diff)
            lin = SimpleNamespace(A=tt(A), B=tt(Bm), a_res=tt(a_res))
        else:
            lin = engine.linearize(sid, s.X, s.U, dt, central=use_central_diff)
        clock("linearize", t0)
        t0 = time.perf_counter()
        ex = {}
        if obs is not None:
            c, cx, cxx = engine.obstacle_cost(s.X[:, :N], obs)
            ex = dict(qxx_extra=cxx, qx_extra=cx, c_extra=c)
        elif host and extra_stage_cost is not None:
            parts = [host_dynamics.stage_cost_terms(extra_stage_cost, Xh[b], Uh[b])
                     for b in range(Xh.shape[0])]
            ex = dict(qxx_extra=tt(np.stack([q[2] for q in parts])),
                      qx_extra=tt(np.stack([q[1] for q in parts])),
                      c_extra=tt(np.stack([q[0] for q in parts])))
        if method == "propagator":
            sel = engine.propagate_traj(lin.A, lin.B, lin.a_res, s.X, s.U, xg_t, ur_t, Q_t,
                                        R_inv, P, w_t, wrap_idx=wrap_idx, n_use=T_max,
                                        t_min=T_min, t_max=T_max, **ex)
            T_star, sel_status, sel_J = sel.t_star, sel.status, sel.J
        else:  # solver.py:607-614: the J curve at lm_lambda = 1e-6, argmin over [T_min, T_max]
            sel_J, st_T = engine.bruteforce_jcurve(lin.A, lin.B, s.X, s.U, xg_t, ur_t, Q_t, R_t,
                                                   Qf_t, T_max, lm_lambda=1e-6, w_stage=w_f,
                                                   wrap_idx=wrap_idx, **ex)
            T_star, _ = engine.select_horizon(sel_J, T_min, T_max)
            # the reference raises at the first failing horizon: any horizon's
            # failure bits make the problem's select status
            sel_status = ((st_T.unsqueeze(-1) & bits) != 0).any(1).to(torch.int32).mul_(
                bits).sum(1, dtype=torch.int32)
        clock("select", t0)
        t0 = time.perf_counter()
        ric = engine.riccati(lin.A, lin.B, s.X, s.U, xg_t, ur_t, Q_t, R_t, Qf_t, T_star, s.lm,
                             mode=0, wrap_idx=wrap_idx, reg_max_tries=1,
                             **({} if not ex else dict(qxx_extra=ex["qxx_extra"],
                                                       qx_extra=ex["qx_extra"],
                                                       c_extra=ex["c_extra"])))
        clock("backward", t0)
        t0 = time.perf_counter()
        # the reference raises out of ilqr_timeopt at the select (FloatingPointError /
        # LinAlgError): such problems become crashed and done; the line search runs
        # the others whose Riccati pass succeeded (one launch for both masks)
        active = engine.ilqr_select_mask(s, sel_status, ric.status)
        if host:
            fw = _host_linesearch(system, Xh, Uh, T_star, ric.K, ric.k, active, cost_np,
                                  alphas, extra_stage_cost, tt)
        else:
            fw = engine.forward_linesearch(sid, s.X, s.U, T_star, ric.K, ric.k, cost, dt,
                                           alphas=alphas, active=active)
        engine.ilqr_accept(s, fw.J, fw.accepted, T_star, warm=warm)
        if warm:
            # solver.py:548-553: X, U <- the line search's output, T_bar from the select
            s.T_bar.copy_(T_star)
        s.X, s.U = fw.X, fw.U
        clock("forward", t0)
        return sel_status, sel_J

    # Problems that met the stop rule (or whose select raised) leave the batch: the
    # remaining ones run as a compact batch, so finished problems cost nothing (a
    # crashed problem would otherwise force the select block's rerun launch every
    # iteration).  The compact state persists across iterations and is gathered
    # again only when the live set shrinks (no per-iteration gather / scatter of
    # the nine per-problem fields).  Needs the cost blocks shared by the batch.
    compact = all(t.dim() == d for t, d in ((xg_t, 1), (ur_t, 1), (Q_t, 2), (Qf_t, 2)))
    fields = ("X", "U", "lm", "T_bar", "J_hist", "T_hist", "n_hist", "done", "crashed")
    pre = pre_bad.to(torch.int32)
    st.crashed |= pre
    st.done |= pre
    pre_status = torch.where(pre_bad, bad, 0).to(torch.int32)
    cur, idx = st, None  # idx: the rows of st that cur holds (None: cur is st)

    def sync_back():
        if idx is not None:
            for f in fields:
                getattr(st, f).index_copy_(0, idx, getattr(cur, f))

    def step(warm):
        """one iteration over the live problems; False when none is left"""
        nonlocal cur, idx
        live = cur.done == 0
        n_live = int(live.sum().item())
        if n_live == 0:
            return False
        base = pre_status if warm else torch.zeros_like(pre_status)
        if not compact:  # per-problem cost blocks: the whole batch, stopped rows masked
            stat, J_sel = iterate(st, warm)
            full = live if n_live < Bn else None
            if full is None:
                J_curve.copy_(J_sel)
                status_log.append(stat)
            else:
                J_curve[full] = J_sel[full]  # problems that had stopped ran no select
                status_log.append(torch.where(full, stat, base))
            return True
        if n_live < live.numel():  # the live set shrank: gather it again
            loc = live.nonzero()[:, 0]
            sync_back()
            cur = IlqrState(*[getattr(cur, f).index_select(0, loc) for f in fields])
            idx = loc if idx is None else idx.index_select(0, loc)
        stat, J_sel = iterate(cur, warm)
        if idx is None:
            J_curve.copy_(J_sel)
            status_log.append(stat)
        else:
            J_curve.index_copy_(0, idx, J_sel)
            status_log.append(base.index_copy(0, idx, stat))
        return True

    status_log = []
    if not step(True):
        status_log.append(pre_status)
    iters = 0
    for _ in range(int(max_iter)):
        if not step(False):
            break
        iters += 1
    sync_back()
    nh = st.n_hist
    last = (nh - 1).clamp(min=0).long()
    T_out = torch.where(nh > 0, st.T_hist.gather(1, last[:, None])[:, 0], st.T_bar)
    return dict(X=st.X, U=st.U, J_hist=st.J_hist, T_hist=st.T_hist, n_hist=nh, T_star=T_out,
                crashed=st.crashed, lm=st.lm, iterations=iters, timers=timers,
                t_rollout=t_rollout, J_curve=J_curve, select_status=torch.stack(status_log, 1))


def _host_linesearch(system, Xh, Uh, T_star, K, k, active, cost_np, alphas, extra, tt):
    """host_dynamics.linesearch_batch in the device line search's result form
    (accepted: the step-size index, -1 none, -2 inactive; inactive rows keep X, U)."""
    torch = _torch()
    Xo, Uo, J, J0, acc = host_dynamics.linesearch_batch(
        system, Xh, Uh, T_star.cpu().numpy(), K.cpu().numpy(), k.cpu().numpy(),
        active.cpu().numpy(), cost_np, alphas, extra)
    return engine.LineSearchResult(tt(Xo), tt(Uo), tt(J), tt(J0),
                                   torch.as_tensor(acc, device=T_star.device))


# ---------------------------------------------------------------------------
# reference-shaped single-problem drop-ins (solver.py names and arguments)
# ---------------------------------------------------------------------------

def _dyn(F):
    from .systems import DeviceDynamics
    if not isinstance(F, DeviceDynamics):
        raise TypeError("F must be a time_opt_ilqr_amd.systems.DeviceDynamics "
                        "(use the systems.make_* makers)")
    return F


def _on_device(F) -> bool:
    from .systems import DeviceDynamics
    if isinstance(F, DeviceDynamics):
        return True
    if not callable(F):
        raise TypeError("F must be a systems.DeviceDynamics or a callable F(x, u) -> x_next")
    return False


def _device_rows(F):
    """F's device kernel on stacked rows, NumPy in / out (x [K, n], u [K, m] -> [K, n]):
    the row-vectorised form host_dynamics uses for a built-in system whose stage cost is
    a Python callable (one launch per FD linearisation, rollout step or line-search step
    instead of one per F call)."""
    def rows(X, U):
        torch = _torch()
        dev = torch.device("cuda", torch.cuda.current_device())
        Xt = torch.as_tensor(np.ascontiguousarray(X, dtype=float), device=dev).reshape(-1, F.n)
        Ut = torch.as_tensor(np.ascontiguousarray(U, dtype=float), device=dev).reshape(-1, F.m)
        return F.batch(Xt, Ut).cpu().numpy()
    return rows


def _is_obstacle_cost(extra_stage_cost) -> bool:
    from . import systems
    return extra_stage_cost is None or extra_stage_cost is systems.obstacle_stage_cost or \
        getattr(extra_stage_cost, "obstacles", None) is not None


def _dev():
    from .horizon_selection import device
    return device()


def _t(a):
    torch = _torch()
    return torch.as_tensor(np.ascontiguousarray(np.asarray(a, dtype=float)), dtype=torch.float64,
                           device=_dev())


def _cost_params(X, xg, u_ref, Q, R, alpha, w, wrap_idx, extra_stage_cost):
    n = X.shape[1]
    obs = _obstacle_rows(extra_stage_cost)
    return engine.CostParams(_t(np.asarray(xg, dtype=float).reshape(-1)),
                             _t(np.atleast_1d(np.asarray(u_ref, dtype=float)).reshape(-1)),
                             _t(Q), _t(np.atleast_2d(R)), _t(as_terminal_weight(alpha, n)),
                             float(w), None if obs is None else _t(obs), wrap_idx)


def rollout(F, x0: np.ndarray, U: np.ndarray, *, max_state_norm: float = 1e6) -> np.ndarray:
    """solver.py:42-62 (GPU; a Python callable F: on the host, host_dynamics.rollout)."""
    U = np.asarray(U, dtype=float)
    if U.ndim == 1:
        U = U.reshape(-1, 1)
    if not _on_device(F):
        return host_dynamics.rollout(F, x0, U, max_state_norm=max_state_norm)
    F = _dyn(F)
    X = engine.rollout(F.system_id, _t(np.asarray(x0, dtype=float).reshape(-1)), _t(U)[None],
                       F.dt, max_state_norm=max_state_norm)
    return X[0].cpu().numpy()


def cost_timeopt_true(X, U, xg, u_ref, Q, R, alpha, w, T_star, wrap_idx=None,
                      extra_stage_cost=None, *, system=None) -> float:
    """solver.py:65-102 (GPU).  ``system`` (id, name or DeviceDynamics) selects the
    kernel instantiation; by default it is inferred from (n, m)."""
    X = np.asarray(X, dtype=float)
    U = np.asarray(U, dtype=float)
    if U.ndim == 1:
        U = U.reshape(-1, 1)
    T = int(T_star)
    if T <= 0:
        return float("inf")
    if T > len(U) or T + 1 > len(X):
        raise IndexError("index out of range")
    if not _is_obstacle_cost(extra_stage_cost):  # a Python stage cost: on the host
        return host_dynamics.cost_true(X, U, np.asarray(xg, dtype=float).reshape(-1),
                                       np.atleast_1d(np.asarray(u_ref, dtype=float)).reshape(-1),
                                       np.asarray(Q, dtype=float), np.atleast_2d(R),
                                       as_terminal_weight(alpha, X.shape[1]), w, T, wrap_idx,
                                       extra_stage_cost)
    sid = _system_for(system, X.shape[1], U.shape[1])
    cost = _cost_params(X, xg, u_ref, Q, R, alpha, w, wrap_idx, extra_stage_cost)
    # the reference reads only X[:T+1] and U[:T] (solver.py:80-102)
    J = engine.cost_true(sid, _t(X[:T + 1])[None], _t(U[:T])[None], [T], cost)
    return float(J[0].item())


def _system_for(system, n, m):
    if system is not None:
        return engine.system_id(getattr(system, "system_id", system))
    cands = [s for s in range(5) if engine.system_dims(s) == (n, m)]
    if not cands:
        raise ValueError(f"no device system with n={n}, m={m}")
    return cands[0]  # the cost does not depend on the dynamics


def forward_linesearch_fixedT(F, X, U, xg, u_ref, Q, R, alpha, w, T_star, k_list, K_list, *,
                              alphas=ALPHAS, wrap_idx=None, extra_stage_cost=None):
    """solver.py:233-286 (GPU; a Python callable F or stage cost: on the host,
    host_dynamics.linesearch) -> (X_new, U_new, J, accepted)."""
    X = np.asarray(X, dtype=float)
    U = np.asarray(U, dtype=float)
    if U.ndim == 1:
        U = U.reshape(-1, 1)
    N, n, m = len(U), X.shape[1], U.shape[1]
    T = int(T_star)
    if T > N or len(K_list) < T or len(k_list) < T:
        raise IndexError("list index out of range")
    K = np.zeros((N, m, n))
    k = np.zeros((N, m))
    for i in range(max(T, 0)):
        K[i] = np.asarray(K_list[i], dtype=float).reshape(m, n)
        k[i] = np.asarray(k_list[i], dtype=float).reshape(-1)
    if not _on_device(F) or not _is_obstacle_cost(extra_stage_cost):
        cost_np = (np.asarray(xg, dtype=float).reshape(-1),
                   np.atleast_1d(np.asarray(u_ref, dtype=float)).reshape(-1),
                   np.asarray(Q, dtype=float), np.atleast_2d(R), as_terminal_weight(alpha, n),
                   float(w), wrap_idx)
        Xn, Un, J, _, acc = host_dynamics.linesearch(F, X, U, T, K, k, cost_np, alphas,
                                                     extra_stage_cost)
        return Xn, Un, float(J), acc >= 0
    F = _dyn(F)
    cost = _cost_params(X, xg, u_ref, Q, R, alpha, w, wrap_idx, extra_stage_cost)
    r = engine.forward_linesearch(F.system_id, _t(X[:N + 1])[None], _t(U)[None], [T],
                                  _t(K)[None], _t(k)[None], cost, F.dt, alphas=alphas)
    acc = int(r.accepted[0].item()) >= 0
    if not acc:
        return X, U, float(r.J[0].item()), False
    return r.X[0].cpu().numpy(), r.U[0].cpu().numpy(), float(r.J[0].item()), True


def ilqr_timeopt(F, x0, xg, u_ref, Q, R, alpha, w, N: int, T_min: int, T_max: int, *,
                 U_init=None, method: str = "propagator", max_iter: int = 15,
                 lm_init: float = 1e-3, S_window: int = 20, wrap_idx: Optional[List[int]] = None,
                 use_central_diff: bool = True, extra_stage_cost=None,
                 onepass_preimage: str = "fixedpoint") -> Dict[str, Any]:
    """solver.py:449-765 for one problem, method="propagator" or "bruteforce" (GPU end
    to end).  S_window / onepass_preimage only matter for method="onepass" (not on
    the device)."""
    if method not in ("propagator", "bruteforce"):
        raise NotImplementedError("the device outer loop implements method='propagator' "
                                  "(the reference's 'ourmethod') and 'bruteforce' "
                                  "('baseline1')")
    x0 = np.asarray(x0, dtype=float).reshape(1, -1)
    n = x0.shape[1]
    if _on_device(F) and _is_obstacle_cost(extra_stage_cost):
        F = _dyn(F)
        system, kw = F.system_id, dict(dt=F.dt, obstacles=_obstacle_rows(extra_stage_cost))
    else:  # a Python callable (dynamics or stage cost): evaluated on the host per problem
        m = np.atleast_2d(np.asarray(R, dtype=float)).shape[0]
        if isinstance(F, host_dynamics.HostDynamics):
            system = F
        elif _on_device(F):  # a built-in system with a Python stage cost: F's rows in one launch
            system = host_dynamics.HostDynamics(_device_rows(F), n, m, name=F.name, vectorized=True)
        else:
            system = host_dynamics.HostDynamics(F, n, m)
        kw = dict(extra_stage_cost=extra_stage_cost)
    res = ilqr_timeopt_batch(system, x0, xg, u_ref,
                             np.asarray(Q, dtype=float), np.atleast_2d(np.asarray(R, dtype=float)),
                             as_terminal_weight(alpha, n), float(w), N, T_min, T_max,
                             U_init=U_init, max_iter=max_iter, lm_init=lm_init,
                             wrap_idx=wrap_idx, use_central_diff=use_central_diff,
                             device=_dev(), method=method, **kw)
    if int(res["crashed"][0].item()):
        raise np.linalg.LinAlgError(
            ("propagator_all_Jt_aug" if method == "propagator" else
             "bruteforce_all_Jt_backward_expansion") + " failed (non-finite or not PD)")
    nh = int(res["n_hist"][0].item())
    return {"X": res["X"][0].cpu().numpy(), "U": res["U"][0].cpu().numpy(),
            "J_hist": [float(v) for v in res["J_hist"][0, :nh].cpu().numpy()],
            "T_hist": [int(v) for v in res["T_hist"][0, :nh].cpu().numpy()],
            "timers": res["timers"], "J_curve": res["J_curve"][0].cpu().numpy(),
            "T_star": int(res["T_star"][0].item()),
            "onepass_error": None}


def ilqr_timeopt_ourmethod(*args, **kwargs):
    return ilqr_timeopt(*args, method="propagator", **kwargs)


def ilqr_timeopt_baseline1(*args, **kwargs):
    """solver.py:775-776"""
    return ilqr_timeopt(*args, method="bruteforce", **kwargs)
