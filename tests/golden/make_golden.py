"""Generate the committed golden vectors by running the REFERENCE itself.

Run in the build container only (the reference tree is not on the GPU box):

    cd /tmp && PYTHONDONTWRITEBYTECODE=1 python /root/repo/tests/golden/make_golden.py [FLAG]

FLAG selects one group: --r4, --r3, --r2, --legacy, --traj, --lin, --ilqr (propagator outer loop),
--ilqr-bf (ilqr_timeopt(method="bruteforce"), ilqr_bf_*.npz), --summary (the
plots/summary.csv comparison runs, summary_*.npz); none runs the base groups.

It imports the reference modules from /root/reference (read-only, no bytecode
written) and stores inputs/outputs as .npz data files next to this script.
Synthetic inputs come from oracle.hop_oracle.synth_* (seeded PCG64), so only
seeds, shapes and the reference outputs are stored for them; real-system
captures (DoubleIntegrator, Quadrotor) store inputs too.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.dont_write_bytecode = True
sys.path.insert(0, REPO)
sys.path.insert(0, REF)
os.environ.setdefault("MPLBACKEND", "Agg")

import utils as ref_utils  # noqa: E402
import horizon_selection as ref_hs  # noqa: E402
import solver as ref_solver  # noqa: E402
import systems as ref_systems  # noqa: E402
import augmented as ref_aug  # noqa: E402
import linearization as ref_lin  # noqa: E402

from oracle import hop_oracle as orc  # noqa: E402


def _lists(*arrs):
    return [list(a) for a in arrs]


def synthetic_lft(tag, s, m, N, base_seed, count, T_min, T_max, efg_steps=4):
    Js, Es, Fs, Gs = [], [], [], []
    for i in range(count):
        A, Bm, Q, R, R_inv, z0, QT = orc.synth_lft_problem(base_seed + i, s, m, N)
        captured = []
        real_chol_inv = ref_hs.chol_inv

        def spy(M, *a, **k):
            out = real_chol_inv(M, *a, **k)
            captured.append(out)
            return out

        ref_hs.chol_inv = spy
        try:
            J = ref_hs.propagator_all_Jt_aug(list(A), list(Bm), list(Q), [R] * N, z0,
                                             list(QT), T_use=N, R_inv_cached=R_inv)
        finally:
            ref_hs.chol_inv = real_chol_inv
        # the first N chol_inv calls are E_k = chol_inv(Q_aug[k]) (horizon_selection.py:58)
        E = np.array(captured[:efg_steps])
        F = np.array([E[k] @ A[k].T for k in range(efg_steps)])
        G = np.array([ref_utils._sym(A[k] @ E[k] @ A[k].T + Bm[k] @ R_inv @ Bm[k].T)
                      for k in range(efg_steps)])
        Js.append(J)
        Es.append(E)
        Fs.append(F)
        Gs.append(G)
    J = np.array(Js)
    Tstar = np.array([int(np.argmin(j[T_min - 1:T_max]) + T_min) for j in J])
    np.savez_compressed(os.path.join(HERE, f"lft_synth_{tag}.npz"), s=s, m=m, N=N,
                        base_seed=base_seed, count=count, T_min=T_min, T_max=T_max,
                        J=J, T_star=Tstar, E=np.array(Es), F=np.array(Fs), G=np.array(Gs))
    print(f"lft_synth_{tag}: J[0,:3]={J[0, :3]} T*={Tstar}")


def synthetic_lft_rlist(tag, s, m, N, seed):
    """R_inv_cached=None path: per-stage R_k inverted inside the propagator."""
    A, Bm, Q, R, R_inv, z0, QT = orc.synth_lft_problem(seed, s, m, N)
    rng = np.random.default_rng(seed + 777)
    Rl = np.array([np.diag(rng.uniform(0.5, 2.0, m)) for _ in range(N)])
    J = ref_hs.propagator_all_Jt_aug(list(A), list(Bm), list(Q), list(Rl), z0, list(QT),
                                     T_use=N, R_inv_cached=None)
    np.savez_compressed(os.path.join(HERE, f"lft_rlist_{tag}.npz"), s=s, m=m, N=N, seed=seed,
                        R_list=Rl, J=J)
    print(f"lft_rlist_{tag}: J[:3]={J[:3]}")


def real_capture(tag, maker_kwargs, maker, T_min=None, T_max=None, max_iter=12,
                 S_window=20, central=False):
    out = maker(**maker_kwargs)
    F, x0, xg, u_ref, Q, R, alpha, w, N, tmin, tmax, wrap_idx, extra = out
    T_min = tmin if T_min is None else T_min
    T_max = tmax if T_max is None else T_max
    prop_calls, bwd_calls = [], []
    real_prop = ref_solver.propagator_all_Jt_aug
    real_bwd = ref_solver.backward_pass_truncated

    def prop_spy(A_aug, B_aug, Q_aug, R_list, z0, QT, T_use=None, R_inv_cached=None):
        J = real_prop(A_aug, B_aug, Q_aug, R_list, z0, QT, T_use=T_use,
                      R_inv_cached=R_inv_cached)
        prop_calls.append(dict(A=np.array(A_aug[:T_use]), B=np.array(B_aug[:T_use]),
                               Q=np.array(Q_aug[:T_use]), QT=np.array(QT[:T_use]),
                               z0=np.array(z0), R_inv=np.array(R_inv_cached),
                               T_use=int(T_use), J=np.array(J)))
        return J

    def bwd_spy(A_list, B_list, X, U, xg_, u_ref_, Q_, R_, alpha_, T_star, **kw):
        res = real_bwd(A_list, B_list, X, U, xg_, u_ref_, Q_, R_, alpha_, T_star, **kw)
        bwd_calls.append(dict(A=np.array(A_list), B=np.array(B_list), X=np.array(X),
                              U=np.array(U), T_star=int(T_star),
                              lm=float(kw.get("lm_lambda", 1e-3)), ok=bool(res[2]),
                              k=None if res[0] is None else np.array(res[0]),
                              K=None if res[1] is None else np.array(res[1])))
        return res

    ref_solver.propagator_all_Jt_aug = prop_spy
    ref_solver.backward_pass_truncated = bwd_spy
    try:
        sol = ref_solver.ilqr_timeopt(F, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max,
                                      method="propagator", max_iter=max_iter,
                                      S_window=S_window, wrap_idx=wrap_idx,
                                      use_central_diff=central, extra_stage_cost=None)
    finally:
        ref_solver.propagator_all_Jt_aug = real_prop
        ref_solver.backward_pass_truncated = real_bwd
    first, last = prop_calls[0], prop_calls[-1]
    b_last = [c for c in bwd_calls if c["ok"]][-1]
    d = dict(N=N, T_min=T_min, T_max=T_max, alpha=alpha, w=w, Q=Q, R=R, xg=xg,
             u_ref=u_ref, wrap_idx=np.array(wrap_idx if wrap_idx else [], dtype=np.int64),
             T_star_final=sol["T_star"], J_hist=np.array(sol["J_hist"]),
             T_hist=np.array(sol["T_hist"]), n_prop_calls=len(prop_calls))
    for name, c in (("first", first), ("last", last)):
        for key in ("A", "B", "Q", "QT", "z0", "R_inv", "J"):
            d[f"p{name}_{key}"] = c[key]
        d[f"p{name}_T_use"] = c["T_use"]
    for key in ("A", "B", "X", "U", "k", "K"):
        d[f"bwd_{key}"] = b_last[key]
    d["bwd_T_star"] = b_last["T_star"]
    d["bwd_lm"] = b_last["lm"]
    # brute-force J curve on the last backward call's linearisation
    d["bf_J"] = np.array(ref_solver.bruteforce_all_Jt_backward_expansion(
        list(b_last["A"]), list(b_last["B"]), b_last["X"], b_last["U"], xg, u_ref, Q, R,
        alpha, w, min(T_max, len(b_last["U"])), wrap_idx=wrap_idx))
    np.savez_compressed(os.path.join(HERE, f"real_{tag}.npz"), **d)
    print(f"real_{tag}: T*={sol['T_star']} J*={sol['J_hist'][-1] if sol['J_hist'] else None} "
          f"prop calls={len(prop_calls)}")


def riccati_synth(tag, n, m, N, seeds, T_stars, lm):
    rows = []
    for seed, T in zip(seeds, T_stars):
        A, B, X, U, xg, u_ref, Q, R, alpha = orc.synth_riccati_problem(seed, n, m, N)
        k_list, K_list, ok = ref_solver.backward_pass_truncated(
            list(A), list(B), X, U, xg, u_ref, Q, R, alpha, T, lm_lambda=lm)
        Vxx, Vx, V0, K2, k2 = ref_hs.value_expansions_and_gains_prefix(
            list(A), list(B), X, U, xg, u_ref, Q, R, alpha, T, 0, lm_lambda=lm, w_stage=0.01)
        rows.append(dict(seed=seed, T=T, ok=ok, k=np.array(k_list), K=np.array(K_list),
                         Vxx=np.array(Vxx), Vx=np.array(Vx), V0=np.array(V0),
                         K2=np.array(K2), k2=np.array(k2)))
    d = dict(n=n, m=m, N=N, lm=lm, seeds=np.array(seeds), T_stars=np.array(T_stars),
             w_stage=0.01)
    for i, r in enumerate(rows):
        for key in ("k", "K", "Vxx", "Vx", "V0", "K2", "k2"):
            d[f"p{i}_{key}"] = r[key]
        d[f"p{i}_ok"] = r["ok"]
    np.savez_compressed(os.path.join(HERE, f"riccati_synth_{tag}.npz"), **d)
    print(f"riccati_synth_{tag}: ok={[r['ok'] for r in rows]} k0={rows[0]['k'][0]}")


def riccati_shift(tag, n, m, N, seed, T_bar, S_right, lm):
    """value_expansions_and_gains_prefix with a negative-time prefix (S_right > 0)."""
    A, B, X, U, xg, u_ref, Q, R, alpha = orc.synth_riccati_problem(seed, n, m, N)
    Vxx, Vx, V0, K, k = ref_hs.value_expansions_and_gains_prefix(
        list(A), list(B), X, U, xg, u_ref, Q, R, alpha, T_bar, S_right, lm_lambda=lm,
        w_stage=0.02, wrap_idx=[1])
    np.savez_compressed(os.path.join(HERE, f"riccati_shift_{tag}.npz"), n=n, m=m, N=N,
                        seed=seed, T_bar=T_bar, S_right=S_right, lm=lm, w_stage=0.02,
                        wrap_idx=np.array([1]), Vxx=np.array(Vxx), Vx=np.array(Vx),
                        V0=np.array(V0), K=np.array(K), k=np.array(k))
    print(f"riccati_shift_{tag}: V0[0]={V0[0]}")


def riccati_fail(tag, n, m, N, seed):
    """Indefinite R -> backward_pass_truncated returns (None, None, False)."""
    A, B, X, U, xg, u_ref, Q, R, alpha = orc.synth_riccati_problem(seed, n, m, N)
    Rneg = -50.0 * np.eye(m)
    res = ref_solver.backward_pass_truncated(list(A), list(B), X, U, xg, u_ref, Q, Rneg,
                                             alpha, N, lm_lambda=1e-3)
    np.savez_compressed(os.path.join(HERE, f"riccati_fail_{tag}.npz"), n=n, m=m, N=N,
                        seed=seed, R=Rneg, ok=res[2])
    print(f"riccati_fail_{tag}: ok={res[2]}")


def bruteforce_synth(tag, n, m, N, seed, T_max, w):
    A, B, X, U, xg, u_ref, Q, R, alpha = orc.synth_riccati_problem(seed, n, m, N)
    J = ref_solver.bruteforce_all_Jt_backward_expansion(list(A), list(B), X, U, xg, u_ref,
                                                         Q, R, alpha, w, T_max)
    np.savez_compressed(os.path.join(HERE, f"bruteforce_{tag}.npz"), n=n, m=m, N=N,
                        seed=seed, T_max=T_max, w=w, J=np.array(J))
    print(f"bruteforce_{tag}: J[:3]={np.array(J)[:3]}")


def chol_inv_cases():
    """Escalation / fallback / failure behaviour of utils.chol_inv (a2)."""
    cases = {
        "spd": np.array([[4.0, 1.0], [1.0, 3.0]]),
        "psd_singular": np.array([[1.0, 1.0], [1.0, 1.0]]),
        "indef_small": np.array([[1.0, 0.0], [0.0, -1e-8]]),   # needs escalation
        "indef_big": np.array([[1.0, 0.0], [0.0, -5.0]]),      # LU fallback
        "asym": np.array([[2.0, 0.5], [0.1, 1.0]]),            # _sym first
    }
    d = {}
    for name, M in cases.items():
        d[f"{name}_in"] = M
        d[f"{name}_out"] = ref_utils.chol_inv(M)
    np.savez_compressed(os.path.join(HERE, "chol_inv_cases.npz"), **d)
    print("chol_inv_cases:", list(cases))


def _lookup_dynamics(X, U, a_raw):
    """F with F(X[k], U[k]) = X[k+1] + a_raw[k] (the reference only evaluates F
    on the trajectory inside compute_affine_residuals)."""
    table = {X[k].tobytes() + U[k].tobytes(): X[k + 1] + a_raw[k] for k in range(len(U))}
    return lambda x, u: table[np.asarray(x, dtype=float).tobytes()
                              + np.asarray(u, dtype=float).tobytes()]


def traj_synth(tag, n, m, N, seeds, rho_regs, blocks_steps=3):
    """Reference builders (augmented.py:10-87) + propagator on trajectory-form inputs."""
    d = dict(n=n, m=m, N=N, seeds=np.array(seeds), rho_regs=np.array(rho_regs))
    Js, a_res, R_inv = [], [], []
    for sd, rho in zip(seeds, rho_regs):
        p = orc.synth_traj_problem(sd, n, m, N)
        F = _lookup_dynamics(p["X"], p["U"], p["a_raw"])
        a_list = ref_lin.compute_affine_residuals(F, p["X"], p["U"])
        Aa, Ba, Qa, R_list, z0, Ri = ref_aug.build_augmented_sequence_QR(
            F, list(p["A"]), list(p["B"]), p["X"], p["U"], p["xg"], p["u_ref"], p["Q"], p["R"],
            p["w"], wrap_idx=p["wrap_idx"], rho_reg=rho)
        QT = ref_aug.build_terminal_aug_list(p["X"], p["xg"], p["alpha"], wrap_idx=p["wrap_idx"],
                                             rho_reg=rho)
        J = ref_hs.propagator_all_Jt_aug(Aa, Ba, Qa, R_list, z0, QT, T_use=N, R_inv_cached=Ri)
        Js.append(np.array(J))
        a_res.append(np.array([a.ravel() for a in a_list]))
        R_inv.append(np.array(Ri))
        if len(Js) == 1:
            for key, v in (("A_aug", Aa), ("B_aug", Ba), ("Q_aug", Qa), ("QT_aug", QT)):
                d[key] = np.array(v[:blocks_steps])
    d.update(J=np.array(Js), a_res=np.array(a_res), R_inv=np.array(R_inv))
    np.savez_compressed(os.path.join(HERE, f"traj_synth_{tag}.npz"), **d)
    print(f"traj_synth_{tag}: J[0][:3]={Js[0][:3]}")


def traj_real(tag, maker_kwargs, maker, T_min=None, T_max=None, S_window=20):
    """Raw inputs of the first build_augmented_sequence_QR call of ilqr_timeopt
    (solver.py:514-522) on a real system, with the J curve that call produced."""
    out = maker(**maker_kwargs)
    F, x0, xg, u_ref, Q, R, alpha, w, N, tmin, tmax, wrap_idx, extra = out
    T_min = tmin if T_min is None else T_min
    T_max = tmax if T_max is None else T_max
    builds, props = [], []
    real_build = ref_solver.build_augmented_sequence_QR
    real_prop = ref_solver.propagator_all_Jt_aug

    def build_spy(F_, A_list, B_list, X, U, *a, **k):
        builds.append(dict(A=np.array(A_list), B=np.array(B_list), X=np.array(X),
                           U=np.array(U),
                           a_res=np.array([r.ravel() for r in
                                           ref_lin.compute_affine_residuals(F_, X, U)])))
        return real_build(F_, A_list, B_list, X, U, *a, **k)

    def prop_spy(*a, **k):
        J = real_prop(*a, **k)
        props.append(np.array(J))
        return J

    ref_solver.build_augmented_sequence_QR = build_spy
    ref_solver.propagator_all_Jt_aug = prop_spy
    try:
        ref_solver.ilqr_timeopt(F, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max,
                                method="propagator", max_iter=1, S_window=S_window,
                                wrap_idx=wrap_idx, use_central_diff=False,
                                extra_stage_cost=None)
    finally:
        ref_solver.build_augmented_sequence_QR = real_build
        ref_solver.propagator_all_Jt_aug = real_prop
    b = builds[0]
    d = dict(N=N, T_min=T_min, T_max=T_max, alpha=alpha, w=w, Q=Q, R=R, xg=xg, u_ref=u_ref,
             wrap_idx=np.array(wrap_idx if wrap_idx else [], dtype=np.int64),
             P=np.array(ref_utils._sym(ref_utils.as_terminal_weight(alpha, len(xg)))),
             R_inv=np.array(ref_utils.chol_inv(ref_utils._sym(R))), J=props[0], **b)
    np.savez_compressed(os.path.join(HERE, f"traj_real_{tag}.npz"), **d)
    print(f"traj_real_{tag}: N={N} T*={int(np.argmin(props[0][T_min - 1:T_max]) + T_min)}")


LIN_SYSTEMS = {  # system id of hop_linearize_f64 -> reference maker (systems.py)
    "di": (0, "make_double_integrator"),
    "cartpole": (1, "make_cartpole_swingup"),
    "quadrotor": (2, "make_quadrotor"),
    "pointmass": (3, "make_pointmass_navigation"),
    "segway": (4, "make_segway_balance"),
}


def lin_golden(name, N, seed, scale):
    """Dynamics F and both finite-difference linearisations of the reference
    (linearization.py:177-270) plus compute_affine_residuals on a seeded random
    trajectory around the system's x0 / u_ref.  The quadrotor capture also holds
    states that trip each NaN guard of its F (systems.py:170-195)."""
    _, maker = LIN_SYSTEMS[name]
    F, x0, xg, u_ref, *_ = getattr(ref_systems, maker)()
    rng = np.random.default_rng(seed)
    n, m = len(x0), len(u_ref)
    X = x0 + scale * rng.standard_normal((N + 1, n))
    U = u_ref + scale * rng.standard_normal((N, m))
    if name == "quadrotor":
        X[3, 7] = np.pi / 2 - 5e-4      # |cos(pitch)| < 1e-3
        X[5, 10] = 2e3                  # |omega| > 1e3
        X[7, 0] = 2e6                   # ||x|| > 1e6
        X[9, 2] = np.nan                # non-finite state
        U[11, 1] = np.inf               # non-finite control
    Fx = np.array([F(X[k], U[k]) for k in range(N)])
    Af, Bf = ref_lin.linearize_forward_diff_traj(F, X, U)
    Ac, Bc = ref_lin.linearize_central_diff_traj(F, X, U)
    a_res = np.array([r.ravel() for r in ref_lin.compute_affine_residuals(F, X, U)])
    np.savez_compressed(os.path.join(HERE, f"lin_{name}.npz"), X=X, U=U, dt=float(F.dt),
                        Fx=Fx, A_fwd=np.array(Af), B_fwd=np.array(Bf), A_cen=np.array(Ac),
                        B_cen=np.array(Bc), a_res=a_res)
    print(f"lin_{name}: n={n} m={m} N={N}")


def main_lin():
    np.seterr(all="ignore")
    lin_golden("di", 20, 9000, 0.5)
    lin_golden("cartpole", 20, 9001, 1.5)
    lin_golden("quadrotor", 24, 9002, 0.4)
    lin_golden("pointmass", 20, 9003, 0.7)
    lin_golden("segway", 20, 9004, 0.8)


def main_traj():
    np.seterr(all="ignore")
    traj_synth("n12_m4_N100", 12, 4, 100, [8000, 8001, 8002, 8003], [1.0, 1.0, 1e-12, 1e-12])
    traj_synth("n4_m1_N60", 4, 1, 60, [8100, 8101], [1.0, 1e-12])
    traj_real("DI_N50", dict(N=50), ref_systems.make_double_integrator, T_min=10, T_max=50)
    traj_real("Quad_N160", {}, ref_systems.make_quadrotor)


ILQR_CASES = [  # (tag, maker, maker kwargs, T_min, T_max, max_iter, central)
    ("di", "make_double_integrator", dict(N=50), 10, 50, 12, False),
    ("cartpole", "make_cartpole_swingup", dict(N=120), 20, 110, 4, False),
    ("quadrotor", "make_quadrotor", dict(N=100), 30, 90, 3, False),
    ("pointmass", "make_pointmass_navigation", dict(N=120), 30, 110, 4, True),
    ("segway", "make_segway_balance", dict(N=120), 20, 110, 4, False),
]


def ilqr_capture(tag, maker, maker_kwargs, T_min, T_max, max_iter, central, keep=3):
    """ilqr_timeopt(method="propagator") end to end (solver.py:449-765), with
    the first `keep` forward_linesearch_fixedT calls (solver.py:233-286) captured
    (inputs X, U, T*, k, K and outputs X', U', J, accepted), plus rollout
    (solver.py:42-62) and cost_timeopt_true (solver.py:65-102) on the final
    trajectory.  extra_stage_cost (point mass obstacles) is passed through."""
    F, x0, xg, u_ref, Q, R, alpha, w, N, _, _, wrap_idx, extra = \
        getattr(ref_systems, maker)(**maker_kwargs)
    esc = extra["extra_stage_cost"] if extra else None
    calls = []
    real_fwd = ref_solver.forward_linesearch_fixedT

    def fwd_spy(F_, X, U, xg_, u_ref_, Q_, R_, alpha_, w_, T_star, k_list, K_list, **kw):
        out = real_fwd(F_, X, U, xg_, u_ref_, Q_, R_, alpha_, w_, T_star, k_list, K_list, **kw)
        if len(calls) < keep:
            calls.append(dict(X=np.array(X), U=np.array(U), T_star=int(T_star),
                              k=np.array(k_list).reshape(len(k_list), -1),
                              K=np.array(K_list), X_new=np.array(out[0]),
                              U_new=np.array(out[1]), J=float(out[2]), acc=bool(out[3])))
        return out

    ref_solver.forward_linesearch_fixedT = fwd_spy
    try:
        sol = ref_solver.ilqr_timeopt(F, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max,
                                      method="propagator", max_iter=max_iter,
                                      wrap_idx=wrap_idx, use_central_diff=central,
                                      extra_stage_cost=esc)
    finally:
        ref_solver.forward_linesearch_fixedT = real_fwd
    U0 = np.tile(np.asarray(u_ref, dtype=float).reshape(1, -1), (N, 1))
    d = dict(N=N, T_min=T_min, T_max=T_max, max_iter=max_iter, central=int(central),
             dt=float(F.dt), x0=x0, xg=xg, u_ref=u_ref, Q=Q, R=R,
             Qf=ref_utils.as_terminal_weight(alpha, len(x0)), w=w,
             wrap_idx=np.array(wrap_idx if wrap_idx else [], dtype=np.int64),
             X0=ref_solver.rollout(F, x0, U0), X=sol["X"], U=sol["U"],
             J_hist=np.array(sol["J_hist"]), T_hist=np.array(sol["T_hist"]),
             T_star=int(sol["T_star"]), n_fwd=len(calls), J_curve=np.array(sol["J_curve"]))
    for i, c in enumerate(calls):
        for key, v in c.items():
            d[f"f{i}_{key}"] = v
    # cost_timeopt_true on the final trajectory at a few horizons
    Ts = np.array([1, T_min, int(sol["T_star"]), T_max])
    d["cost_T"] = Ts
    d["cost_J"] = np.array([ref_solver.cost_timeopt_true(sol["X"], sol["U"], xg, u_ref, Q, R,
                                                         alpha, w, int(T), wrap_idx, esc)
                            for T in Ts])
    # rollout with a blow-up: controls scaled until the state norm guard trips
    Ubig = sol["U"] * 1e4
    d["U_big"] = Ubig
    d["X_big"] = ref_solver.rollout(F, x0, Ubig, max_state_norm=1e3)
    np.savez_compressed(os.path.join(HERE, f"ilqr_{tag}.npz"), **d)
    print(f"ilqr_{tag}: T*={sol['T_star']} J_hist={sol['J_hist']} T_hist={sol['T_hist']} "
          f"fwd captured={len(calls)}")


ILQR_BF_CASES = [  # (tag, maker, maker kwargs, T_min, T_max, max_iter, central)
    ("di", "make_double_integrator", dict(N=50), 10, 50, 8, False),
    ("cartpole", "make_cartpole_swingup", dict(N=80), 20, 70, 3, False),
    ("segway", "make_segway_balance", dict(N=60), 10, 60, 3, False),
    ("quadrotor", "make_quadrotor", dict(N=60), 20, 55, 3, False),
    ("pointmass", "make_pointmass_navigation", dict(N=60), 20, 55, 3, True),
]


def ilqr_bruteforce_capture(tag, maker, maker_kwargs, T_min, T_max, max_iter, central):
    """ilqr_timeopt(method="bruteforce") end to end (solver.py:449-765 with the
    brute-force J curve of solver.py:293-358 as the select step)."""
    F, x0, xg, u_ref, Q, R, alpha, w, N, _, _, wrap_idx, extra = \
        getattr(ref_systems, maker)(**maker_kwargs)
    esc = extra["extra_stage_cost"] if extra else None
    sol = ref_solver.ilqr_timeopt(F, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max,
                                  method="bruteforce", max_iter=max_iter, wrap_idx=wrap_idx,
                                  use_central_diff=central, extra_stage_cost=esc)
    d = dict(N=N, T_min=T_min, T_max=T_max, max_iter=max_iter, central=int(central),
             dt=float(F.dt), x0=x0, xg=xg, u_ref=u_ref, Q=Q, R=R,
             Qf=ref_utils.as_terminal_weight(alpha, len(x0)), w=w,
             wrap_idx=np.array(wrap_idx if wrap_idx else [], dtype=np.int64),
             X=sol["X"], U=sol["U"], J_hist=np.array(sol["J_hist"]),
             T_hist=np.array(sol["T_hist"]), T_star=int(sol["T_star"]),
             J_curve=np.array(sol["J_curve"]))
    np.savez_compressed(os.path.join(HERE, f"ilqr_bf_{tag}.npz"), **d)
    print(f"ilqr_bf_{tag}: T*={sol['T_star']} J_hist={sol['J_hist']} T_hist={sol['T_hist']}")


def main_ilqr_bruteforce():
    np.seterr(all="ignore")
    for case in ILQR_BF_CASES:
        ilqr_bruteforce_capture(*case)


# plots/summary.csv (the reference's committed output of its published comparison):
# T*, J* of the DoubleIntegrator and Quadrotor_Hover rows, per method
SUMMARY_ROWS = {"di": "DoubleIntegrator", "quadrotor": "Quadrotor_Hover"}


def summary_capture(tag, maker, method):
    """ilqr_timeopt with the published comparison's settings (max_iter=20, lm_init=1e-3,
    central differences, each maker's default N / T_min / T_max; the legacy driver,
    ilqr_propagator.py:759-790, that wrote plots/summary.csv) through the current
    solver (solver.py:449-765), which reproduces the csv's T* and J* for these two
    cases.  The csv row's values ride along as data."""
    import csv
    import time
    F, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max, wrap_idx, extra = \
        getattr(ref_systems, maker)()
    T_max = min(T_max, N)
    t0 = time.perf_counter()
    sol = ref_solver.ilqr_timeopt(F, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max,
                                  method=method, max_iter=20, lm_init=1e-3,
                                  wrap_idx=wrap_idx, use_central_diff=True)
    wall = time.perf_counter() - t0
    row = None
    with open(os.path.join(REF, "plots", "summary.csv")) as f:
        for r in csv.DictReader(f):
            if r["case"] == SUMMARY_ROWS[tag] and r["method"] == method:
                row = r
    d = dict(N=N, T_min=T_min, T_max=T_max, max_iter=20, central=1, dt=float(F.dt), x0=x0,
             xg=xg, u_ref=u_ref, Q=Q, R=R, Qf=ref_utils.as_terminal_weight(alpha, len(x0)), w=w,
             wrap_idx=np.array(wrap_idx if wrap_idx else [], dtype=np.int64),
             X=sol["X"], U=sol["U"], J_hist=np.array(sol["J_hist"]),
             T_hist=np.array(sol["T_hist"]), T_star=int(sol["T_star"]),
             J_curve=np.array(sol["J_curve"]),
             ref_here_timers=np.array([sol["timers"][k] for k in
                                       ("linearize", "select", "backward", "forward")]),
             ref_here_wall=wall,
             csv_T_star=int(row["T_star"]), csv_J_star=float(row["J_star"]),
             csv_timers=np.array([float(row[k]) for k in
                                  ("t_linearize", "t_select", "t_backward", "t_forward")]),
             csv_n_iterations=int(row["n_iterations"]))
    np.savez_compressed(os.path.join(HERE, f"summary_{tag}_{method}.npz"), **d)
    print(f"summary_{tag}_{method}: T*={sol['T_star']} J*={sol['J_hist'][-1]!r} "
          f"(csv {row['T_star']}, {row['J_star']}) timers={sol['timers']}")


def main_summary():
    np.seterr(all="ignore")
    for tag, maker in (("di", "make_double_integrator"), ("quadrotor", "make_quadrotor")):
        for method in ("propagator", "bruteforce"):
            summary_capture(tag, maker, method)


def main_ilqr():
    np.seterr(all="ignore")
    for case in ILQR_CASES:
        ilqr_capture(*case)


# round 6: eight problems (was two), horizons from 1 to N, so the per-step gain
# checks of tests/test_gpu_parity.py see short, mid and full horizons
RICCATI_SYNTH = ("n12_m4_N100", 12, 4, 100, [7000, 7001, 7002, 7003, 7004, 7005, 7006, 7007],
                 [100, 57, 1, 13, 34, 77, 99, 64], 1e-3)


def main():
    np.seterr(all="ignore")
    synthetic_lft("s13_m4_N100", 13, 4, 100, 1000, 4, 40, 100)
    synthetic_lft("s5_m1_N200", 5, 1, 200, 2000, 4, 20, 200)
    synthetic_lft("s3_m1_N50", 3, 1, 50, 3000, 4, 10, 50)
    synthetic_lft("s13_m4_N128", 13, 4, 128, 4000, 2, 40, 128)
    synthetic_lft("s16_m6_N40", 16, 6, 40, 5000, 2, 5, 40)
    synthetic_lft_rlist("s7_m3_N30", 7, 3, 30, 6000)
    real_capture("DI_N50", dict(N=50), ref_systems.make_double_integrator, T_min=10, T_max=50)
    real_capture("Quad_N160", {}, ref_systems.make_quadrotor, max_iter=3)
    riccati_synth(*RICCATI_SYNTH)
    riccati_shift("n6_m2_N60", 6, 2, 60, 7100, 45, 15, 1e-6)
    riccati_fail("n4_m2_N20", 4, 2, 20, 7200)
    bruteforce_synth("n4_m2_N40", 4, 2, 40, 7300, 40, 0.05)
    chol_inv_cases()


# ---------------------------------------------------------------------------
# round 2: wider synthetic goldens, config 5, the legacy twin + plots/, LU slot
# ---------------------------------------------------------------------------

def synthetic_lft_wide(tag, s, m, N, base_seed, count, T_min, T_max):
    """J(t) and T* of `count` synthetic problems (no E/F/G): the default-path goldens."""
    J = np.array([ref_hs.propagator_all_Jt_aug(*_prop_args(orc.synth_lft_problem(base_seed + i,
                                                                                 s, m, N), N))
                  for i in range(count)])
    Tstar = np.array([int(np.argmin(j[T_min - 1:T_max]) + T_min) for j in J])
    np.savez_compressed(os.path.join(HERE, f"lft_wide_{tag}.npz"), s=s, m=m, N=N,
                        base_seed=base_seed, count=count, T_min=T_min, T_max=T_max,
                        J=J, T_star=Tstar)
    print(f"lft_wide_{tag}: {count} problems, T*={Tstar}")


def _prop_args(prob, N):
    A, Bm, Q, R, R_inv, z0, QT = prob
    return (list(A), list(Bm), list(Q), [R] * N, z0, list(QT))


def _prop(prob, N, **kw):
    A, Bm, Q, R, R_inv, z0, QT = prob
    return ref_hs.propagator_all_Jt_aug(list(A), list(Bm), list(Q), [R] * N, z0, list(QT),
                                        T_use=N, R_inv_cached=R_inv, **kw)


def config5_golden(N=128, base_seed=9000, count=12, T_min=40, T_max=128):
    """Mixed Segway / Cartpole / Quadrotor shapes (i mod 3) at their TRUE sizes."""
    J = np.array([_prop(orc.synth_config5_problem(base_seed, i, N), N) for i in range(count)])
    Tstar = np.array([int(np.argmin(j[T_min - 1:T_max]) + T_min) for j in J])
    np.savez_compressed(os.path.join(HERE, "config5_mixed_N128.npz"), N=N, base_seed=base_seed,
                        count=count, T_min=T_min, T_max=T_max, J=J, T_star=Tstar)
    print(f"config5_mixed_N128: T*={Tstar}")


def lu_slot_cases(seed=9500):
    """chol_inv's LU fallback (utils.py:88-93, np.linalg.solve = gesv with partial
    pivoting) on NON-diagonal indefinite blocks, alone and inside a propagator
    sweep: Q_k of problem 0 at step 3 and QT of problem 1 at step 5 are replaced by
    symmetric indefinite matrices whose eigenvalues lie in [-3, -0.5] u [0.5, 3]
    (Cholesky fails for every jitter up to 1e-2)."""
    rng = np.random.default_rng(seed)
    d = {}

    def indef(s):
        Qm, _ = np.linalg.qr(rng.standard_normal((s, s)))
        ev = rng.uniform(0.5, 3.0, s) * np.where(np.arange(s) % 2 == 0, 1.0, -1.0)
        return Qm @ np.diag(ev) @ Qm.T

    for s in (3, 5, 13):
        M = indef(s)
        d[f"inv_s{s}_in"] = M
        d[f"inv_s{s}_out"] = ref_utils.chol_inv(M)
    for tag, s, m, N in (("s13_m4_N20", 13, 4, 20), ("s5_m1_N20", 5, 1, 20)):
        probs = [list(orc.synth_lft_problem(seed + 10 + i, s, m, N)) for i in range(3)]
        probs[0][2] = probs[0][2].copy()
        probs[0][2][3] = indef(s)
        probs[1][6] = probs[1][6].copy()
        probs[1][6][5] = indef(s)
        d[f"lft_{tag}_Q03"] = probs[0][2][3]
        d[f"lft_{tag}_QT15"] = probs[1][6][5]
        d[f"lft_{tag}_J"] = np.array([_prop(tuple(p), N) for p in probs])
        d[f"lft_{tag}_base_seed"] = seed + 10
    np.savez_compressed(os.path.join(HERE, "lu_slot_cases.npz"), **d)
    print("lu_slot_cases:", sorted(d))


LEGACY_CASES = ("DoubleIntegrator", "Segway_Balance", "Ballbot_Balance", "Quadrotor_Hover")


def legacy_plots(case):
    """The legacy twin (ilqr_propagator.py) exactly as its main() runs it
    (ilqr_propagator.py:759-781): capture the FINAL brute-force curve call of the
    'bruteforce' run (ilqr_propagator.py:636, the J_bruteforce column of
    plots/<case>_Jt.csv) and the final propagator call of the 'propagator' run
    (ilqr_propagator.py:641, J_propagator), inputs and outputs, next to the CSV
    columns the reference committed."""
    import csv
    import ilqr_propagator as leg
    makers = {"DoubleIntegrator": leg.make_double_integrator, "Segway_Balance": leg.make_segway,
              "Ballbot_Balance": leg.make_ballbot, "Quadrotor_Hover": leg.make_quadrotor}
    F, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max, wrap_idx = makers[case]()
    d = dict(N=N, T_min=T_min, T_max=T_max, alpha=alpha, w=w, Q=Q, R=R, xg=xg, u_ref=u_ref,
             wrap_idx=np.array(wrap_idx if wrap_idx else [], dtype=np.int64))
    real_bf, real_prop = leg.bruteforce_all_Jt_backward_expansion, leg.propagator_all_Jt_aug
    calls = []

    def bf_spy(A_list, B_list, X, U, *a, **k):
        J = real_bf(A_list, B_list, X, U, *a, **k)
        calls.append(("bf", dict(A=np.array(A_list), B=np.array(B_list), X=np.array(X),
                                 U=np.array(U), J=np.array(J))))
        return J

    def prop_spy(A_aug, B_aug, Q_aug, R_list, z0, QT, T_use=None, R_inv_cached=None):
        J = real_prop(A_aug, B_aug, Q_aug, R_list, z0, QT, T_use=T_use, R_inv_cached=R_inv_cached)
        calls.append(("prop", dict(A=np.array(A_aug[:T_use]), B=np.array(B_aug[:T_use]),
                                   Q=np.array(Q_aug[:T_use]), QT=np.array(QT[:T_use]),
                                   z0=np.array(z0), R_inv=np.array(R_inv_cached),
                                   J=np.array(J))))
        return J

    leg.bruteforce_all_Jt_backward_expansion, leg.propagator_all_Jt_aug = bf_spy, prop_spy
    try:
        res = {}
        for method in ("propagator", "bruteforce"):
            calls.clear()
            res[method] = leg.ilqr_timeopt(F, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max,
                                           method=method, max_iter=20, lm_init=1e-3,
                                           S_window=10, wrap_idx=wrap_idx, use_central_diff=True)
            bf = [c for kind, c in calls if kind == "bf"][-1]
            pr = [c for kind, c in calls if kind == "prop"][-1]
            if method == "bruteforce":
                for key in ("A", "B", "X", "U", "J"):
                    d[f"bf_{key}"] = bf[key]
            else:
                for key in ("A", "B", "Q", "QT", "z0", "R_inv", "J"):
                    d[f"prop_{key}"] = pr[key]
            d[f"{method}_T_star"] = int(res[method]["T_star"])
            d[f"{method}_J_star"] = float(res[method]["J_hist"][-1])
    finally:
        leg.bruteforce_all_Jt_backward_expansion, leg.propagator_all_Jt_aug = real_bf, real_prop
    with open(os.path.join(REF, "plots", f"{case}_Jt.csv")) as f:
        rows = list(csv.DictReader(f))
    d["csv_J_bruteforce"] = np.array([float(r["J_bruteforce"]) for r in rows])
    d["csv_J_propagator"] = np.array([float(r["J_propagator"]) for r in rows])
    with open(os.path.join(REF, "plots", "summary.csv")) as f:
        for r in csv.DictReader(f):
            if r["case"] == case and r["method"] in ("propagator", "bruteforce"):
                d[f"csv_{r['method']}_T_star"] = int(r["T_star"])
                d[f"csv_{r['method']}_J_star"] = float(r["J_star"])
    np.savez_compressed(os.path.join(HERE, f"plots_{case}.npz"), **d)
    rel = np.max(np.abs(d["bf_J"] - d["csv_J_bruteforce"]) / np.abs(d["csv_J_bruteforce"]))
    print(f"plots_{case}: T*={d['bruteforce_T_star']}/{d['csv_bruteforce_T_star']} "
          f"bf vs csv {rel:.2e}")


def legacy_twin_cases(seed=9700):
    """The legacy twin's chol_inv (ilqr_propagator.py:21-31: 4 tries, then
    np.linalg.inv at eps = 1e-5) inside its propagator (ilqr_propagator.py:209-232):
    problem 0 has a Q block that needs the 3rd jitter (min eigenvalue -5e-8),
    problem 1 a QT block that exhausts the 4 tries (non-diagonal, indefinite),
    problem 2 is clean."""
    import ilqr_propagator as leg
    rng = np.random.default_rng(seed)
    d = {}
    for tag, s, m, N in (("s13_m4_N20", 13, 4, 20), ("s5_m1_N20", 5, 1, 20)):
        probs = [list(orc.synth_lft_problem(seed + 10 + i, s, m, N)) for i in range(3)]
        Qb = probs[0][2][4].copy()
        Qb = Qb - np.eye(s) * (np.linalg.eigvalsh(Qb).min() + 5e-8)
        probs[0][2] = probs[0][2].copy()
        probs[0][2][4] = Qb
        Qm, _ = np.linalg.qr(rng.standard_normal((s, s)))
        ev = rng.uniform(0.5, 3.0, s) * np.where(np.arange(s) % 2 == 0, 1.0, -1.0)
        probs[1][6] = probs[1][6].copy()
        probs[1][6][7] = Qm @ np.diag(ev) @ Qm.T
        d[f"{tag}_Q04"] = Qb
        d[f"{tag}_QT17"] = probs[1][6][7]
        d[f"{tag}_base_seed"] = seed + 10
        J = []
        for p in probs:
            A, Bm, Q, R, R_inv, z0, QT = p
            J.append(leg.propagator_all_Jt_aug(list(A), list(Bm), list(Q), [R] * N, z0, list(QT),
                                               T_use=N, R_inv_cached=R_inv))
        d[f"{tag}_J"] = np.array(J)
    np.savez_compressed(os.path.join(HERE, "legacy_twin_cases.npz"), **d)
    print("legacy_twin_cases:", sorted(d))


def bruteforce_edge_cases(seed=9800):
    """Round 3: where solver.py:293-358 raises and where it does not.  It checks
    nothing itself -- only chol_solve raises (non-finite Quu_reg / Qu / Qux, or no
    jitter factors) -- so a non-finite e at t = 0 or an overflowing V_0 leaves
    inf/NaN in J without raising.  Shapes n=4/m=2 (generic kernel) and n=12/m=4
    (the exact-size kernel); each case stores its perturbation, whether the
    reference raised, and J when it did not."""
    d = {}
    for n, m, N in ((4, 2, 12), (12, 4, 12)):
        tag = f"n{n}_m{m}"
        cases = {"clean": None, "e0_nan": ("X", (0, 1), np.nan),
                 "xT_huge": ("X", (5, 0), 1e160), "A0_inf": ("A", (0, 1, 1), np.inf),
                 "du0_nan": ("U", (0, 0), np.nan), "x3_nan": ("X", (3, 2), np.nan)}
        for name, pert in cases.items():
            A, B, X, U, xg, u_ref, Q, R, alpha = orc.synth_riccati_problem(seed, n, m, N)
            arrs = {"A": A.copy(), "X": X.copy(), "U": U.copy()}
            if pert is not None:
                arrs[pert[0]][pert[1]] = pert[2]
            raised = ""
            J = np.full(N, np.nan)
            try:
                J = np.array(ref_solver.bruteforce_all_Jt_backward_expansion(
                    list(arrs["A"]), list(B), arrs["X"], arrs["U"], xg, u_ref, Q, R, alpha,
                    0.5, N))
            except (FloatingPointError, np.linalg.LinAlgError) as e:
                raised = type(e).__name__
            k = f"{tag}_{name}"
            d[f"{k}_A"], d[f"{k}_X"], d[f"{k}_U"] = arrs["A"], arrs["X"], arrs["U"]
            d[f"{k}_raised"] = raised
            d[f"{k}_J"] = J
            print(f"bruteforce_edge {k}: raised={raised or '-'} J[:6]={J[:6]}")
        d[f"{tag}_seed"] = seed
    np.savez_compressed(os.path.join(HERE, "bruteforce_edge_cases.npz"), **d)


def legacy_bruteforce_cases(seed=9850):
    """Round 3: the legacy twin's brute force (ilqr_propagator.py:426-454) with its
    chol_solve (ilqr_propagator.py:33-43: 4 jitters, then np.linalg.lstsq of
    sym(A)).  Problem 0 has R = diag(-1, 1, ...): Quu_reg is indefinite at every
    step, all 4 jitters fail and every solve is the least-squares one; problem 1
    is clean (first try)."""
    import ilqr_propagator as leg
    d = {}
    for n, m, N in ((4, 2, 10), (12, 4, 10)):
        tag = f"n{n}_m{m}"
        for i in range(2):
            A, B, X, U, xg, u_ref, Q, R, alpha = orc.synth_riccati_problem(seed + i, n, m, N)
            if i == 0:
                R = R.copy()
                R[0, 0] = -1.0
            calls = []
            real = leg.np.linalg.lstsq

            def spy(*a, **k):
                calls.append(1)
                return real(*a, **k)

            leg.np.linalg.lstsq = spy
            try:
                J = leg.bruteforce_all_Jt_backward_expansion(list(A), list(B), X, U, xg, u_ref, Q,
                                                             R, alpha, 0.5, N)
            finally:
                leg.np.linalg.lstsq = real
            d[f"{tag}_p{i}_R"] = R
            d[f"{tag}_p{i}_J"] = np.array(J)
            d[f"{tag}_p{i}_lstsq_calls"] = len(calls)
            print(f"legacy_bruteforce {tag} p{i}: lstsq calls {len(calls)} J[:4]={np.array(J)[:4]}")
        d[f"{tag}_seed"] = seed
    np.savez_compressed(os.path.join(HERE, "legacy_bruteforce_cases.npz"), **d)


def lu_pivot_cases(seed=9900):
    """Round 3: chol_inv's LU slot where the row exchanges of gesv's partial pivoting
    matter (utils.py:88-93): an indefinite block with A[0, 0] = -0.1, so the leading
    entry of A + 0.1 I -- the first pivot of an unpivoted elimination -- is exactly
    zero while the block is regular.  Alone (inv_s*) and inside propagator sweeps
    (Q_k of problem 0 at step 3, QT of problem 1 at step 5), s = 3 (small-s kernel),
    5 (generic kernel) and 13 (hand-over -> rerun kernel)."""
    rng = np.random.default_rng(seed)
    d = {}

    def indef0(s):
        Qm, _ = np.linalg.qr(rng.standard_normal((s, s)))
        ev = rng.uniform(0.5, 3.0, s) * np.where(np.arange(s) % 2 == 0, 1.0, -1.0)
        M = Qm @ np.diag(ev) @ Qm.T
        M = 0.5 * (M + M.T)
        M[0, 0] = -0.1
        return M

    for s in (3, 5, 13):
        M = indef0(s)
        d[f"inv_s{s}_in"] = M
        d[f"inv_s{s}_out"] = ref_utils.chol_inv(M)
    for tag, s, m, N in (("s13_m4_N20", 13, 4, 20), ("s5_m1_N20", 5, 1, 20),
                         ("s3_m1_N20", 3, 1, 20)):
        probs = [list(orc.synth_lft_problem(seed + 10 + i, s, m, N)) for i in range(3)]
        probs[0][2] = probs[0][2].copy()
        probs[0][2][3] = indef0(s)
        probs[1][6] = probs[1][6].copy()
        probs[1][6][5] = indef0(s)
        d[f"lft_{tag}_Q03"] = probs[0][2][3]
        d[f"lft_{tag}_QT15"] = probs[1][6][5]
        d[f"lft_{tag}_J"] = np.array([_prop(tuple(p), N) for p in probs])
        d[f"lft_{tag}_base_seed"] = seed + 10
    np.savez_compressed(os.path.join(HERE, "lu_pivot_cases.npz"), **d)
    print("lu_pivot_cases:", sorted(d))


def legacy_riccati_cases(seed=9950):
    """Round 4: the legacy twin's Riccati passes with its chol_solve
    (ilqr_propagator.py:33-43): backward_pass_truncated (ilqr_propagator.py:375-400,
    Cholesky gate without jitter, then chol_solve) and
    value_expansions_and_gains_prefix (ilqr_propagator.py:237-287, chol_solve's
    4 jitters then np.linalg.lstsq).  Per shape, problem 0 is clean and problem 1
    has R[0, 0] = -1: Quu_reg is indefinite, mode 0 returns (None, None, False)
    and mode 1 takes the least-squares fallback at every step."""
    import ilqr_propagator as leg
    d = {}
    for n, m, N in ((4, 2, 10), (12, 4, 10)):
        tag = f"n{n}_m{m}"
        T_star, T_bar, S_right, lm = 8, 7, 2, 1e-6
        for i in range(2):
            A, B, X, U, xg, u_ref, Q, R, alpha = orc.synth_riccati_problem(seed + i, n, m, N)
            if i == 1:
                R = R.copy()
                R[0, 0] = -1.0
            k0, K0, ok = leg.backward_pass_truncated(list(A), list(B), X, U, xg, u_ref, Q, R,
                                                     alpha, T_star, lm_lambda=lm)
            d[f"{tag}_p{i}_R"] = R
            d[f"{tag}_p{i}_m0_ok"] = bool(ok)
            if ok:
                d[f"{tag}_p{i}_m0_K"] = np.array(K0)
                d[f"{tag}_p{i}_m0_k"] = np.array(k0).reshape(T_star, m)
            calls = []
            real = leg.np.linalg.lstsq

            def spy(*a, **k):
                calls.append(1)
                return real(*a, **k)

            leg.np.linalg.lstsq = spy
            try:
                Vxx, Vx, V0, K, k = leg.value_expansions_and_gains_prefix(
                    list(A), list(B), X, U, xg, u_ref, Q, R, alpha, T_bar, S_right,
                    lm_lambda=lm, w_stage=0.5)
            finally:
                leg.np.linalg.lstsq = real
            d[f"{tag}_p{i}_m1_Vxx"] = np.array(Vxx)
            d[f"{tag}_p{i}_m1_Vx"] = np.array(Vx)
            d[f"{tag}_p{i}_m1_V0"] = np.array(V0)
            d[f"{tag}_p{i}_m1_K"] = np.array(K)
            d[f"{tag}_p{i}_m1_k"] = np.array(k).reshape(len(k), m)
            d[f"{tag}_p{i}_m1_lstsq_calls"] = len(calls)
            print(f"legacy_riccati {tag} p{i}: mode0 ok={ok} mode1 lstsq calls {len(calls)}")
        d[f"{tag}_seed"] = seed
        d[f"{tag}_params"] = np.array([T_star, T_bar, S_right, lm])
    np.savez_compressed(os.path.join(HERE, "legacy_riccati_cases.npz"), **d)


def main_r4():
    np.seterr(all="ignore")
    legacy_riccati_cases()


def main_r3():
    np.seterr(all="ignore")
    bruteforce_edge_cases()
    legacy_bruteforce_cases()
    lu_pivot_cases()


def main_r2():
    np.seterr(all="ignore")
    synthetic_lft_wide("s13_m4_N100", 13, 4, 100, 11000, 16, 40, 100)
    synthetic_lft_wide("s13_m4_N128", 13, 4, 128, 12000, 16, 40, 128)
    synthetic_lft_wide("s5_m1_N200", 5, 1, 200, 13000, 16, 20, 200)
    synthetic_lft_wide("s3_m1_N50", 3, 1, 50, 14000, 16, 10, 50)
    config5_golden()
    lu_slot_cases()
    legacy_twin_cases()
    for case in LEGACY_CASES:
        legacy_plots(case)


if __name__ == "__main__":
    if "--r6" in sys.argv:  # round-6 fixtures only
        np.seterr(all="ignore")
        riccati_synth(*RICCATI_SYNTH)
    elif "--r4" in sys.argv:  # round-4 fixtures only
        main_r4()
    elif "--r3" in sys.argv:  # round-3 fixtures only
        main_r3()
    elif "--r2" in sys.argv:  # round-2 fixtures only
        main_r2()
    elif "--legacy" in sys.argv:
        np.seterr(all="ignore")
        legacy_twin_cases()
    elif "--traj" in sys.argv:  # only the trajectory-form fixtures
        main_traj()
    elif "--lin" in sys.argv:  # only the dynamics / linearisation fixtures
        main_lin()
    elif "--summary" in sys.argv:  # the plots/summary.csv comparison, both methods
        main_summary()
    elif "--ilqr-bf" in sys.argv:  # ilqr_timeopt(method="bruteforce") end to end
        main_ilqr_bruteforce()
    elif "--ilqr" in sys.argv:  # only the forward line search / outer loop fixtures
        main_ilqr()
    else:
        main()
        main_traj()
        main_lin()
        main_ilqr()
