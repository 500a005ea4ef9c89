"""Batch-scale parity on real linearisations (test infrastructure; used by
tests/test_gpu_real_lin.py and tools/real_lin_parity.py).

For one of the reference's systems (systems.py makers) build B perturbed
problems the way the first select of ilqr_timeopt sees them
(/root/reference/solver.py:480-522): x0 and U = u_ref jittered, X = rollout,
(A_k, B_k) = central-difference linearisation, residuals, the augmented
builders with the reference's q_reg = 1e-9, rho_reg = 1e-12
(augmented.py:10-87), then propagator_all_Jt_aug with T_use = T_max and the
argmin over [T_min, T_max].  Every stage runs on the device; the candidates
compared on the same inputs are

  traj      hop_lft_sweep_traj (the product select block: the conditioned
            association + its rerun launch; s = 13 the closed-form kernel,
            s <= 5 lft_small_traj_kernel<COND>)
  traj_ref  the same under HOP_OPT_REFERENCE_ASSOC: the reference association
            alone (s = 13 the trajectory LFT kernel, s <= 5 the LFT
            instantiation of lft_small_traj_kernel)
  aug       hop_augment -> hop_lft_sweep (the conditioned kernel on HBM blocks
            + its rerun launch; since round 5 also for fp64 s <= 5)
  aug_ref   the same under HOP_OPT_REFERENCE_ASSOC
  aug_gen   the same under HOP_OPT_FORCE_GENERIC (lft_sweep.hip, the reference
            association: the fp64 s = 5 drop-in path of round 4)
  oracle    oracle/hop_oracle.py (the reference's association in NumPy, pinned
            by tests/golden) on a sample of problems, from the same device
            linearisation copied to the host

None of these is ground truth on these inputs (fp64 evaluations of an
ill-conditioned association); tools/real_lin_capture.py + tests/golden/
make_hp_batch.py adjudicate their disagreements in 50-digit arithmetic.

and the hand-over count of the conditioned kernels (HOP_OPT_NO_RERUN leaves
HOP_ST_HANDOVER in status).
"""
from __future__ import annotations

import numpy as np

from oracle import hop_oracle as orc

# per system: (maker, N or None = the maker's, x0 jitter, U jitter)
SYSTEMS = {
    "quadrotor": ("make_quadrotor", 100, 0.1, 0.1),
    "segway": ("make_segway_balance", None, 0.02, 0.2),
    "cartpole": ("make_cartpole_swingup", None, 0.1, 0.5),
    "di": ("make_double_integrator", None, 0.2, 0.2),
}


def near_tie_tol(J, ta, tb):
    """Relative gap |J(ta) - J(tb)| / |J(tb)| on one J curve (1-based horizons)."""
    ja, jb = J[ta - 1], J[tb - 1]
    return abs(float(ja - jb)) / max(abs(float(jb)), 1e-300)


def build(name, Bn, seed, dev):
    """Device tensors of B problems of system `name` (see the module docstring)."""
    import torch
    from time_opt_ilqr_amd import engine, systems
    mk, N_over, sx, su = SYSTEMS[name]
    kw = {} if N_over is None else {"N": N_over}
    F, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max, wrap, _ = getattr(systems, mk)(**kw)
    T_max = min(T_max, N)
    rng = np.random.default_rng(seed)
    n, m = F.n, F.m
    X0 = x0 + sx * rng.standard_normal((Bn, n))
    U = u_ref + su * rng.standard_normal((Bn, N, m))
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float64, device=dev)  # noqa
    Ut = t(U)
    X = engine.rollout(F.system_id, t(X0), Ut, F.dt)
    lin = engine.linearize(F.system_id, X, Ut, F.dt, central=True)
    P = orc.terminal_weight(alpha, n)
    Ri = orc.spd_inverse(orc.sym(R))[0]
    return dict(F=F, X=X, U=Ut, X0=X0, U_np=U, lin=lin, xg=xg, u_ref=u_ref, Q=Q, R=R, Ri=Ri, P=P, alpha=alpha,
                w=w, N=N, T_min=T_min, T_max=T_max, wrap=wrap, t=t)


def run(d, dev):
    """The four device candidates (+ the hand-over counts) on one built batch."""
    import torch
    from time_opt_ilqr_amd import _lib, engine
    t = d["t"]
    lin = d["lin"]
    common = dict(wrap_idx=d["wrap"], t_min=d["T_min"], t_max=d["T_max"], n_use=d["T_max"])
    targs = (lin.A, lin.B, lin.a_res, d["X"], d["U"], t(d["xg"]), t(d["u_ref"]), t(d["Q"]),
             t(d["Ri"]), t(d["P"]), t(np.array([d["w"]])))
    out = {}

    def traj():
        return engine.propagate_traj(*targs, **common)

    def aug():
        blk = engine.augment(lin.A, lin.B, lin.a_res, d["X"], d["U"], t(d["xg"]), t(d["u_ref"]),
                             t(d["Q"]), t(d["P"]), t(np.array([d["w"]])), wrap_idx=d["wrap"],
                             n_build=d["T_max"])
        return engine.propagate(blk.A, blk.B, blk.Q, t(d["Ri"]), blk.z0, blk.QT,
                                t_min=d["T_min"], t_max=d["T_max"])

    out["traj"] = traj()
    out["aug"] = aug()
    with _lib.options(reference_assoc=True):
        out["traj_ref"] = traj()
        out["aug_ref"] = aug()
    with _lib.options(force_generic=True):
        out["aug_gen"] = aug()
    with _lib.options(no_rerun=True):
        ho_traj = traj().status
        ho_aug = aug().status
    torch.cuda.synchronize()
    res = {k: (v.J.cpu().numpy(), v.t_star.cpu().numpy(), v.status.cpu().numpy())
           for k, v in out.items()}
    res["handover_traj"] = int(((ho_traj & _lib.ST_HANDOVER) != 0).sum().item())
    res["handover_aug"] = int(((ho_aug & _lib.ST_HANDOVER) != 0).sum().item())
    res["ho_status_traj"] = ho_traj.cpu().numpy()
    res["ho_status_aug"] = ho_aug.cpu().numpy()
    return res


REASONS = {1: "stage inverse pivot", 2: "stage sigma", 4: "update pivot", 8: "query sigma",
           16: "query pivot", 32: "non-finite J"}


def handover_reasons(ho_status, final_status):
    """Developer builds: (reason, first failing horizon, the rerun's final status) of
    every handed-over problem (status bits 5.. of the NO_RERUN launch)."""
    out = []
    for b in np.nonzero(ho_status & 16)[0]:
        why = int(ho_status[b]) >> 5
        out.append((int(b), REASONS.get(why & 255, str(why & 255)), why >> 8,
                    int(final_status[b])))
    return out


def oracle_sample(d, idx):
    """The oracle's J curve / T* / status of problems idx from the device linearisation."""
    X = d["X"].cpu().numpy()
    U = d["U"].cpu().numpy()
    A = d["lin"].A.cpu().numpy()
    B = d["lin"].B.cpu().numpy()
    ar = d["lin"].a_res.cpu().numpy()
    Tm = d["T_max"]
    out = []
    for b in idx:
        Aa, Ba, Qa, _, z0, Ri = orc.augment_stage(list(A[b, :Tm]), list(B[b, :Tm]), ar[b, :Tm],
                                                  X[b, :Tm + 1], U[b, :Tm], d["xg"], d["u_ref"],
                                                  d["Q"], d["R"], d["w"], wrap_idx=d["wrap"])
        QT = orc.augment_terminal(X[b, :Tm + 1], d["xg"], d["alpha"], wrap_idx=d["wrap"])
        o = orc.lft_sweep(Aa, Ba, Qa, Ri, z0, QT, Tm)
        ts, _ = orc.select_horizon(o["J"], d["T_min"], Tm)
        out.append((o["J"], int(ts), int(o["status"])))
    return out


def compare(Ja, ta, Jb, tb, ok, T_min, T_max):
    """Agreement of candidate a with b over the problems `ok`: T* equality rate,
    the near-tie gap of every flipped T* (on b's curve), and the relative J
    differences in the [T_min, T_max] window."""
    sl = slice(T_min - 1, T_max)
    a, b = Ja[ok][:, sl], Jb[ok][:, sl]
    rel = np.abs(a - b) / np.maximum(np.abs(b), 1e-300)
    rel_max = np.max(rel, axis=1) if rel.size else np.zeros(0)
    flips = [int(i) for i in np.nonzero(ok)[0] if ta[i] != tb[i]]
    gaps = [near_tie_tol(Jb[i], int(ta[i]), int(tb[i])) for i in flips]
    q = (lambda p: float(np.quantile(rel_max, p))) if rel_max.size else (lambda p: 0.0)
    # J at b's selected horizon (J*): the value the select hands on
    idx = np.nonzero(ok)[0]
    js = np.array([abs(Ja[i, tb[i] - 1] - Jb[i, tb[i] - 1]) / max(abs(Jb[i, tb[i] - 1]), 1e-300)
                   for i in idx]) if idx.size else np.zeros(0)
    qs = (lambda p: float(np.quantile(js, p))) if js.size else (lambda p: 0.0)
    return dict(n=int(ok.sum()), t_equal=int(ok.sum()) - len(flips), flips=len(flips),
                jstar_rel_p50=qs(0.5), jstar_rel_p99=qs(0.99), jstar_rel_max=qs(1.0),
                flip_gap_max=max(gaps) if gaps else 0.0,
                rel_p50=q(0.5), rel_p99=q(0.99), rel_max=q(1.0),
                frac_rel_gt_1e6=float(np.mean(rel_max > 1e-6)) if rel_max.size else 0.0,
                flip_examples=[(i, int(ta[i]), int(tb[i]), g) for i, g in zip(flips[:5], gaps)])


def stats(name, Bn, seed, dev, n_oracle=32, want_raw=False):
    d = build(name, Bn, seed, dev)
    r = run(d, dev)
    T_min, T_max = d["T_min"], d["T_max"]
    Jr, tr, sr = r["traj_ref"]
    # problems the reference would select on: a finite select-window trajectory
    # (a non-finite one raises in the first select; the outer loop removes them)
    X = d["X"].cpu().numpy()
    ok = np.isfinite(X[:, :T_max + 1]).all(axis=(1, 2)) & ((sr & 12) == 0)
    out = dict(system=name, batch=Bn, seed=seed, N=d["N"], s=d["F"].n + 1, m=d["F"].m,
               T_min=T_min, T_max=T_max, finite=int(ok.sum()),
               handover_traj=r["handover_traj"], handover_aug=r["handover_aug"])
    for k in ("traj", "aug", "aug_ref", "aug_gen"):
        J, ts, st = r[k]
        out[f"{k}_vs_traj_ref"] = compare(J, ts, Jr, tr, ok, T_min, T_max)
        out[f"{k}_status_equal"] = bool(np.array_equal(st[ok], sr[ok]))
    # the two product entry points (trajectory form, augmented blocks) against each other
    Jt, tt, _ = r["traj"]
    for k in ("aug", "aug_gen"):
        J, ts, _ = r[k]
        out[f"{k}_vs_traj"] = compare(J, ts, Jt, tt, ok, T_min, T_max)
    hist = lambda st: {int(v): int(c) for v, c in zip(*np.unique(st[ok], return_counts=True))}  # noqa
    out["status_hist"] = {k: hist(r[k][2]) for k in ("traj", "traj_ref", "aug", "aug_ref",
                                                     "aug_gen")}
    # hand-overs the reference association finishes with status 0 (no jitter
    # escalation: a false positive of the conditioned form's own tests)
    for k in ("traj", "aug"):
        ho = (r[f"ho_status_{k}"] & 16) != 0
        out[f"handover_{k}_clean_final"] = int((ho & (r[k][2] == 0)).sum())
        out[f"handover_{k}_reasons"] = handover_reasons(r[f"ho_status_{k}"], r[k][2])[:40]
    # oracle spot check: evenly spread sample of the finite problems
    cand = np.nonzero(ok)[0]
    idx = cand[np.linspace(0, len(cand) - 1, min(n_oracle, len(cand))).astype(int)]
    orr = oracle_sample(d, idx)
    Jo = np.zeros((Bn, T_max))
    to = np.zeros(Bn, dtype=np.int64)
    so = np.zeros(Bn, dtype=np.int64)
    sel = np.zeros(Bn, dtype=bool)
    for b, (J, ts, st) in zip(idx, orr):
        Jo[b], to[b], so[b], sel[b] = J, ts, st, True
    for k in ("traj", "traj_ref", "aug", "aug_gen"):
        J, ts, st = r[k]
        out[f"{k}_vs_oracle"] = compare(J, ts, Jo, to, sel, T_min, T_max)
    if want_raw:
        return out, dict(d=d, r=r, ok=ok, oracle_idx=idx, oracle_J=Jo[idx], oracle_t=to[idx])
    return out
