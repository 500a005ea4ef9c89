#!/usr/bin/env python3
"""Benchmark: batched LFT backward sweeps/s (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
                    [--workload lft|config3|config5|select_gains|bruteforce]
    torchrun --nproc-per-node N bench.py --gpus N ...      (driver form, N > 1)

A "step" is one pass of the hot path over one batch: the fused LFT sweep
(stage + prefix compose + all-horizon query) of every problem plus the fused
horizon argmin, with the (T*, J*) all-gather over RCCL when N > 1.  Inputs are
synthetic blocks resident in HBM before timing.  Rank 0 prints ONE JSON line.

Workloads (BASELINE.json configs):
  lft (default)  N=1: config 2 -- Quadrotor shape s=13, m=4, N=100, 4096 problems, fp64.
                 N>1: config 4 -- the same shape, 32768 problems per GPU (262144 on 8
                 GPUs), contiguous shards, weak scaling.  --scaling strong keeps config
                 4's global batch of 262144 for every N (--global-batch to change it);
                 the N=1 default line carries both config-4 anchors (32768 and 262144
                 problems on one GPU).
  config3        Cartpole shape s=5, m=1, N=200, 65536 problems, fp32 (small-s kernel),
                 blocks in the kernel's native tile64 layout (include/hop.h; --layout
                 batch for batch-major blocks, which is also timed as a side figure).
  config5        mixed Segway / Cartpole / Quadrotor (i mod 3) padded to s=13, m=4,
                 N=128, 16384 problems per GPU (131072 on 8), fp32 blocks.
  select_gains   the select + backward of solver.py:581-597: trajectory-form select
                 (in-kernel augmentation + LFT + argmin) followed by the truncated
                 Riccati gains at each problem's T* (n=12, m=4, N=100, 4096, fp64).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

PEAK_F64_TFLOPS = 78.6   # MI355X dense fp64 (vector == matrix), MI355X_MICROARCH.md / datasheet
PEAK_F32_TFLOPS = 157.3  # MI355X fp32 vector (packed)
PEAK_HBM_GBS = 8000.0
SMALL_SHAPES = {"f32": {(2, 1), (3, 1), (4, 1), (4, 2), (5, 1), (5, 2)},
                "f64": {(2, 1), (3, 1), (4, 1), (4, 2)}}
CONFIG5_ALG_FLOPS = 2472905  # mean over the true shapes (13/4 and 5/1 x2)


def baseline_metric():
    """BASELINE.json's metric string (the driver compares the line against it)."""
    try:
        with open(os.path.join(REPO, "BASELINE.json")) as f:
            return json.load(f)["metric"]
    except (OSError, ValueError, KeyError):
        return "batched iLQR backward sweeps/sec, Quadrotor n=13 N=100, at 1/2/4/8 GPU"


def _cu_count():
    """CUs of the current device, as the library's dispatcher sees them (its cu_count
    reads hipDeviceAttributeMultiprocessorCount; 256 if unknown, as the library)."""
    try:
        import torch
        if torch.cuda.is_available():
            return int(torch.cuda.get_device_properties(torch.cuda.current_device())
                       .multi_processor_count)
    except Exception:  # noqa: BLE001 - a CPU dry run
        pass
    return 256


def kernel_path(s, m, dtype, batch=4096, cus=None):
    """Which kernel libhop_amd.so dispatches for this shape, and its roofline bound.
    The s=13 kernels are compute-bound on the fp64 pipe (MI355X: vector fp64 peak ==
    matrix fp64 peak); they issue DPP-broadcast FMAs, not MFMA.  Above
    one wave per SIMD (4 problems per wave, 4 SIMDs per CU) the s=13 fp64 path takes the
    packed two-waves-per-SIMD layout."""
    if dtype == "f64" and (s, m) == (13, 4):
        packed = (batch + 3) // 4 > 4 * (cus or _cu_count())
        return f"lft_cond_kernel<{'SchedCondLSymP' if packed else 'SchedCondLSymL'},13,4>", "fp64"
    if dtype == "f32" and (s, m) == (13, 4):
        return "lft_cond_kernel<SchedCond,13,4,float>", "fp64"  # fp32 blocks, fp64 arithmetic
    if (s, m) in SMALL_SHAPES[dtype]:
        return f"lft_small_kernel<{'float' if dtype == 'f32' else 'double'},{s},{m}>", "hbm"
    return "lft_sweep_kernel", "fp64" if dtype == "f64" else "fp32"


def lft_flops(N, s, m):
    """Algorithmic FLOPs of one sweep."""
    return N * (23 * s ** 3 + 2 * s * m * m + 2 * s * s * m) - 11 * s ** 3


def cond_flops(N, s, m):
    """FLOPs the conditioned-prefix kernel executes per sweep: two
    SPD inverses (2 s^3), the update LDL^T with its (s+1)-wide forward substitution
    and rank-1 streams (~10/3 s^3), the predict products (4 s^3 + B R^-1 B^T) and
    the bordered query elimination (s^3 / 3)."""
    return N * (29 * s ** 3 // 3 + 2 * s * m * m + 2 * s * s * m)


def cf_flops(N, s, m):
    """FLOPs the trajectory-form conditioned kernel (lft_cond_cf_kernel, closed-form
    stage inverses) executes per sweep: cond_flops without the two per-step
    Gauss-Jordan inverses (2 s^3), plus per step the three n x n mat-vecs (Qi q,
    Q e, Pi e: 6 n^2) and the two rank-1 corrections of the closed forms (4 s^2),
    and once per problem the two n x n inverses (Qs + eps I, P + eps I: 2 n^3)."""
    n = s - 1
    return N * (23 * s ** 3 // 3 + 2 * s * m * m + 2 * s * s * m + 6 * n * n + 4 * s * s) + 2 * n ** 3


def small_flops(N, s, m):
    """FLOPs the small-s kernel (lft_small_kernel, conditioned association, one
    problem per lane) executes per sweep: the conditioned count at the true s."""
    return cond_flops(N, s, m)


def lft_bytes(N, s, m, w=8):
    """Algorithmic HBM bytes of one sweep."""
    return w * (N * (3 * s * s + s * m) + m * m + s + N)


def riccati_flops(n, m, T, mode=0):
    """SURVEY.md 8(d) Riccati add-on, (4n^3 + 10n^2 m + O(n^2 + nm^2 + m^3)) per step
    (~1.49 MFLOP at n=12, m=4, T=100), with the lower-order terms counted term by
    term as a competent implementation does them (solver.py:199-225 for mode 0,
    horizon_selection.py:150-207 for mode 1): lx = Q e (2n^2), lu = R du (2m^2);
    Qx, Qu (2n^2 + 2nm); V [A|B] (2n^2 (n+m)); Qxx = Q + A^T(VA) (2n^3 + n^2);
    Qux (2n^2 m); Quu = R + B^T(VB) (2nm^2 + m^2); the m x m factor (m^3/3) and
    the k, K solves (2m^2 + 2m^2 n).  Mode 0's value update Vx = Qx + K^T Qu +
    Qux^T k + K^T Quu k (6nm + 2m^2) and Vxx = Qxx + K^T Qux + Qux^T K + K^T Quu K
    (6n^2 m + 2nm^2); mode 1's Vxx = Qxx - Qux^T Quu^-1 Qux (2n^2 m), Vx (2nm) and
    V0 with l0 (4n + 4m)."""
    step = (2 * n * n + 2 * m * m + 2 * n * n + 2 * n * m + 2 * n * n * (n + m)
            + 2 * n ** 3 + n * n + 2 * n * n * m + 2 * n * m * m + m * m + m ** 3 // 3
            + 2 * m * m + 2 * m * m * n)
    if mode == 0:
        step += 6 * n * m + 2 * m * m + 6 * n * n * m + 2 * n * m * m
    else:
        step += 2 * n * n * m + 2 * n * m + 4 * n + 4 * m
    return step * T


def riccati_bytes(n, m, T, mode=0, want_v=None):
    """Algorithmic HBM bytes per problem of one Riccati pass (fp64): per step A_k,
    B_k, x_k, u_k read and K_k, k_k written; with the value expansions (mode 1, or
    mode 0 when Vxx is requested) Vxx, Vx, V0 written at every step and the
    terminal one; plus x_T and the terminal reads.  Mode 1 moves 3,336 B per step
    at n = 12, m = 4 against ~1.2e4 FLOP: its bound is HBM, not fp64."""
    want_v = (mode == 1) if want_v is None else want_v
    step = n * n + n * m + n + m + m * n + m
    if want_v:
        step += n * n + n + 1
    return 8 * (step * T + n + ((n * n + n + 1) if want_v else 0))


# ---------------------------------------------------------------------------
# CPU baseline: the oracle's NumPy restatement on the host cores (rank 0 only)
# ---------------------------------------------------------------------------

def host_cores():
    """CPUs this process may actually use: the affinity mask, capped by a cgroup
    v2 cpu.max quota when one is set (a GPU box shows the whole machine in
    os.cpu_count() but grants a share of it)."""
    n = os.cpu_count() or 1
    try:
        n = min(n, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_worker(args):
    seed0, count, s, m, N = args
    from oracle import hop_oracle as orc
    t0 = time.perf_counter()
    for i in range(count):
        A, Bm, Q, R, Ri, z0, QT = orc.synth_lft_problem(seed0 + i, s, m, N)
        orc.lft_sweep(A, Bm, Q, Ri, z0, QT, N)
    return count, time.perf_counter() - t0


def _cpu_worker_bf(args):
    seed0, count, n, m, N = args
    from oracle import hop_oracle as orc
    t0 = time.perf_counter()
    for i in range(count):
        A, Bm, X, U, xg, ur, Q, R, Qf = synth_riccati_problem(seed0 + i, n, m, N)
        orc.bruteforce_J(list(A), list(Bm), X, U, xg, ur, Q, R, Qf, 0.5, N)
    return count, time.perf_counter() - t0


def synth_riccati_problem(seed, n, m, N):
    """One problem of the Riccati workloads' distribution (NumPy PCG64; the device
    runs draw the same distribution from torch's generator)."""
    import numpy as np
    rng = np.random.default_rng(int(seed))
    A = np.eye(n) + 0.05 * rng.standard_normal((N, n, n))
    Bm = 0.1 * rng.standard_normal((N, n, m))
    X = 0.5 * rng.standard_normal((N + 1, n))
    U = 0.3 * rng.standard_normal((N, m))
    xg = 0.2 * rng.standard_normal(n)
    ur = 0.1 * rng.standard_normal(m)
    M = rng.standard_normal((n, n))
    Q = M @ M.T / n + 0.5 * np.eye(n)
    R = np.diag(0.5 + 1.5 * rng.random(m))
    Qf = np.diag(1.0 + 9.0 * rng.random(n))
    return A, Bm, X, U, xg, ur, Q, R, Qf


def cpu_baseline(s, m, N, target_s=8.0, bruteforce=False):
    """Sweeps/s of the NumPy restatement on every usable host core (one process
    per core, one BLAS thread each); the per-process sample is sized from a
    one-sweep probe to about target_s seconds of work."""
    import multiprocessing as mp
    cores = host_cores()
    os.environ["OPENBLAS_NUM_THREADS"] = "1"
    os.environ["OMP_NUM_THREADS"] = "1"
    ctx = mp.get_context("spawn")
    work = _cpu_worker_bf if bruteforce else _cpu_worker
    dim = s - 1 if bruteforce else s  # the brute-force curve runs on the raw n = s - 1
    with ctx.Pool(cores) as pool:
        probe = pool.map(work, [(0, 1 if bruteforce else 2, dim, m, N)] * cores)  # imports + probe
        per_sweep = max(t / c for c, t in probe)
        per_core = max(2 if bruteforce else 4, int(target_s / max(per_sweep, 1e-6)))
        jobs = [(10_000 + c * per_core, per_core, dim, m, N) for c in range(cores)]
        t0 = time.perf_counter()
        res = pool.map(work, jobs)
        wall = time.perf_counter() - t0
    done = sum(r[0] for r in res)
    if bruteforce:
        return {"value": done / wall, "unit": "problems/s", "cores": cores, "kind": "port",
                "cpu_model": cpu_model(), "os_cpu_count": os.cpu_count(),
                "sample": f"{done} brute-force J curves (n={dim}, m={m}, T_max={N}, fp64: "
                          f"{N} Riccati sweeps each) of oracle/hop_oracle.bruteforce_J, {cores} "
                          f"processes x 1 BLAS thread, {wall:.1f} s wall"}
    return {"value": done / wall, "unit": "sweeps/s", "cores": cores, "kind": "port",
            "cpu_model": cpu_model(), "os_cpu_count": os.cpu_count(),
            "sample": f"{done} synthetic sweeps (s={s}, m={m}, N={N}, fp64) of the NumPy "
                      f"restatement oracle/hop_oracle.py, {cores} processes x 1 BLAS thread, "
                      f"{wall:.1f} s wall"}


# ---------------------------------------------------------------------------
# workloads: each returns (launch(), problems per step, description dict)
# ---------------------------------------------------------------------------

def _lft_workload(args, world, lo, hi, dev):
    import torch
    from time_opt_ilqr_amd import engine, synth
    s, m, N = args.s, args.m, args.N
    dtype = torch.float64 if args.dtype == "f64" else torch.float32
    A, Bm, Q, Ri, z0, QT = synth.device_batch(hi - lo, s, m, N, seed=1234 + lo, device=dev,
                                              dtype=dtype)
    t_min, t_max = min(args.t_min, N), N
    small = (s, m) in SMALL_SHAPES[args.dtype]
    tiled = args.layout == "tile64" or (args.layout == "auto" and small and s == 5)
    if tiled and not small:
        raise SystemExit("--layout tile64: s <= 5 small-s shapes only")

    def launch_bm():
        return engine.propagate(A, Bm, Q, Ri, z0, QT, t_min=t_min, t_max=t_max)

    launch, host, alt = launch_bm, (A, Bm, Q, Ri, z0, QT), None
    if tiled:  # the layout conversion is setup, outside the timed region
        At, Bt, Qt, QTt = (engine.to_tile64(x) for x in (A, Bm, Q, QT))

        def launch():
            return engine.propagate(At, Bt, Qt, Ri, z0, QTt, t_min=t_min, t_max=t_max)

        host, alt = (At.data, Bt.data, Qt.data, Ri, z0, QTt.data), launch_bm

    side = _traj64_side(hi - lo, s, m, N, t_min, dtype, dev) if tiled else None
    if (s, m, args.dtype) == (13, 4, "f64") and not tiled and world == 1 and not args.no_alt:
        side = _quad_side(hi - lo, N, t_min, dev)
    kname, bound = kernel_path(s, m, args.dtype, hi - lo)
    if small:
        kname = kname[:-1] + (",LY=2 tile64>" if tiled else ",LY=1 batch-major>")
    w = 8 if args.dtype == "f64" else 4
    info = dict(kernel=kname, bound=bound, flops=lft_flops(N, s, m), bytes=lft_bytes(N, s, m, w),
                executed=(cond_flops(N, s, m) if kname.startswith("lft_cond") else
                          small_flops(N, s, m) if kname.startswith("lft_small") else None),
                t_min=t_min, t_max=t_max, s=s, m=m, N=N, host=host, alt=alt,
                layout="tile64" if tiled else "batch-major", side=side)
    return launch, info


def _traj64_side(Bn, s, m, N, t_min, dtype, dev):
    """Config 3 from the raw linearisation, timed beside the
    line (cart-pole, s = 5, m = 1 only): Bn cart-pole rollouts (systems.py:57-112)
    linearised by central differences straight into the tile64 layout
    (hop_linearize_tile64_*, linearization.py:177-211), then the select block
    (augmented.py:10-87 built per lane in registers + propagator + argmin,
    solver.py:514-522) streaming those raw A_k, B_k, a_k, x_k, u_k
    (hop_lft_sweep_traj_tile64_*).  `select_traj64` times the select alone on one
    linearisation, `linearize_select_traj64` both stages.  The cost is the
    well-conditioned one of tests/test_gpu_traj.py's config-3-size test at
    rho_reg = 1: the maker's zero angle weight and rho_reg = 1e-12 give Schur
    complements an fp32 sweep cannot resolve (they hand problems to the rerun)."""
    if (s, m) != (5, 1):
        return None
    import numpy as np
    import torch
    from time_opt_ilqr_amd import engine, systems
    g = torch.Generator(device=dev)
    g.manual_seed(17)
    F, x0, xg, u_ref = systems.make_cartpole_swingup(N=N)[:4]
    wrap = [2]
    g64 = dict(device=dev, dtype=torch.float64, generator=g)
    U = 2.0 * torch.randn((Bn, N, 1), **g64)
    X = engine.rollout(F.system_id, torch.as_tensor(x0, device=dev) +
                       0.3 * torch.randn((Bn, 4), **g64), U, F.dt)
    f = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float64), device=dev, dtype=dtype)  # noqa
    alpha = np.array([5.0, 5.0, 20.0, 5.0])
    shared = (f(xg), f(u_ref), f(np.diag([1.0, 0.5, 2.0, 0.5])), f([[10.0]]), f(np.diag(alpha)),
              f([0.03]))

    def lin():
        return engine.linearize(F.system_id, X, U, F.dt, central=True, tile64=True,
                                tile64_dtype=dtype)

    lin0 = lin()

    def select_on(L):
        return engine.propagate_traj(L.A, L.B, L.a_res, L.X, L.U, *shared, wrap_idx=wrap,
                                     rho_reg=1.0, t_min=t_min, t_max=N)

    n = s - 1
    return {"name": "config3_from_linearisation", "select_key": "select_traj64",
            "fns": {"select_traj64": lambda: select_on(lin0),
                    "linearize_select_traj64": lambda: select_on(lin())},
            "select_bytes_per_sweep": (N * (n * n + n * m + 2 * n + m) + n) *
                                      (4 if dtype == torch.float32 else 8),
            "note": ("cart-pole rollouts linearised into tile64 (hop_linearize_tile64), raw A_k, "
                     "B_k, a_k, x_k, u_k streamed by hop_lft_sweep_traj_tile64; select_traj64 = "
                     "the select alone, linearize_select_traj64 = both stages in the timing; "
                     "well-conditioned cost, rho_reg = 1 (fp32)")}


def _quad_side(Bn, N, t_min, dev):
    """Config 2's shape from the raw linearisation, timed beside the line: Bn perturbed
    quadrotor rollouts (systems.py:119-230 maker, x0 + 0.1 N(0, 1), U = u_ref + 0.05
    N(0, 1)), the forward-difference linearisation of ilqr_timeopt's default
    (linearization.py:177-211), then the select block on it (augmented.py:10-87 in
    registers + the closed-form conditioned kernel + argmin, solver.py:514-522) with
    the maker's cost at the reference's rho_reg = 1e-12.  `select_traj` times the select
    alone on one linearisation, `linearize_select_traj` both stages."""
    import numpy as np
    import torch
    from time_opt_ilqr_amd import engine, systems
    from time_opt_ilqr_amd.utils import as_terminal_weight
    F, x0, xg, u_ref, Q, R, alpha, w, _, _, _, wrap, _ = systems.make_quadrotor(N=N)
    g = torch.Generator(device=dev)
    g.manual_seed(23)
    kw = dict(device=dev, dtype=torch.float64, generator=g)
    U = torch.as_tensor(u_ref, device=dev) + 0.05 * torch.randn((Bn, N, F.m), **kw)
    X = engine.rollout(F.system_id, torch.as_tensor(x0, device=dev) +
                       0.1 * torch.randn((Bn, F.n), **kw), U, F.dt)
    t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float64), device=dev)  # noqa: E731
    shared = (t(xg), t(u_ref), t(Q), torch.linalg.inv(t(R)).contiguous(), t(as_terminal_weight(alpha, F.n)),
              t([w]))

    def lin():
        return engine.linearize(F.system_id, X, U, F.dt, central=False)

    lin0 = lin()

    def select_on(L):
        return engine.propagate_traj(L.A, L.B, L.a_res, X, U, *shared, wrap_idx=wrap,
                                     t_min=t_min, t_max=N)

    n, m = F.n, F.m
    return {"name": "config2_from_linearisation", "select_key": "select_traj",
            "fns": {"select_traj": lambda: select_on(lin0),
                    "linearize_select_traj": lambda: select_on(lin())},
            "select_bytes_per_sweep": (N * (n * n + n * m + 2 * n + m) + n) * 8,
            "note": ("quadrotor rollouts linearised by forward differences (hop_linearize_f64), "
                     "then hop_lft_sweep_traj_f64 (closed-form conditioned kernel) at "
                     "rho_reg = 1e-12; select_traj = the select alone, linearize_select_traj = "
                     "both stages; problems_status_ok counts the problems with a clean status "
                     "and finite curve")}


def _s5_aug_side(dev, Bn=4096, N=200, t_min=40):
    """fp64 s = 5 augmented blocks, timed beside the config-2 line:
    Bn perturbed cart-pole rollouts (systems.py:57-112 maker: its Q with the zero angle
    weight, R, alpha, w, the angle wrap), central-difference linearisation
    (linearization.py:177-211), the reference's builders on the device (augmented.py:
    10-87, hop_augment_f64, rho_reg = 1e-12), then propagator_all_Jt_aug + argmin on
    those blocks (horizon_selection.py:36-86, solver.py:521): the drop-in's path, the
    small-s conditioned kernel + its rerun launch (hop_lft_sweep_f64).  `select_aug`
    times the sweep alone, `augment_select_aug` the builders too; `select_aug_reference_
    assoc` the same sweep with the reference association (HOP_OPT_REFERENCE_ASSOC); the
    T* agreement with the trajectory-form select (hop_lft_sweep_traj_f64) on the same
    linearisation is counted."""
    import numpy as np
    import torch
    from time_opt_ilqr_amd import _lib, engine, systems
    from time_opt_ilqr_amd.utils import as_terminal_weight
    F, x0, xg, u_ref, Q, R, alpha, w, _, _, _, wrap, _ = systems.make_cartpole_swingup(N=N)
    g = torch.Generator(device=dev)
    g.manual_seed(29)
    kw = dict(device=dev, dtype=torch.float64, generator=g)
    U = torch.as_tensor(u_ref, device=dev) + 2.0 * torch.randn((Bn, N, F.m), **kw)
    X = engine.rollout(F.system_id, torch.as_tensor(x0, device=dev) +
                       0.3 * torch.randn((Bn, F.n), **kw), U, F.dt)
    t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float64), device=dev)  # noqa: E731
    P = t(as_terminal_weight(alpha, F.n))
    Ri = torch.linalg.inv(t(R)).contiguous()
    lin = engine.linearize(F.system_id, X, U, F.dt, central=True)
    shared = (t(xg), t(u_ref), t(Q))

    def build():
        return engine.augment(lin.A, lin.B, lin.a_res, X, U, *shared, P, w, wrap_idx=wrap)

    blk = build()

    def sweep(b):
        return engine.propagate(b.A, b.B, b.Q, Ri, b.z0, b.QT, t_min=t_min, t_max=N)

    def timed(fn, opts=None):
        with _lib.options(**(opts or {})):
            r_ = fn()
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                fn()
            e1.record()
            torch.cuda.synchronize()
        return r_, e0.elapsed_time(e1) / 10

    out = {}
    r_a, ms = timed(lambda: sweep(blk))
    for key, fn, opts in (("select_aug", None, None),
                          ("augment_select_aug", lambda: sweep(build()), None),
                          ("select_aug_reference_assoc", lambda: sweep(blk),
                           {"reference_assoc": True})):
        r_, ms_ = (r_a, ms) if fn is None else timed(fn, opts)
        fin = torch.isfinite(r_.J).all(dim=1)
        out[key] = {"ms": ms_, "sweeps_per_s": Bn / (ms_ * 1e-3),
                    "problems_status_ok": int(((r_.status == 0) & fin).sum().item())}
    tr = engine.propagate_traj(lin.A, lin.B, lin.a_res, X, U, *shared, Ri, P, w, wrap_idx=wrap,
                               t_min=t_min, t_max=N)
    torch.cuda.synchronize()
    ok = torch.isfinite(r_a.J).all(dim=1) & torch.isfinite(tr.J).all(dim=1)
    out["t_star_equal_traj_form"] = int(((r_a.t_star == tr.t_star) & ok).sum().item())
    # s <= 5 hand-overs: one of these problems with the stage block made
    # indefinite at every other step (chol_inv's ladder ends in the LU slot there, as the
    # point-mass obstacle cost makes it), so the conditioned kernel hands them over; the
    # pipelined rerun against the one-lane rerun (HOP_OPT_RERUN_LANE), bitwise compared
    h = slice(0, 1)
    Qh = blk.Q[h].clone()
    Qh[:, 1::2, 0, 0] -= 1.0
    hargs = (blk.A[h].contiguous(), blk.B[h].contiguous(), Qh, Ri, blk.z0, blk.QT[h].contiguous())
    r_p, ms_p = timed(lambda: engine.propagate(*hargs, t_min=t_min, t_max=N))
    r_l, ms_l = timed(lambda: engine.propagate(*hargs, t_min=t_min, t_max=N), {"rerun_lane": True})
    out["handover_rerun"] = {
        "ms_pipelined": ms_p, "ms_one_lane": ms_l, "speedup": ms_l / ms_p,
        "problems_lu_slot": int(((r_p.status & _lib.ST_LU) != 0).sum().item()),
        "bitwise_equal": bool(torch.equal(r_p.J.nan_to_num(7.0), r_l.J.nan_to_num(7.0)) and
                              torch.equal(r_p.status, r_l.status) and torch.equal(r_p.t_star, r_l.t_star)),
        "workload": "one of the batch's problems, Q_aug[k][0][0] - 1 at odd k (ladder + LU slot): "
                    "select + rerun launch, pipelined against one lane"}
    out["problems_finite_both"] = int(ok.sum().item())
    out["workload"] = (f"fp64 s = 5, m = 1, N = {N}, B = {Bn}: cart-pole augmented blocks "
                       "(rho_reg = 1e-12) through propagator_all_Jt_aug + argmin")
    return out


def _config5_workload(args, world, lo, hi, dev):
    import torch
    from time_opt_ilqr_amd import engine, synth
    N = args.N
    Bn = hi - lo
    mb, groups = synth.config5_batch(Bn, N, seed=77 + lo, device=dev, dtype=torch.float32)
    t_min = min(args.t_min, N)

    def launch_padded():
        return engine.propagate(mb.A, mb.B, mb.Q, mb.R_inv, mb.z0, mb.QT, t_min=t_min, t_max=N)

    if args.layout in ("auto", "bucketed"):
        # shape buckets: the Quadrotor third on the s=13 fp32-block kernel, the
        # Segway / Cartpole members at their true s=5 on the small-s kernel (tile64
        # blocks, side stream); J as the padded launch (block-decoupled embedding)
        from time_opt_ilqr_amd.packing import merge_by_shape
        sgroups, sorder = merge_by_shape(groups, torch.arange(Bn) % 3)  # s=5 kinds: one launch
        plan = engine.mixed_plan(sorder, len(sgroups), dev)
        tg = []
        for A, B, Q, Ri, z0, QT in sgroups:
            if A.shape[-1] <= 5:
                A, B, Q, QT = (engine.to_tile64(x) for x in (A, B, Q, QT))
            tg.append((A, B, Q, Ri, z0, QT))

        def launch():
            return engine.propagate_groups(tg, plan, t_min=t_min, t_max=N)

        kname = ("lft_cond_kernel<SchedCond,13,4,float> (Quadrotor third) + "
                 "lft_small_kernel<float,5,1,LY=2 tile64> (Segway/Cartpole, side stream)")
        alg_bytes = (lft_bytes(N, 13, 4, 4) + 2 * lft_bytes(N, 5, 1, 4)) // 3
        info = dict(kernel=kname, bound="fp64", flops=CONFIG5_ALG_FLOPS, bytes=alg_bytes,
                    executed=(cond_flops(N, 13, 4) + 2 * small_flops(N, 5, 1)) // 3,
                    t_min=t_min, t_max=N, s=13, m=4, N=N, host=None,
                    alt=launch_padded, layout="shape-bucketed (true s; padded s=13 timed beside)")
        return launch, info
    info = dict(kernel="lft_cond_kernel<SchedCond,13,4,float>", bound="fp64",
                flops=CONFIG5_ALG_FLOPS, bytes=lft_bytes(N, 13, 4, 4),
                executed=cond_flops(N, 13, 4), t_min=t_min, t_max=N, s=13, m=4, N=N,
                host=(mb.A, mb.B, mb.Q, mb.R_inv, mb.z0, mb.QT), layout="padded to s=13")
    return launch_padded, info


def _select_gains_workload(args, world, lo, hi, dev):
    import torch
    from time_opt_ilqr_amd import engine
    Bn, n, m, N = hi - lo, args.s - 1, args.m, args.N
    g = torch.Generator(device=dev)
    g.manual_seed(11 + lo)
    kw = dict(device=dev, dtype=torch.float64, generator=g)
    eye = torch.eye(n, device=dev, dtype=torch.float64)
    A = eye + 0.05 * torch.randn((Bn, N, n, n), **kw)
    Bm = 0.1 * torch.randn((Bn, N, n, m), **kw)
    X = 0.5 * torch.randn((Bn, N + 1, n), **kw)
    U = 0.3 * torch.randn((Bn, N, m), **kw)
    a_res = 0.02 * torch.randn((Bn, N, n), **kw)
    xg = 0.2 * torch.randn((n,), **kw)
    ur = 0.1 * torch.randn((m,), **kw)
    M = torch.randn((n, n), **kw)
    Q = M @ M.T / n + 0.5 * eye
    R = torch.diag(0.5 + 1.5 * torch.rand((m,), **kw))
    Rinv = torch.linalg.inv(R).contiguous()  # linalg.inv is column-major: a copy per call otherwise
    P = torch.diag(1.0 + 9.0 * torch.rand((n,), **kw))
    w = 0.5
    t_min = min(args.t_min, N)

    def launch():
        sel = engine.propagate_traj(A, Bm, a_res, X, U, xg, ur, Q, Rinv, P, w, t_min=t_min,
                                    t_max=N, rho_reg=args.rho_reg)
        ric = engine.riccati(A, Bm, X, U, xg, ur, Q, R, P, sel.t_star, 1e-3, mode=0)
        sel.riccati_status = ric.status
        return sel

    # the Riccati gains run to each problem's T*, not to N: both counts take the
    # batch's mean T* once the step has run (flops_fn / executed_fn)
    info = dict(kernel="lft_cond_cf_kernel<SchedCondTraj,13,4> + riccati_fast_kernel<0>",
                bound="fp64", flops=lft_flops(N, n + 1, m) + riccati_flops(n, m, N),
                bytes=8 * (N * (n * n + n * m + 2 * n + m) + n),
                executed=cf_flops(N, n + 1, m) + riccati_flops(n, m, N),
                flops_fn=lambda tbar: lft_flops(N, n + 1, m) + riccati_flops(n, m, 1) * tbar,
                executed_fn=lambda tbar: cf_flops(N, n + 1, m) + riccati_flops(n, m, 1) * tbar,
                t_min=t_min, t_max=N, s=n + 1, m=m, N=N, host=None, rho_reg=args.rho_reg)
    return launch, info


def _bruteforce_workload(args, world, lo, hi, dev):
    """baseline1's select (solver.py:293-358 + the argmin of solver.py:613): the
    brute-force J curve of T_max = N Riccati sweeps per problem in one launch."""
    import types
    import torch
    from time_opt_ilqr_amd import engine
    Bn, n, m, N = hi - lo, args.s - 1, args.m, args.N
    g = torch.Generator(device=dev)
    g.manual_seed(13 + lo)
    kw = dict(device=dev, dtype=torch.float64, generator=g)
    eye = torch.eye(n, device=dev, dtype=torch.float64)
    A = eye + 0.05 * torch.randn((Bn, N, n, n), **kw)
    Bm = 0.1 * torch.randn((Bn, N, n, m), **kw)
    X = 0.5 * torch.randn((Bn, N + 1, n), **kw)
    U = 0.3 * torch.randn((Bn, N, m), **kw)
    xg = 0.2 * torch.randn((n,), **kw)
    ur = 0.1 * torch.randn((m,), **kw)
    M = torch.randn((n, n), **kw)
    Q = M @ M.T / n + 0.5 * eye
    R = torch.diag(0.5 + 1.5 * torch.rand((m,), **kw))
    Qf = torch.diag(1.0 + 9.0 * torch.rand((n,), **kw))
    t_min = min(args.t_min, N)

    def launch():
        J, st = engine.bruteforce_jcurve(A, Bm, X, U, xg, ur, Q, R, Qf, N, lm_lambda=1e-6,
                                         w_stage=0.5)
        t, j = engine.select_horizon(J, t_min, N)
        return types.SimpleNamespace(t_star=t, j_star=j, J=J, status=st)

    bf = sum(riccati_flops(n, m, T, 1) for T in range(1, N + 1))
    info = dict(kernel="riccati_fast_jcurve_kernel (J-curve form, horizon pairs)", bound="fp64",
                flops=bf, bytes=8 * (N * (n * n + n * m + m) + (N + 1) * n) + 12 * N,
                executed=bf,  # the J-curve steps are mode-1 steps: the counted arithmetic
                t_min=t_min, t_max=N, s=n + 1, m=m, N=N, host=None)
    return launch, info


WORKLOADS = {"lft": _lft_workload, "config3": _lft_workload, "config5": _config5_workload,
             "select_gains": _select_gains_workload, "bruteforce": _bruteforce_workload}


def _free_port():
    import socket
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    port = so.getsockname()[1]
    so.close()
    return port


def _self_launch(args, argv):
    """`python bench.py --gpus N` with N > 1 and no torchrun environment: start one
    rank per GPU through torch.distributed.run as a CHILD process (nothing in this
    process has touched the GPU: torch.cuda.device_count() does not initialise it on
    this image) and exit with its return code."""
    import subprocess
    if not args.dry_run and args.dist_backend == "nccl":
        import torch
        have = torch.cuda.device_count()
        if have < args.gpus:
            print(f"bench.py: --gpus {args.gpus} but only {have} HIP device(s) visible",
                  file=sys.stderr, flush=True)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def _dry_workload(args, world, lo, hi, dev):
    """--dry-run: the CPU stand-in for a rank's shard (no HIP), loaded from tests/
    (it computes (T*, J*) with the oracle).  Only the gloo rehearsal of bench.py's
    rank / shard / gather path uses it; the product path never does."""
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "_bench_dry_standin", os.path.join(REPO, "tests", "bench_dry_standin.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.workload(args, world, lo, hi, dev)


def args_with_batch(args, batch):
    import copy
    a = copy.copy(args)
    a.batch = batch
    return a


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default per workload: about 2-5 s of GPU time, so the "
                         "run's GPU phase is long enough to observe; 20 when N > 1)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="lft")
    ap.add_argument("--batch", type=int, default=None,
                    help="problems per GPU (default: the workload's config size)")
    ap.add_argument("--s", type=int, default=None)
    ap.add_argument("--m", type=int, default=None)
    ap.add_argument("--N", type=int, default=None)
    ap.add_argument("--t-min", type=int, default=40)
    ap.add_argument("--dtype", choices=["f64", "f32"], default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-h2d", action="store_true", help="skip the PCIe-inclusive side figure")
    ap.add_argument("--prewarm-s", type=float, default=0.5,
                    help="untimed launches before the warm-up steps (GPU clock ramp)")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "traffic.json"))
    ap.add_argument("--layout", choices=["auto", "batch", "tile64", "bucketed", "padded"],
                    default="auto",
                    help="lft/config3: block layout (auto: tile64 for the config-3 small-s "
                         "shape, batch-major otherwise); config5: shape-bucketed (auto) or "
                         "padded to s=13")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: gloo + CPU tensors + the oracle stand-in of tests/ (a "
                         "rehearsal of the rank/shard/gather path, never a measurement)")
    ap.add_argument("--dry-out", "--gather-out", dest="dry_out", default=None,
                    help="rank 0 writes the gathered (T*, J*) here (.npz); --dry-run or N > 1")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="N > 1: nccl (RCCL over xGMI, one rank per GPU; the default and the "
                         "driver's) or gloo: the real kernels with the collectives through the "
                         "host, every rank on device LOCAL_RANK mod the visible devices -- a "
                         "rehearsal of this path on a one-GPU box, never a scaling measurement")
    ap.add_argument("--event-every", type=int, default=0,
                    help="HIP event pair around every k-th timed step for kernel_ms (0: "
                         "K // 256, at least 1; 1: every step)")
    ap.add_argument("--no-alt", action="store_true",
                    help="skip the side timing of the other layout (profiling passes)")
    ap.add_argument("--no-anchor", action="store_true",
                    help="N=1 lft: skip the config-4 anchors (the 32,768-problem shard and the "
                         "262,144-problem global batch on one GPU)")
    ap.add_argument("--rho-reg", type=float, default=1e-12,
                    help="select_gains: the terminal/stage regulariser of the augmented "
                         "builders (the reference's default 1e-12, augmented.py:14, 64)")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak",
                    help="weak (default): --batch problems per GPU; strong: a fixed global "
                         "batch (--global-batch) sharded over the N GPUs")
    ap.add_argument("--global-batch", type=int, default=None,
                    help="--scaling strong: problems over all GPUs (default: 8 x the "
                         "workload's per-GPU size; lft: config 4's 262,144)")
    args = ap.parse_args(argv)
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")

    from time_opt_ilqr_amd import distributed as hd
    launched = "WORLD_SIZE" in os.environ
    if not launched and args.gpus > 1:
        sys.exit(_self_launch(args, argv))
    rank, world, local = hd.env_rank_world()
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr, flush=True)
        sys.exit(2)

    import torch
    import torch.distributed as dist
    dry = args.dry_run
    gloo = args.dist_backend == "gloo"
    if not dry and not gloo and torch.cuda.device_count() < world:
        print(f"bench.py: {world} ranks but {torch.cuda.device_count()} HIP device(s) visible",
              file=sys.stderr, flush=True)
        sys.exit(2)
    wl = args.workload
    # workload defaults (BASELINE.json configs)
    dflt = {"lft": (4096 if world == 1 else 32768, 13, 4, 100, "f64"),
            "config3": (65536, 5, 1, 200, "f32"),
            "config5": (16384, 13, 4, 128, "f32"),
            "select_gains": (4096, 13, 4, 100, "f64"),
            "bruteforce": (4096, 13, 4, 100, "f64")}[wl]
    if args.steps is None:  # ~2-5 s of timed GPU work at N = 1 (config 2: 10,000 x 0.48 ms)
        args.steps = 20 if world > 1 else {"lft": 10000, "config3": 5000, "config5": 3000,
                                           "select_gains": 10000, "bruteforce": 300}[wl]
    args.batch_given = args.batch
    args.batch = args.batch or dflt[0]
    args.s = args.s or dflt[1]
    args.m = args.m or dflt[2]
    args.N = args.N or dflt[3]
    args.dtype = args.dtype or dflt[4]
    if wl == "config3":
        args.t_min = min(args.t_min, 20)
    if dry:
        if world > 1:
            dist.init_process_group("gloo")
        dev = torch.device("cpu")
    else:
        # gloo rehearsal: ranks share the visible devices (local mod count)
        ldev = local % max(torch.cuda.device_count(), 1) if gloo else local
        if world > 1:
            torch.cuda.set_device(ldev)
            if gloo:
                dist.init_process_group("gloo")
            else:
                dist.init_process_group("nccl", device_id=torch.device("cuda", ldev))
        dev = torch.device("cuda", ldev if world > 1 else 0)
        if rank == 0:
            from time_opt_ilqr_amd import build as hop_build
            hop_build.build(verbose=False)
    if world > 1:
        dist.barrier()

    def sync():
        if not dry:
            torch.cuda.synchronize()

    def event():
        if dry:
            class _Ev:  # wall clock stands in for HIP events in the rehearsal
                def record(self):
                    self.t = time.perf_counter()

                def elapsed_time(self, other):
                    return (other.t - self.t) * 1e3
            return _Ev()
        return torch.cuda.Event(enable_timing=True)

    strong = args.scaling == "strong"
    if strong:  # config 4: a fixed global batch over N GPUs
        if args.global_batch is not None:
            total_b = args.global_batch
        elif dry:  # the rehearsal's stand-in problems are slow: --batch per GPU
            total_b = args.batch * world
        else:  # lft: 8 x 32,768 = 262,144 (BASELINE config 4)
            total_b = 8 * (32768 if wl == "lft" else dflt[0])
        if total_b < 1:
            raise SystemExit("bench.py: --global-batch must be >= 1")
    else:
        total_b = args.batch * world
    lo, hi = hd.shard_bounds(total_b, rank, world)
    Bn = hi - lo  # this rank's problems (weak: args.batch on every rank)
    launch, info = (_dry_workload if dry else WORKLOADS[wl])(args, world, lo, hi, dev)
    s, m, N = info["s"], info["m"], info["N"]

    def step():
        r = launch()
        if world > 1:
            hd.gather_selection(r.t_star, r.j_star, total_b)
        return r

    gathered = None

    # DVFS pre-warm: ~1 ms launches leave the chip below its steady clock for
    # the first ~30 launches (measured: 3 warm-up steps read 13 % slow), so spin
    # untimed launches for >= prewarm_s before the W warm-up steps.  The timed
    # region below is unchanged: exactly K full steps.
    prewarm = 0
    t_pw = time.perf_counter()
    while time.perf_counter() - t_pw < args.prewarm_s:
        for _ in range(8):  # local launches only: ranks may differ in count, no collective
            launch()
            prewarm += 1
        sync()
    for _ in range(args.warmup):
        step()
    sync()
    K = args.steps
    # HIP events on the stream the kernels are launched on (engine launches on
    # torch's current stream), around every `every`-th step of the timed region: an
    # event pair on every step costs ~0.9 % of the step (tools/ab_step_events.py,
    # profiles/r06_step_events.json), a sample of >= 256 steps averages the same
    every = max(1, K // 256) if args.event_every <= 0 else args.event_every
    ev = [(event(), event()) for _ in range(0, K, every)]
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(K):
        if i % every == 0:
            ev[i // every][0].record()
            r = launch()
            ev[i // every][1].record()
        else:
            r = launch()
        if world > 1:
            gathered = hd.gather_selection(r.t_star, r.j_star, total_b)
    sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / len(ev)
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        hd.all_reduce_max(t)
        elapsed, kern_ms = float(t[0]), float(t[1])
    if gathered is None:
        gathered = (r.t_star, r.j_star)
    if "flops_fn" in info:  # counts that depend on the selected horizons (mean T*)
        tbar = float(r.t_star.double().mean().item()) if r.t_star.numel() else 0.0
        info["flops"], info["executed"] = info["flops_fn"](tbar), info["executed_fn"](tbar)
        info["t_star_mean"] = tbar
    status_ok = int(r.status.abs().sum().item()) == 0 and bool(torch.isfinite(r.J).all())
    if hasattr(r, "riccati_status"):
        status_ok = status_ok and int(r.riccati_status.abs().sum().item()) == 0
    # every rank's shard must be clean, not only rank 0's
    if world > 1:
        ok = torch.tensor([0 if status_ok else 1], dtype=torch.int32, device=dev)
        hd.all_reduce_max(ok)
        status_ok = int(ok.item()) == 0
    if dry:
        if rank == 0 and args.dry_out:
            import numpy as np
            np.savez(args.dry_out, t_star=gathered[0].cpu().numpy(),
                     j_star=gathered[1].cpu().numpy())
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "steps": K,
                              "ms_per_step": elapsed / K * 1e3, "scaling": args.scaling,
                              "config": {"batch_per_gpu": Bn, "global_batch": total_b,
                                         "scaling": args.scaling,
                                         "parallelism": f"dp{world}"},
                              "status_ok": status_ok}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    if rank == 0 and args.dry_out and world > 1:  # the gathered selection (tests)
        import numpy as np
        np.savez(args.dry_out, t_star=gathered[0].cpu().numpy(), j_star=gathered[1].cpu().numpy())

    # the config-4-shard anchor at N=1: the per-GPU batch of the N>1 lines (32,768),
    # so a 1->N curve can compare equal per-GPU work (a side figure, not `value`)
    # and the config-4 global batch (262,144) on one GPU: the N = 1 point of the
    # strong-scaling curve (`--scaling strong --gpus N` shards that same batch)
    anchor = anchor_g = None
    if (rank == 0 and world == 1 and wl == "lft" and Bn != 32768 and not args.no_anchor
            and args.batch_given is None and not strong):
        def time_batch(nb, ka):
            launch_a, _ = WORKLOADS[wl](args_with_batch(args, nb), 1, 0, nb, dev)
            for _ in range(2):
                launch_a()
            sync()
            ta = time.perf_counter()
            for _ in range(ka):
                ra = launch_a()
            sync()
            ms_a = (time.perf_counter() - ta) / ka * 1e3
            ok_a = int(ra.status.abs().sum().item()) == 0
            del launch_a, ra
            torch.cuda.empty_cache()
            return ms_a, ok_a

        ka = min(max(3, K // 4), 50)
        ms_a, ok_a = time_batch(32768, ka)
        anchor = {"workload": "config 4 shard: LFT sweep + fused argmin (32,768 problems on "
                  "one GPU, the per-GPU batch of the N>1 weak-scaling lines)",
                  "batch_per_gpu": 32768, "steps": ka, "ms_per_step": ms_a,
                  "value": 32768 / ms_a * 1e3, "unit": "sweeps/s", "status_ok": ok_a}
        kg = min(ka, 10)
        ms_g, ok_g = time_batch(262144, kg)
        anchor_g = {"workload": "config 4 global batch: LFT sweep + fused argmin (262,144 "
                    "problems on one GPU, the N = 1 point of --scaling strong)",
                    "global_batch": 262144, "steps": kg, "ms_per_step": ms_g,
                    "value": 262144 / ms_g * 1e3, "unit": "sweeps/s", "scaling": "strong",
                    "status_ok": ok_g}

    # PCIe-inclusive side figure (never `value`): the step's inputs start in pinned
    # host memory and are copied H2D inside the timed region
    h2d = None
    if rank == 0 and not args.no_h2d and info["host"] is not None:
        dev_in = info["host"]
        pinned = [t.cpu().pin_memory() for t in dev_in]
        reps = 3
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(reps):
            for d_, h_ in zip(dev_in, pinned):
                d_.copy_(h_, non_blocking=True)
            launch()
        torch.cuda.synchronize()
        h2d_s = (time.perf_counter() - t1) / reps
        nbytes = sum(t.numel() * t.element_size() for t in pinned)
        h2d = {"value": (hi - lo) / h2d_s, "unit": "sweeps/s", "ms_per_step": h2d_s * 1e3,
               "h2d_bytes_per_step": nbytes, "note": "inputs copied from pinned host memory "
               "each step (PCIe-inclusive); not the headline value"}
        del pinned

    # side figures: the select from the raw linearisation (config 3: tile64 cart-pole;
    # config 2: batch-major quadrotor)
    side_fig = None
    if rank == 0 and info.get("side") is not None and not args.no_alt:
        sd = info["side"]
        side_fig = {}
        for key, fn in sd["fns"].items():
            r_ = fn()
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 10
            fin = torch.isfinite(r_.J).all(dim=1)
            side_fig[key] = {"ms": ms, "sweeps_per_s": (hi - lo) / (ms * 1e-3),
                             "status_ok": bool(fin.all() and (r_.status == 0).all()),
                             "problems_status_ok": int(((r_.status == 0) & fin).sum().item())}
        sel = side_fig.get(sd["select_key"])
        if sel is not None:
            bps = sd["select_bytes_per_sweep"]
            sel["alg_bytes_per_sweep"] = bps
            sel["hbm_frac"] = bps * (hi - lo) / (sel["ms"] * 1e-3) / 1e9 / PEAK_HBM_GBS
        side_fig["note"] = sd["note"]
        side_fig = (sd["name"], side_fig)
        info["side"] = None

    # side figure: fp64 s = 5 augmented blocks (the drop-in's path at the cart-pole shape)
    s5_aug = None
    if (rank == 0 and world == 1 and wl == "lft" and (args.s, args.m, args.dtype) == (13, 4, "f64")
            and not args.no_alt):
        s5_aug = _s5_aug_side(dev)

    # side figure: the same sweep on batch-major blocks (tile64 runs only)
    alt_ms = None
    if rank == 0 and info.get("alt") is not None and not args.no_alt:
        ea = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(5)]
        info["alt"]()
        for a_, b_ in ea:
            a_.record()
            info["alt"]()
            b_.record()
        torch.cuda.synchronize()
        alt_ms = sum(a_.elapsed_time(b_) for a_, b_ in ea) / len(ea)

    if rank == 0:
        total = total_b * K
        value = total / elapsed
        per_launch = hi - lo
        if info["bound"] == "hbm":
            achieved = info["bytes"] * per_launch / (kern_ms * 1e-3) / 1e9
            peak, unit = PEAK_HBM_GBS, "GB/s"
        else:
            achieved = info["flops"] * per_launch / (kern_ms * 1e-3) / 1e12
            peak = PEAK_F64_TFLOPS if info["bound"] == "fp64" else PEAK_F32_TFLOPS
            unit = "TFLOP/s"
        traffic = None
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            key = f"{wl}_s{s}_m{m}_N{N}_B{per_launch}_{args.dtype}" + ("_tile64" if info.get("layout") == "tile64" else "")
            if key in tj:
                traffic = tj[key]["hbm_bytes_per_launch"]
        except (OSError, ValueError, KeyError):
            traffic = None
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(s, m, N, bruteforce=wl == "bruteforce")
            if wl == "select_gains":
                cpu["note"] = "LFT sweep only (the Riccati gains are not in the CPU sample)"
        roof = {"bound": info["bound"], "achieved": achieved, "peak": peak, "unit": unit,
                "frac": achieved / peak, "traffic": traffic, "kernel": info["kernel"],
                "kernel_ms": kern_ms, "kernel_ms_samples": len(ev),
                "flops_per_sweep": info["flops"],
                "alg_bytes_per_sweep": info["bytes"]}
        if info["executed"] and info["bound"] != "hbm":
            ex = info["executed"] * per_launch / (kern_ms * 1e-3) / 1e12
            roof.update(executed_flops_per_sweep=info["executed"], executed_tflops=ex,
                        executed_frac=ex / peak)
        elif info["executed"]:  # HBM-bound: the executed arithmetic beside the byte roofline
            ex = info["executed"] * per_launch / (kern_ms * 1e-3) / 1e12
            pk = PEAK_F32_TFLOPS if args.dtype == "f32" else PEAK_F64_TFLOPS
            roof.update(executed_flops_per_sweep=info["executed"], executed_tflops=ex,
                        executed_frac_of_compute_peak=ex / pk)
        if "t_star_mean" in info:
            roof["t_star_mean"] = info["t_star_mean"]
        if args.dtype == "f32" and info["bound"] == "fp64":
            roof["arithmetic"] = "f64 (fp32 blocks in HBM/LDS)"
        if info["bound"] != "hbm":
            roof["hbm_gbs"] = info["bytes"] * per_launch / (kern_ms * 1e-3) / 1e9
        if alt_ms is not None and wl == "config5":
            roof["padded_s13_ms"] = alt_ms
            roof["padded_s13_frac"] = (info["flops"] * per_launch / (alt_ms * 1e-3) / 1e12
                                       / peak)
        elif alt_ms is not None:
            roof["batch_major_kernel_ms"] = alt_ms
            roof["batch_major_frac"] = (info["bytes"] * per_launch / (alt_ms * 1e-3) / 1e9
                                        / PEAK_HBM_GBS)
        names = {"lft": ("config 4: LFT sweep + fused argmin, a fixed global batch sharded "
                         "over the GPUs" if strong else
                         "config 2: LFT sweep + fused argmin" if world == 1 and Bn != 32768
                         else "config 4 shard: LFT sweep + fused argmin"),
                 "config3": "config 3: LFT sweep + fused argmin (small-s kernel)",
                 "config5": "config 5: mixed Segway/Cartpole/Quadrotor (i mod 3), "
                            "LFT sweep + fused argmin",
                 "select_gains": "select (in-kernel augmentation + LFT + argmin) + truncated "
                                 "Riccati gains at each T* (solver.py:581-597)",
                 "bruteforce": "baseline1 select: brute-force J curve (T_max = N Riccati "
                               "sweeps per problem, solver.py:293-358) + argmin"}
        line = {
            "metric": baseline_metric(),
            "value": value,
            "unit": "sweeps/s" if wl not in ("select_gains", "bruteforce") else "problems/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "prewarm_launches": prewarm,
            "ms_per_step": elapsed / K * 1e3,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (device RNG, well-conditioned SPD blocks; SURVEY.md 8(d))",
            "config": {"workload": f"{names[wl]}, s={s} m={m} N={N}",
                       "batch_per_gpu": Bn, "global_batch": total_b,
                       "scaling": args.scaling, "s": s, "m": m,
                       "N": N, "t_min": info["t_min"], "t_max": info["t_max"],
                       "layout": info.get("layout", "batch-major"),
                       **({"rho_reg": info["rho_reg"]} if "rho_reg" in info else {}),
                       "parallelism": f"dp{world}",
                       **({"dist_backend": args.dist_backend} if world > 1 else {})},
            "roofline": roof,
            "cpu_baseline": cpu,
            "h2d_inclusive": h2d,
            "config4_shard_anchor": anchor,
            "config4_global_1gpu": anchor_g,
            **({side_fig[0]: side_fig[1]} if side_fig else {}),
            **({"s5_f64_aug_blocks": s5_aug} if s5_aug else {}),
            "status_ok": status_ok,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
