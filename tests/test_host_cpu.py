"""CPU: the C ABI library loads and exports every symbol of include/hop.h;
argument validation rejects bad calls before touching a device; host-side
preparation (augmented builders, wrap, terminal weight, shard plan) matches the
oracle; the product path refuses to run without a HIP device."""
import ctypes as C
import os
import re
import sys

import numpy as np
import pytest

from oracle import hop_oracle as orc

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    from time_opt_ilqr_amd import _lib, build
    build.build(verbose=False)
    return _lib.load()


def _header_functions():
    src = open(os.path.join(REPO, "include", "hop.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|size_t|const char\*)\s+(hop_\w+)\s*\(", src,
                                 flags=re.M)))


def test_header_symbols_exported(lib):
    names = _header_functions()
    assert len(names) == 40
    from time_opt_ilqr_amd import _lib
    assert sorted(_lib.SIGNATURES) == names
    for n in names:
        assert hasattr(lib, n)
    out = os.popen(f"nm -D {_lib.LIB_PATH}").read()
    for n in names:
        assert re.search(rf"\bT {n}\b", out), n
    assert lib.hop_abi_version() == 1


def test_tile64_host_side_checks(lib):
    """tile64 (include/hop.h): the element count covers whole tiles; shapes without a
    small-s kernel and debug-free misuse are rejected before any launch."""
    import ctypes as C
    assert lib.hop_tile64_elems(70, 9, 25) == 128 * 9 * 25
    assert lib.hop_tile64_elems(64, 3, 5) == 64 * 3 * 5
    assert lib.hop_tile64_elems(0, 3, 5) == 0
    assert lib.hop_tile64_elems(-1, 3, 5) == -1
    d = C.c_void_p(16)  # never dereferenced: these calls are rejected on the host
    args = lambda s, m, rbs=0: (d, d, d, d, rbs, 1, d, d, 0, 4, 10, 10, s, m, 8, 0, 0, d, d,  # noqa: E731
                                None, None, None)
    assert lib.hop_lft_sweep_tile64_f64(*args(13, 4)) == -2  # HOP_E_SIZE: s = 13
    assert b"tile64" in lib.hop_last_error()
    assert lib.hop_lft_sweep_tile64_f64(*args(6, 1)) == -2  # no small-s kernel at s = 6
    assert lib.hop_lft_sweep_tile64_f32(*args(6, 1)) == -2
    assert lib.hop_tile64_f32(d, d, 5, 2, 0, 0, None) == -1  # elems < 1


def test_options_are_explicit_and_product_build_has_no_ab_schedules(lib):
    """Test/diagnostic controls go through hop_set_options only (no environment
    variable is read by the library); a product build rejects A/B schedule numbers
    and stamps, and carries no getenv import."""
    from time_opt_ilqr_amd import _lib
    assert lib.hop_build_flags() == 0
    assert lib.hop_set_options(0, 41) == -1 and b"developer builds" in lib.hop_last_error()
    assert lib.hop_set_options(_lib.OPT_STAMPS, 0) == -1
    assert lib.hop_set_options(1 << 9, 0) == -1
    with _lib.options(force_generic=True):
        with _lib.options(traj_unfused=True, no_rerun=True):
            assert _lib.get_options() == (_lib.OPT_FORCE_GENERIC | _lib.OPT_TRAJ_UNFUSED |
                                          _lib.OPT_NO_RERUN, 0)
        assert _lib.get_options() == (_lib.OPT_FORCE_GENERIC, 0)
    assert _lib.get_options() == (0, 0)
    out = os.popen(f"nm -D {_lib.LIB_PATH}").read()
    assert not re.search(r"\bU getenv\b", out)


def test_options_are_per_host_thread(lib):
    """SURVEY.md 8(b) re-entrancy: hop_set_options from one host thread does not
    change the options another thread's launches read (thread-local state)."""
    import threading
    from time_opt_ilqr_amd import _lib
    seen, go, done = {}, threading.Barrier(2), threading.Barrier(2)

    def worker(name, kw):
        with _lib.options(**kw):
            go.wait()          # both threads hold their own setting at once
            seen[name] = _lib.get_options()
            done.wait()
        seen[name + "_after"] = _lib.get_options()

    ts = [threading.Thread(target=worker, args=("a", dict(force_generic=True))),
          threading.Thread(target=worker, args=("b", dict(reference_assoc=True, no_rerun=True)))]
    with _lib.options(force_handover=True):  # the main thread's own setting
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert _lib.get_options() == (_lib.OPT_FORCE_HANDOVER, 0)
    assert seen["a"] == (_lib.OPT_FORCE_GENERIC, 0)
    assert seen["b"] == (_lib.OPT_REFERENCE_ASSOC | _lib.OPT_NO_RERUN, 0)
    assert seen["a_after"] == seen["b_after"] == (0, 0)
    assert _lib.get_options() == (0, 0)
    assert lib.hop_cu_fallbacks() == 0  # no launch has asked for the CU count here


def test_library_is_gfx950_code_object(lib):
    from time_opt_ilqr_amd import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_argument_validation_without_gpu(lib):
    """Bad shapes are rejected on the host (no launch happens)."""
    nul = None
    rc = lib.hop_lft_sweep_f64(nul, nul, nul, nul, 0, 0, 1, nul, nul, 0, 4, 10, 10, 17, 4, 8,
                               0, 0, nul, nul, nul, nul, nul, nul, nul)
    assert rc == -2 and b"s must be" in lib.hop_last_error()
    rc = lib.hop_lft_sweep_f64(nul, nul, nul, nul, 0, 0, 1, nul, nul, 0, 4, 10, 11, 13, 4, 8,
                               0, 0, nul, nul, nul, nul, nul, nul, nul)
    assert rc == -1 and b"n_use > n_alloc" in lib.hop_last_error()
    # n_use <= 0 is the reference's empty result: accepted, nothing launched
    assert lib.hop_lft_sweep_f64(nul, nul, nul, nul, 0, 0, 1, nul, nul, 0, 4, 10, 0, 13, 4, 8,
                                 0, 0, nul, nul, nul, nul, nul, nul, nul) == 0
    rc = lib.hop_select_horizon_f64(nul, 3, 10, 5, 11, nul, nul, nul)
    assert rc == -1
    rc = lib.hop_riccati_f64(*([nul] * 4), nul, 0, nul, 0, nul, 0, nul, 0, nul, 0, nul, nul, nul,
                             nul, nul, 0.0, 0, 2, 12, 4, 10, 12, 4, *([nul] * 6), nul)
    assert rc == -1 and b"mode" in lib.hop_last_error()
    # the brute-force J curve: t_max > n_alloc is the reference's IndexError
    jc = lambda t_max, n_alloc, wrap=0: lib.hop_bruteforce_jcurve_f64(  # noqa: E731
        *([nul] * 4), nul, 0, nul, 0, nul, 0, nul, 0, nul, 0, nul, nul, nul, 1e-6, 0.0, wrap,
        3, n_alloc, 12, 4, t_max, nul, nul, nul)
    assert jc(11, 10) == -1 and b"t_max > n_alloc" in lib.hop_last_error()
    assert jc(0, 10) == -1 and b"t_max < 1" in lib.hop_last_error()
    assert jc(10, 10, 1 << 12) == -1 and b"wrap_mask" in lib.hop_last_error()
    assert jc(10, 10) == -1 and b"null pointer" in lib.hop_last_error()


def test_product_path_has_no_cpu_fallback():
    import torch
    from time_opt_ilqr_amd import HopError, engine
    A = torch.zeros((1, 2, 3, 3), dtype=torch.float64)
    with pytest.raises(HopError):
        engine.propagate(A, torch.zeros((1, 2, 3, 1), dtype=torch.float64), A,
                         torch.eye(1, dtype=torch.float64), torch.zeros(3, dtype=torch.float64), A)


def test_wrap_and_terminal_weight():
    from time_opt_ilqr_amd import utils
    e = np.array([7.0, -7.0, 3.2, np.pi])
    w = utils.wrap_error(e, [0, 1, 2, 3])
    assert np.array_equal(w, orc.wrap_angles(e, [0, 1, 2, 3]))
    for a in (2.0, np.array([1.0, 2.0]), np.array([[1.0, 0.5], [0.0, 1.0]])):
        assert np.array_equal(utils.as_terminal_weight(a, 2), orc.terminal_weight(a, 2))
    with pytest.raises(ValueError):
        utils.as_terminal_weight(np.ones(3), 2)


def test_wrap_mask():
    from time_opt_ilqr_amd.engine import wrap_mask
    assert wrap_mask([6, 7, 8], 12) == (1 << 6) | (1 << 7) | (1 << 8)
    assert wrap_mask(None, 4) == 0
    assert wrap_mask([-1], 4) == 8
    with pytest.raises(IndexError):
        wrap_mask([5], 4)


def test_shard_bounds_cover_batch():
    from time_opt_ilqr_amd.distributed import shard_bounds
    for total in (0, 1, 7, 4096, 262144, 131071):
        for world in (1, 2, 3, 8):
            spans = [shard_bounds(total, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [hi - lo for lo, hi in spans]
            assert max(sizes) - min(sizes) <= 1


def test_dpp_blocks_generated_in_sync():
    """csrc/dpp_blocks.inc is exactly what tools/gen_dpp.py produces."""
    import subprocess
    import sys
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "x.inc")
        subprocess.check_call([sys.executable, os.path.join(REPO, "tools", "gen_dpp.py"), out],
                              stdout=subprocess.DEVNULL)
        want = open(out).read()
    have = open(os.path.join(REPO, "time_opt_ilqr_amd", "csrc", "dpp_blocks.inc")).read()
    assert want == have


@pytest.mark.parametrize("n", [2, 5, 13, 16])
def test_hand_scheduled_blocks_emulated(n):
    """The whole-sweep asm blocks (SweepQ / ElimQ in dpp_blocks.inc) compute the
    offset-form negated inverse and the bordered quadratic form (CPU emulation
    of the instruction strings, tools/emu_dpp.py)."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import emu_dpp as E
    inc = open(os.path.join(REPO, "time_opt_ilqr_amd", "csrc", "dpp_blocks.inc")).read()
    rng = np.random.default_rng(n)
    M = rng.standard_normal((n, n))
    M = M @ M.T + n * np.eye(n)
    eps = 1e-9
    regs = {}
    for i in range(n):  # register i = row i, lane c = column c; diagonal offset by eps - 1
        col = rng.standard_normal(16)
        col[:n] = M[i]
        col[i] += eps - 1.0
        regs[i] = col
    regs[n] = np.ones(16)
    for j in range(7):
        regs[n + 1 + j] = np.full(16, np.nan)
    E.run(E.extract(inc, "SweepQ", n), regs)
    got = np.array([regs[i][:n] for i in range(n)])
    want = np.eye(n) - np.linalg.inv(M + eps * np.eye(n))
    assert np.abs(got - want).max() < 1e-12
    assert regs[n][0] > 0
    if n == 16:
        return  # the bordered form needs a free lane
    z = rng.standard_normal(n)
    regs = {}
    for i in range(n):
        col = rng.standard_normal(16)
        col[:n] = M[i]
        col[n] = z[i]
        regs[i] = col
    regs[n], regs[n + 1] = np.zeros(16), np.ones(16)
    for j in range(8):
        regs[n + 2 + j] = np.full(16, np.nan)
    regs[n + 10] = np.full(16, eps)
    E.run(E.extract(inc, "ElimQ", n), regs)
    q = z @ np.linalg.solve(M + eps * np.eye(n), z)
    assert abs(regs[n][n] - q) <= 1e-12 * abs(q)


@pytest.mark.parametrize("n", [2, 3, 4, 5, 6])
def test_small_dual_sweep_block_emulated(n):
    """SweepQ2<n> (the small-s row-group kernel's stage and terminal sweeps as one
    interleaved block) computes exactly what SweepQ<n> and SweepQP<n>
    compute separately, register for register (CPU emulation of the instruction
    strings, tools/emu_dpp.py), and SweepQ's part is the offset-form negated inverse."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import emu_dpp as E
    inc = open(os.path.join(REPO, "time_opt_ilqr_amd", "csrc", "dpp_blocks.inc")).read()
    rng = np.random.default_rng(40 + n)
    eps = 1e-9

    def rows(M):
        out = []
        for i in range(n):
            col = rng.standard_normal(16)
            col[:n] = M[i]
            col[i] += eps - 1.0
            out.append(col)
        return out

    def spd():
        M = rng.standard_normal((n, n))
        return M @ M.T + n * np.eye(n)
    M1, M2 = spd(), spd()
    r1, r2 = rows(M1), rows(M2)
    both = {}
    for i in range(n):
        both[i], both[n + 8 + i] = r1[i].copy(), r2[i].copy()
    both[n], both[2 * n + 8] = np.ones(16), np.ones(16)
    for j in range(7):
        both[n + 1 + j] = np.full(16, np.nan)
        both[2 * n + 9 + j] = np.full(16, np.nan)
    E.run(E.extract(inc, "SweepQ2", n), both)
    for name, r0, base, dm in (("SweepQ", r1, 0, n), ("SweepQP", r2, n + 8, 2 * n + 8)):
        sep = {i: r0[i].copy() for i in range(n)}
        sep[n] = np.ones(16)
        for j in range(7):
            sep[n + 1 + j] = np.full(16, np.nan)
        E.run(E.extract(inc, name, n), sep)
        for i in range(n):
            assert np.array_equal(both[base + i], sep[i]), (name, i)
        assert np.array_equal(both[dm], sep[n])
    got = np.array([both[i][:n] for i in range(n)])
    assert np.abs(got - (np.eye(n) - np.linalg.inv(M1 + eps * np.eye(n)))).max() < 1e-12


@pytest.mark.parametrize("n", [3, 5])
def test_small_sweeps_with_query_block_emulated(n):
    """SweepQ2ElimQ<n> (the A/B switch HOP_SMALL_QPIPE: a step's query interleaved with
    the next step's two sweeps) computes exactly SweepQ2<n> and ElimQ<n> run one after
    the other, register for register (CPU emulation, tools/emu_dpp.py)."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import emu_dpp as E
    inc = open(os.path.join(REPO, "time_opt_ilqr_amd", "csrc", "dpp_blocks.inc")).read()
    rng = np.random.default_rng(70 + n)

    def rows(off):
        M = rng.standard_normal((n, n))
        M = M @ M.T + n * np.eye(n)
        out = []
        for i in range(n):
            col = rng.standard_normal(16)
            col[:n] = M[i]
            col[i] += off
            out.append(col)
        return out
    r1, r2, q = rows(1e-9 - 1.0), rows(1e-9 - 1.0), rows(0.0)
    for col, z in zip(q, rng.standard_normal(n)):
        col[n] = z
    eps = 2.0
    both = {}
    for i in range(n):
        both[i], both[n + 8 + i], both[2 * n + 16 + i] = r1[i].copy(), r2[i].copy(), q[i].copy()
    both[n], both[2 * n + 8] = np.ones(16), np.ones(16)
    both[3 * n + 16], both[3 * n + 17] = np.zeros(16), np.ones(16)
    for j in range(7):
        both[n + 1 + j] = np.full(16, np.nan)
        both[2 * n + 9 + j] = np.full(16, np.nan)
    for j in range(8):
        both[3 * n + 18 + j] = np.full(16, np.nan)
    both[3 * n + 26] = np.full(16, eps)
    E.run(E.extract(inc, "SweepQ2ElimQ", n), both)
    two = {}
    for i in range(n):
        two[i], two[n + 8 + i] = r1[i].copy(), r2[i].copy()
    two[n], two[2 * n + 8] = np.ones(16), np.ones(16)
    for j in range(7):
        two[n + 1 + j] = np.full(16, np.nan)
        two[2 * n + 9 + j] = np.full(16, np.nan)
    E.run(E.extract(inc, "SweepQ2", n), two)
    el = {i: q[i].copy() for i in range(n)}
    el[n], el[n + 1] = np.zeros(16), np.ones(16)
    for j in range(8):
        el[n + 2 + j] = np.full(16, np.nan)
    el[n + 10] = np.full(16, eps)
    E.run(E.extract(inc, "ElimQ", n), el)
    for i in range(n):
        assert np.array_equal(both[i], two[i]) and np.array_equal(both[n + 8 + i], two[n + 8 + i])
        assert np.array_equal(both[2 * n + 16 + i], el[i])
    assert np.array_equal(both[n], two[n]) and np.array_equal(both[2 * n + 8], two[2 * n + 8])
    assert np.array_equal(both[3 * n + 16], el[n]) and np.array_equal(both[3 * n + 17], el[n + 1])


@pytest.mark.parametrize("n", [3, 13])
def test_query_ldl_block_emulated(n):
    """QueryLdl<n>: X0 = Ebar - H^T (Mt + eps I)^-1 H from the offset-form Mt
    (diag - 1 + eps), by elimination + row operations + rank-1 streams."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import emu_dpp as E
    inc = open(os.path.join(REPO, "time_opt_ilqr_amd", "csrc", "dpp_blocks.inc")).read()
    rng = np.random.default_rng(100 + n)
    M = rng.standard_normal((n, n))
    M = M @ M.T + n * np.eye(n)
    H = rng.standard_normal((n, n))
    Eb = rng.standard_normal((n, n))
    Eb = Eb + Eb.T
    eps = 1e-9
    regs = {}
    for i in range(n):
        for base, src in ((0, M), (n, H), (2 * n, Eb)):
            col = rng.standard_normal(16)
            col[:n] = src[i]
            regs[base + i] = col
        regs[i][i] += eps - 1.0
    regs[3 * n] = np.ones(16)
    for j in range(10):
        regs[3 * n + 1 + j] = np.full(16, np.nan)
    E.run(E.extract(inc, "QueryLdl", n), regs)
    got = np.array([regs[2 * n + i][:n] for i in range(n)])
    want = Eb - H.T @ np.linalg.solve(M + eps * np.eye(n), H)
    assert np.abs(got - want).max() <= 1e-12 * np.abs(want).max()
    assert regs[3 * n][0] > 0


@pytest.mark.parametrize("block", ["SweepQSym", "SweepQAB"])
def test_sweep_blocks_with_lds_reads_emulated(block):
    """SweepQSym / SweepQAB (the conditioned kernel's sweeps with LDS reads riding
    in the same asm statement) compute exactly SweepQ<13> (reads are skipped by
    the emulator; their destinations are outputs only)."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import emu_dpp as E
    inc = open(os.path.join(REPO, "time_opt_ilqr_amd", "csrc", "dpp_blocks.inc")).read()
    n = 13
    rng = np.random.default_rng(7)
    M = rng.standard_normal((n, n))
    M = M @ M.T + n * np.eye(n)
    out = []
    for name in ("SweepQ", block):
        regs = {}
        for i in range(n):
            col = np.zeros(16)
            col[:n] = M[i]
            col[i] += 1e-9 - 1.0
            regs[i] = col
        regs[n] = np.ones(16)
        for j in range(7):
            regs[n + 1 + j] = np.full(16, np.nan)
        E.run(E.extract(inc, name, n), regs)
        out.append(np.array([regs[i] for i in range(n + 1)]))
    assert np.array_equal(out[0], out[1])
    want = np.eye(n) - np.linalg.inv(M + 1e-9 * np.eye(n))
    assert np.abs(out[1][:n, :n] - want).max() < 1e-12


@pytest.mark.parametrize("n,block", [(3, "CondLdl"), (13, "CondLdl"), (13, "CondLdlN"),
                                     (13, "CondLdl2")])
def test_cond_ldl_block_emulated(n, block):
    """CondLdl<n> (the conditioned-prefix update of SchedCond): from the offset-form
    S - I and Psi = [Sigma | m] (m on lane n), stream Sigma' = Sigma - Sigma S^-1 Sigma,
    m' = m - Sigma S^-1 m on lane n, and gamma' = gamma - m^T S^-1 m on lane n of
    the extra row n."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import emu_dpp as E
    inc = open(os.path.join(REPO, "time_opt_ilqr_amd", "csrc", "dpp_blocks.inc")).read()
    rng = np.random.default_rng(200 + n)
    Sg = rng.standard_normal((n, n))
    Sg = Sg @ Sg.T
    Ek = rng.standard_normal((n, n))
    Ek = Ek @ Ek.T / n + np.eye(n)
    S = Sg + Ek
    m = rng.standard_normal(n)
    gam = -0.7
    regs = {}
    for i in range(n):
        col = rng.standard_normal(16)
        col[:n] = S[i]
        if block == "CondLdl":  # offset form; CondLdlN takes S itself
            col[i] -= 1.0
        elif block == "CondLdl2":  # the SYM2 kernel's offset 2
            col[i] -= 2.0
        regs[i] = col
        for base in (n, 2 * n):
            col = np.zeros(16)
            col[:n] = Sg[i]
            col[n] = m[i]
            regs[base + i] = col
    regs[3 * n] = np.zeros(16)
    regs[3 * n][n] = gam
    regs[3 * n + 1] = np.ones(16)
    for j in range(10):
        regs[3 * n + 2 + j] = np.full(16, np.nan)
    E.run(E.extract(inc, block, n), regs)
    X = np.array([regs[2 * n + i] for i in range(n)])
    Si = np.linalg.inv(S)
    want = Sg - Sg @ Si @ Sg
    assert np.abs(X[:, :n] - want).max() <= 1e-12 * np.abs(want).max()
    mw = m - Sg @ Si @ m
    assert np.abs(X[:, n] - mw).max() <= 1e-12 * np.abs(mw).max()
    gw = gam - m @ Si @ m
    assert abs(regs[3 * n][n] - gw) <= 1e-12 * abs(gw)
    assert regs[3 * n + 1][0] > 0


def _cond_model(A, Bm, Q, Ri, z0, QT, N):
    """NumPy model of lft_cond_kernel: the J curve by the
    conditioned prefix (Sigma, m, gamma) with the reference's jitters placed as
    Sigma + eps I (W and X0 jitters) and Sigma + X_t + eps I (Wt jitter)."""
    s = A.shape[1]
    eps = 1e-9 * np.eye(s)
    Sig, m, gam = np.zeros((s, s)), np.asarray(z0, float).copy(), 0.0
    J = np.zeros(N)
    for k in range(N):
        E, _ = orc.spd_inverse(Q[k])
        Se = Sig + eps
        Sinv = np.linalg.inv(Se + E)
        Sig1 = Se - Se @ Sinv @ Se
        m1 = m - Se @ Sinv @ m
        gam -= m @ Sinv @ m
        Sig = A[k] @ Sig1 @ A[k].T + Bm[k] @ Ri @ Bm[k].T
        m = A[k] @ m1
        X, _ = orc.spd_inverse(QT[k])
        J[k] = 0.5 * (m @ np.linalg.solve(Sig + eps + X, m) - gam)
    return J


@pytest.mark.parametrize("tag", ["s13_m4_N100", "s5_m1_N200", "s3_m1_N50", "s16_m6_N40"])
def test_conditioned_prefix_model_vs_golden(golden_dir, tag):
    """The association the fast s=13 kernel uses (z0 folded into the prefix first,
    the reference's jitters moved onto Sigma) reproduces the reference's J curves
    (golden vectors made by importing the reference) to 1e-11."""
    d = np.load(os.path.join(golden_dir, f"lft_synth_{tag}.npz"))
    s, m, N, bs, cnt = (int(d[k]) for k in ("s", "m", "N", "base_seed", "count"))
    A, Bm, Q, R, Ri, z0, QT = orc.synth_lft_batch(bs, min(cnt, 2), s, m, N)
    for b in range(min(cnt, 2)):
        r = Ri if Ri.ndim == 2 else Ri[b]
        J = _cond_model(A[b], Bm[b], Q[b], r, z0[b] if z0.ndim == 2 else z0, QT[b], N)
        assert _rel_err(J, d["J"][b]) <= 1e-11


@pytest.mark.parametrize("tag,tol", [("real_DI_N50", 1e-3), ("real_Quad_N160", 5e-2)])
def test_conditioned_prefix_model_real_captures(golden_dir, tag, tol):
    """Same model on the reference's own first/last select linearisations
    (ill-conditioned terminal blocks): same T*, J within the real-capture bars."""
    d = np.load(os.path.join(golden_dir, f"{tag}.npz"))
    for p in ("pfirst", "plast"):
        N = int(d[p + "_T_use"])
        J = _cond_model(d[p + "_A"], d[p + "_B"], d[p + "_Q"], d[p + "_R_inv"], d[p + "_z0"],
                        d[p + "_QT"], N)
        Jr = d[p + "_J"]
        assert _rel_err(J, Jr) <= tol
        lo, hi = int(d["T_min"]), min(int(d["T_max"]), N)
        assert int(np.argmin(J[lo - 1:hi])) == int(np.argmin(Jr[lo - 1:hi]))


def _cond_model_cf(p, rho, N, q_reg=1e-9):
    """NumPy model of lft_cond_cf_kernel: the conditioned prefix on the trajectory
    form with the closed-form inverses of Q_aug + eps I and QT_aug + eps I."""
    n = p["X"].shape[1]
    eps = 1e-9
    Q = np.asarray(p["Q"], float)
    P = orc.sym(orc.terminal_weight(p["alpha"], n))
    Aa, Ba, _, _, z0, Ri = orc.augment_stage(list(p["A"]), list(p["B"]), p["a_res"], p["X"],
                                             p["U"], p["xg"], p["u_ref"], Q, p["R"], p["w"],
                                             wrap_idx=p["wrap_idx"], rho_reg=rho)
    Qi = np.linalg.inv(orc.sym(Q) + (q_reg + eps) * np.eye(n))
    Pi = np.linalg.inv(P + eps * np.eye(n))
    ext = lambda M: np.pad(M, ((0, 1), (0, 1)))  # noqa: E731
    err = lambda t: orc.wrap_angles(p["X"][t] - p["xg"], p["wrap_idx"])  # noqa: E731
    s = n + 1
    Sig, m, gam = np.zeros((s, s)), z0.copy(), 0.0
    J = np.zeros(N)
    for k in range(N):
        e = err(k)
        q = Q @ e
        v = Qi @ q
        sig = float(e @ q) + 2.0 * float(p["w"]) + rho + eps - q @ v
        vp = np.append(v, -1.0)
        E = ext(Qi) + np.outer(vp, vp) / sig
        Se = Sig + eps * np.eye(s)
        Si = np.linalg.inv(Se + E)
        Sig1, m1 = Se - Se @ Si @ Se, m - Se @ Si @ m
        gam -= m @ Si @ m
        Sig = Aa[k] @ Sig1 @ Aa[k].T + Ba[k] @ Ri @ Ba[k].T
        m = Aa[k] @ m1
        e1 = err(k + 1)
        u = e1 - eps * (Pi @ e1)
        sT = rho + eps + eps * float(e1 @ u)
        up = np.append(u, -1.0)
        X = ext(Pi) + np.outer(up, up) / sT
        J[k] = 0.5 * (m @ np.linalg.solve(Sig + eps * np.eye(s) + X, m) - gam)
    return J


@pytest.mark.parametrize("seed", [1, 2])
def test_closed_form_traj_model_vs_reference(seed):
    """Closed-form stage inverses (lft_cond_cf_kernel's arithmetic) on the
    trajectory form: 1e-11 of the reference association (oracle builders +
    propagator) at rho_reg = 1."""
    p = orc.synth_traj_problem(seed, 12, 4, 60)
    Aa, Ba, Qa, _, z0, Ri = orc.augment_stage(list(p["A"]), list(p["B"]), p["a_res"], p["X"],
                                              p["U"], p["xg"], p["u_ref"], p["Q"], p["R"], p["w"],
                                              wrap_idx=p["wrap_idx"], rho_reg=1.0)
    QT = orc.augment_terminal(p["X"], p["xg"], p["alpha"], wrap_idx=p["wrap_idx"], rho_reg=1.0)
    Jref = orc.lft_sweep(Aa, Ba, Qa, Ri, z0, QT)["J"]
    assert _rel_err(_cond_model_cf(p, 1.0, 60), Jref) <= 1e-11


@pytest.mark.parametrize("tag,tol", [("traj_real_DI_N50", 1e-4), ("traj_real_Quad_N160", 1e-3)])
def test_closed_form_traj_model_real_captures(golden_dir, tag, tol):
    """Same model on the reference's own first-select linearisations (rho_reg =
    1e-12, ill-conditioned terminal blocks): same T*, J within 5e-6 (DI) / 8e-5
    (Quadrotor) measured, asserted at 1e-4 / 1e-3."""
    d = np.load(os.path.join(golden_dir, f"{tag}.npz"))
    p = {k: d[k] for k in d.files}
    p["wrap_idx"] = list(d["wrap_idx"])
    N = int(d["N"])
    J = _cond_model_cf(p, 1e-12, N)
    assert _rel_err(J, d["J"]) <= tol
    lo, hi = int(d["T_min"]), min(int(d["T_max"]), N)
    assert int(np.argmin(J[lo - 1:hi])) == int(np.argmin(d["J"][lo - 1:hi]))


@pytest.fixture(scope="module")
def small_host(tmp_path_factory):
    """g++ build of csrc/small_math.hpp (the small-s kernel's per-problem math)."""
    import subprocess
    d = tmp_path_factory.mktemp("small")
    so = str(d / "libsmall_host.so")
    src = os.path.join(REPO, "time_opt_ilqr_amd", "csrc", "small_host.cpp")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-DHOP_HD=", src, "-o", so])
    return C.CDLL(so)


@pytest.mark.parametrize("tag,dt", [("s5_m1_N200", np.float64), ("s3_m1_N50", np.float64),
                                    ("s5_m1_N200", np.float32)])
def test_small_cond_math_vs_golden(small_host, golden_dir, tag, dt):
    """The conditioned-prefix arithmetic of the small-s COND kernels (small_math.hpp
    cond_*), run on the CPU: the reference's J curves and T*, nothing handed over."""
    d = np.load(os.path.join(golden_dir, f"lft_synth_{tag}.npz"))
    s, m, N, bs, cnt = (int(d[k]) for k in ("s", "m", "N", "base_seed", "count"))
    A, Bm, Q, R, Ri, z0, QT = orc.synth_lft_batch(bs, cnt, s, m, N)
    cast = lambda x: np.ascontiguousarray(x, dtype=dt)  # noqa: E731
    J = np.zeros((cnt, N), dt)
    st = np.zeros(cnt, np.int32)
    ts = np.zeros(cnt, np.int32)
    fn = (small_host.small_host_cond_sweep_f64 if dt == np.float64
          else small_host.small_host_cond_sweep_f32)
    args = [cast(x) for x in (A, Bm, Q, Ri, QT, np.broadcast_to(z0[0], (cnt, s)))]
    p = lambda x: x.ctypes.data_as(C.c_void_p)  # noqa: E731
    rc = fn(*[p(x) for x in args], C.c_int64(cnt), N, s, m, int(d["T_min"]), int(d["T_max"]),
            p(J), p(st), p(ts))
    assert rc == 0
    tol = 1e-10 if dt == np.float64 else 2e-3
    assert _rel_err(J, d["J"]) <= tol
    assert (st == 0).all()
    if dt == np.float64:
        assert ts.tolist() == d["T_star"].tolist()


@pytest.mark.parametrize("name", ["segway", "cartpole", "di"])
def test_small_cond_math_real_linearisations_vs_50_digit(small_host, golden_dir, name):
    """The small-s conditioned arithmetic (small_math.hpp cond_step + cond_query, the
    code the COND kernels run) on real linearisations at rho_reg = 1e-12
    (tests/golden/real_lin_hp.npz): within 1e-9 of the 50-digit evaluation of the
    reference's algorithm and the same T*, where the fp64 NumPy reference is 5e-6 ..
    6 away and picks a different T* on one cart-pole problem; the round-3 query
    (cond_query_direct: the elimination of Sigma_eps + X_t with X_t formed) is
    worse than the new one on every problem."""
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    import make_hp as mh
    d = np.load(os.path.join(golden_dir, "real_lin_hp.npz"))
    sid, N, T_min, T_max = mh.CASES[name][:4]
    p = lambda x: x.ctypes.data_as(C.c_void_p)  # noqa: E731
    win = slice(T_min - 1, T_max)
    for i in range(int(d[f"{name}_count"])):
        t = f"{name}_p{i}"
        prob = {k: d[f"{t}_{k}"] for k in ("A", "B", "a_res", "X", "U")}
        Aa, Ba, Qa, Ri, z0, QT = (np.ascontiguousarray(x, dtype=np.float64)
                                  for x in mh.blocks(name, prob))
        s, m = Aa.shape[-1], Ba.shape[-1]
        Jh = d[f"{t}_J_hp"]
        errs = []
        for fn in (small_host.small_host_cond_sweep_f64, small_host.small_host_cond_sweep_direct_f64):
            J = np.zeros((1, N))
            st, ts = np.zeros(1, np.int32), np.zeros(1, np.int32)
            assert fn(p(Aa), p(Ba), p(Qa), p(Ri), p(QT), p(np.ascontiguousarray(z0)), C.c_int64(1),
                      N, s, m, T_min, T_max, p(J), p(st), p(ts)) == 0
            errs.append(float(np.max(np.abs(J[0, win] - Jh[win]) / np.abs(Jh[win]))))
            if len(errs) == 1:
                assert st[0] == 0, t
                assert int(ts[0]) == int(np.argmin(Jh[win]) + T_min), t
        assert errs[0] <= 1e-9, (t, errs)
        assert errs[0] <= errs[1], (t, errs)


@pytest.mark.parametrize("tag,dt", [("s5_m1_N200", np.float64), ("s3_m1_N50", np.float64),
                                    ("s5_m1_N200", np.float32)])
def test_small_kernel_math_vs_golden(small_host, golden_dir, tag, dt):
    """The packed-symmetric sweep-operator arithmetic of lft_small.hip, run on the
    CPU, reproduces the reference's J curves and T* (golden vectors)."""
    d = np.load(os.path.join(golden_dir, f"lft_synth_{tag}.npz"))
    s, m, N, bs, cnt = (int(d[k]) for k in ("s", "m", "N", "base_seed", "count"))
    A, Bm, Q, R, Ri, z0, QT = orc.synth_lft_batch(bs, cnt, s, m, N)
    cast = lambda x: np.ascontiguousarray(x, dtype=dt)  # noqa: E731
    J = np.zeros((cnt, N), dt)
    st = np.zeros(cnt, np.int32)
    ts = np.zeros(cnt, np.int32)
    fn = small_host.small_host_sweep_f64 if dt == np.float64 else small_host.small_host_sweep_f32
    args = [cast(x) for x in (A, Bm, Q, Ri, QT, np.broadcast_to(z0[0], (cnt, s)))]
    p = lambda x: x.ctypes.data_as(C.c_void_p)  # noqa: E731
    rc = fn(*[p(x) for x in args], C.c_int64(cnt), N, s, m, 8, int(d["T_min"]), int(d["T_max"]),
            p(J), p(st), p(ts))
    assert rc == 0
    tol = 1e-10 if dt == np.float64 else 2e-3
    assert _rel_err(J, d["J"]) <= tol
    assert (st == 0).all()
    if dt == np.float64:
        assert ts.tolist() == d["T_star"].tolist()


def _rel_err(got, ref):
    got, ref = np.asarray(got, float), np.asarray(ref, float)
    return float(np.max(np.abs(got - ref)) / max(np.max(np.abs(ref)), 1e-300))


@pytest.mark.parametrize("dt", [np.float64, np.float32])
def test_wrap_angle_matches_python_remainder(small_host, dt):
    """csrc/wrap.hpp (used by every kernel) == angle_normalize (utils.py:127-128):
    (a + pi) % (2 pi) - pi with Python's float remainder, bit for bit in fp64."""
    import math
    rng = np.random.default_rng(3)
    two_pi = 2.0 * math.pi
    k = np.arange(-40, 41, dtype=np.float64)
    vals = np.concatenate([
        rng.uniform(-50, 50, 20000), rng.uniform(-1e6, 1e6, 2000), rng.standard_normal(2000),
        k * two_pi - math.pi, k * two_pi + math.pi, k * two_pi,
        np.nextafter(k * two_pi - math.pi, np.inf), np.nextafter(k * two_pi - math.pi, -np.inf),
        np.array([0.0, -0.0, math.pi, -math.pi, 1e-300, -1e-300, 3 * math.pi, -3 * math.pi])])
    vals = np.ascontiguousarray(vals.astype(dt))
    out = np.zeros_like(vals)
    fn = small_host.small_host_wrap_f64 if dt == np.float64 else small_host.small_host_wrap_f32
    p = lambda x: x.ctypes.data_as(C.c_void_p)  # noqa: E731
    fn(p(vals), p(out), C.c_int64(len(vals)))
    if dt == np.float64:
        ref = np.array([(float(a) + math.pi) % (2.0 * math.pi) - math.pi for a in vals])
        assert np.array_equal(out.view(np.uint64), ref.view(np.uint64))
    else:  # same formula in fp32 (np.float32 remainder has the same semantics)
        pi32, tp32 = np.float32(math.pi), np.float32(2.0 * math.pi)
        ref = np.remainder(vals + pi32, tp32) - pi32
        assert np.array_equal(out, ref.astype(np.float32))


def test_traj_entry_validation_and_workspace_query(lib):
    """hop_lft_sweep_traj_* / hop_augment_* reject bad shapes on the host; the
    workspace query is 0 exactly for the shapes with an in-kernel builder."""
    nul = None
    traj_args = [nul] * 6 + [0, nul, 0, nul, 0, nul, 0, nul, 0, nul, nul, nul]
    # n = 16 (s = 17) is over the 16-lane limit
    rc = lib.hop_lft_sweep_traj_f64(*traj_args, 0, 1e-9, 1e-12, nul, 0, 4, 10, 10, 16, 4, 8, 0, 0,
                                    nul, nul, nul, nul, nul, 0, nul)
    assert rc == -2 and b"n must be" in lib.hop_last_error()
    rc = lib.hop_lft_sweep_traj_f64(*traj_args, 0, 1e-9, 1e-12, nul, 0, 4, 10, 11, 12, 4, 8, 0, 0,
                                    nul, nul, nul, nul, nul, 0, nul)
    assert rc == -1 and b"n_use > n_alloc" in lib.hop_last_error()
    rc = lib.hop_augment_f64(*traj_args, 1 << 12, 1e-9, 1e-12, 4, 10, 10, 12, 4,
                             nul, nul, nul, nul, nul, nul)
    assert rc == -1  # null inputs (checked before the wrap mask)
    ws = lib.hop_lft_sweep_traj_workspace_bytes
    assert ws(4096, 100, 12, 4, 8, 0) == 0          # Quadrotor shape, fp64: fused
    assert ws(65536, 200, 4, 1, 4, 0) == 0          # Cartpole shape, fp32: fused (small s)
    assert ws(16385, 200, 4, 1, 8, 0) == 0          # fp64 above kSmallRowGroupMax: fused
    assert ws(16384, 200, 4, 1, 8, 0) >= 8 * 16384 * 200 * (3 * 25 + 5)  # augment + row groups
    from time_opt_ilqr_amd import _lib
    with _lib.options(small_lane=True):
        assert ws(4096, 200, 4, 1, 8, 0) == 0       # HOP_OPT_SMALL_LANE: the fused lane kernel
    assert ws(4096, 100, 12, 4, 8, 1) > 0           # extra_stage_cost: builder + sweep
    s, m, steps = 16, 6, 7 * 30
    need = ws(7, 30, 15, 6, 8, 0)
    assert need >= 8 * steps * (3 * s * s + s * m)
    assert ws(0, 30, 15, 6, 8, 0) == 0


def test_block_decoupled_packing_matches_oracle_embedding():
    """packing.pack_mixed (torch, device-agnostic plumbing) builds exactly the
    oracle's block-decoupled embedding, and the embedded problems keep their
    true-shape J."""
    import torch
    from time_opt_ilqr_amd.packing import pack_mixed
    N = 9
    probs = [orc.synth_config5_problem(300, i, N) for i in range(7)]
    groups = []
    for g in range(3):
        mem = [p for i, p in enumerate(probs) if i % 3 == g]
        t = lambda j: torch.as_tensor(np.stack([p[j] for p in mem]))  # noqa: E731
        groups.append((t(0), t(1), t(2), t(4), torch.as_tensor(mem[0][5]), t(6)))
    mb = pack_mixed(groups, np.arange(7) % 3, 13, 4)
    for i, p in enumerate(probs):
        A, Bm, Q, R, Ri, z0, QT = p
        ref = orc.embed_block_decoupled(A, Bm, Q, Ri, z0, QT, 13, 4)
        got = (mb.A[i], mb.B[i], mb.Q[i], mb.R_inv[i], mb.z0[i], mb.QT[i])
        for a, b in zip(got, ref):
            assert np.array_equal(a.numpy(), b)
        J0 = orc.lft_sweep(A, Bm, Q, Ri, z0, QT)["J"]
        J1 = orc.lft_sweep(*ref)["J"]
        assert np.max(np.abs(J1 - J0) / J0) <= 1e-12
    assert mb.true_s.tolist() == [5, 5, 13, 5, 5, 13, 5]
    assert mb.true_m.tolist() == [1, 1, 4, 1, 1, 4, 1]


def test_merge_by_shape_regroups_kinds_in_slot_order():
    """packing.merge_by_shape (config 5 by shape bucket): kinds sharing (s, m) merge
    into one group whose members follow the batch slots; other kinds pass through."""
    import torch
    from time_opt_ilqr_amd.packing import merge_by_shape
    N = 3

    def kind(b, s, m, base):
        A = base + torch.arange(b, dtype=torch.float64).reshape(b, 1, 1, 1).expand(b, N, s, s)
        return (A.clone(), torch.zeros(b, N, s, m), A.clone(), torch.eye(m),
                torch.full((s,), base), A.clone())

    groups = [kind(4, 5, 1, 100.0), kind(4, 5, 1, 200.0), kind(3, 13, 4, 300.0)]
    order = torch.tensor([0, 1, 2, 0, 1, 2, 0, 1, 2, 0, 1])
    sg, so = merge_by_shape(groups, order)
    assert so.tolist() == [0, 0, 1, 0, 0, 1, 0, 0, 1, 0, 0]
    assert len(sg) == 2 and sg[1][0] is groups[2][0]
    A5 = sg[0][0][:, 0, 0, 0].tolist()
    assert A5 == [100.0, 200.0, 101.0, 201.0, 102.0, 202.0, 103.0, 203.0]
    assert sg[0][3].shape == (1, 1)  # equal shared R_inv stays shared
    assert sg[0][4].shape == (8, 5)  # different shared z0 expanded per member
    assert sg[0][4][:, 0].tolist() == [100.0, 200.0] * 4


def test_tile64_descriptor_checks_shape():
    """engine.Tile64.check: the kernels read whole tiles, so a data tensor that is not
    exactly [ceil(batch/64), N, rows*cols, 64] is rejected before any launch."""
    import torch
    from time_opt_ilqr_amd.engine import Tile64
    assert Tile64(torch.zeros(2, 3, 25, 64), 70, 5, 5).check().shape == (70, 3, 5, 5)
    for bad in (torch.zeros(1, 3, 25, 64), torch.zeros(2, 3, 24, 64), torch.zeros(2, 3, 25, 32),
                torch.zeros(2, 3, 25, 64).transpose(0, 1)):
        with pytest.raises(ValueError):
            Tile64(bad, 70, 5, 5).check()


def test_bench_bruteforce_counts_and_cpu_worker():
    """bench.py --workload bruteforce: the FLOP count is the mode-1 Riccati count summed
    over the horizons, and its CPU leg (the oracle's bruteforce_J on the workload's
    distribution) equals the J curve of T_max separate oracle value sweeps"""
    import bench
    n, m, N = 4, 1, 6
    assert sum(bench.riccati_flops(n, m, T, 1) for T in range(1, N + 1)) == \
        bench.riccati_flops(n, m, 1, 1) * N * (N + 1) // 2
    cnt, secs = bench._cpu_worker_bf((3, 1, n, m, N))
    assert cnt == 1 and secs >= 0.0
    A, Bm, X, U, xg, ur, Q, R, Qf = bench.synth_riccati_problem(3, n, m, N)
    J = orc.bruteforce_J(list(A), list(Bm), X, U, xg, ur, Q, R, Qf, 0.5, N)
    for T in (1, N):
        _, _, V0, _, _ = orc.riccati_expand(list(A), list(Bm), X, U, xg, ur, Q, R, Qf, T, 0,
                                            lm_lambda=1e-6, w_stage=0.5, reg_max_tries=1)
        assert J[T - 1] == V0[0]


def test_predict_eps_block_emulated():
    """PredictEps<13> (the SYM2 conditioned kernel's predict): T = [Sigma' | m'] A~^T
    with A~^T's row 13 = e_13, the eps I rows read from the zero-padded LDS vector
    (lane c, row I: element 15 + I - c), then X = eps I + A T -- so lanes 0..12 hold
    eps I + A Sigma' A^T and lane 13 holds A m'."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import emu_dpp as E
    inc = open(os.path.join(REPO, "time_opt_ilqr_amd", "csrc", "dpp_blocks.inc")).read()
    n = 13
    rng = np.random.default_rng(77)
    Sg = rng.standard_normal((n, n))
    Sg = Sg @ Sg.T
    mp = rng.standard_normal(n)
    A = np.eye(n) + 0.1 * rng.standard_normal((n, n))
    regs = {}
    for i in range(n):
        x = np.zeros(16)
        x[:n] = Sg[i]
        x[n] = mp[i]
        x[n + 1:] = 7.0  # lanes > 13 are don't-care in the kernel
        regs[i] = x
        regs[n + i] = np.full(16, np.nan)  # T: outputs
        at = np.zeros(16)
        at[:n] = A[:, i]  # at[j] on lane c = A[c][j] (column j of A)
        regs[2 * n + i] = at
        ar = np.zeros(16)
        ar[:n] = A[i]  # ar[i] on lane j = A[i][j]
        regs[3 * n + 1 + i] = ar
    es = np.zeros(16)
    es[n] = 1.0
    regs[3 * n] = es  # at[13] = e_13
    base = 4096
    lds = np.full(8192 // 8, np.nan)
    lds[base // 8: base // 8 + 32] = 0.0
    lds[base // 8 + 15] = 1e-9
    regs[4 * n + 1] = base + 8.0 * (15 - np.arange(16))
    E.run(E.extract(inc, "PredictEps", n), regs, lds=lds)
    X = np.array([regs[i] for i in range(n)])
    want = 1e-9 * np.eye(n) + A @ Sg @ A.T
    assert np.abs(X[:, :n] - want).max() <= 1e-13 * np.abs(want).max()
    assert np.abs(X[:, n] - A @ mp).max() <= 1e-13 * np.abs(A @ mp).max()


def test_lu_slot_pivoting_host_build(small_host, golden_dir):
    """lu_pivot.hpp (the kernels' LU slot, utils.py:88-93) on the host: the
    reference's chol_inv outputs for blocks whose A + 0.1 I has a zero leading entry
    (an unpivoted elimination divides by zero there) and random regular ones."""
    fn = small_host.small_host_lu_sym_solve_f64
    fn.argtypes = [C.c_void_p, C.c_int, C.c_double, C.c_void_p, C.c_void_p]
    fn.restype = C.c_int
    d = np.load(os.path.join(golden_dir, "lu_pivot_cases.npz"))

    def inv(A, eps):
        n = A.shape[0]
        A = np.ascontiguousarray(A, dtype=np.float64)
        out = np.zeros((n, n))
        for c in range(n):
            b = np.zeros(n)
            b[c] = 1.0
            x = np.zeros(n)
            assert fn(A.ctypes.data, n, eps, b.ctypes.data, x.ctypes.data) == 0
            out[:, c] = x
        return out

    for s in (3, 5, 13):
        got = inv(d[f"inv_s{s}_in"], 0.1)
        ref = d[f"inv_s{s}_out"]
        assert np.max(np.abs(got - ref)) <= 1e-12 * np.max(np.abs(ref)), s
    rng = np.random.default_rng(3)
    for n in (2, 7, 16):
        A = rng.standard_normal((n, n))
        ref = np.linalg.solve(0.5 * (A + A.T) + 1e-3 * np.eye(n), np.eye(n))
        got = inv(A, 1e-3)
        assert np.max(np.abs(got - ref)) <= 1e-10 * np.max(np.abs(ref)), n


def test_mfma_predict_lane_maps_emulated():
    """The fp32-block kernel's MFMA predict (SchedCondMfma): LDS staging addresses, the
    v_mfma_f32_16x16x4_f32 operand / result lane maps and the write-back, emulated for
    one wave of 4 problems (tools/emu_mfma_predict.py), give A [Sigma' | m'] A~^T to
    f32 rounding; lanes 14, 15 come back 0."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import emu_mfma_predict as emu
    assert emu.main() < 5e-7


def test_packed_sweep_colchain_block_emulated():
    """SweepQColChainOff<4, 12, 12> (the Riccati kernel's packed [Qux | Quu] rows: the
    4 x 4 block on lanes 12..15 in offset form, the RHS Qux on lanes 0..11): one
    Gauss-Jordan sweep leaves (M + eps I)^-1 Qux on lanes 0..11 and I - (M + eps I)^-1
    on lanes 12..15, and the fused column chains acc[r] += sum_j x[j]@r * y[j]
    (CPU emulation of the instruction strings, tools/emu_dpp.py)."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import emu_dpp as E
    inc = open(os.path.join(REPO, "time_opt_ilqr_amd", "csrc", "dpp_blocks.inc")).read()
    rng = np.random.default_rng(41)
    M = rng.standard_normal((4, 4))
    M = M @ M.T + 4 * np.eye(4)
    Y = rng.standard_normal((4, 12))
    eps = 1e-9
    regs = {}
    for r in range(4):
        v = np.empty(16)
        v[:12] = Y[r]
        v[12:] = M[r]
        v[12 + r] += eps - 1.0
        regs[r] = v
    regs[4] = np.ones(16)
    for j in range(7):
        regs[5 + j] = np.full(16, np.nan)
    acc0 = rng.standard_normal((12, 16))
    X = rng.standard_normal((12, 16))
    Yc = rng.standard_normal((12, 16))
    for j in range(12):
        regs[12 + j], regs[24 + j], regs[36 + j] = acc0[j].copy(), X[j], Yc[j]
    E.run(E.extract(inc, "SweepQColChainOff", "4, 12, 12"), regs)
    Mi = np.linalg.inv(M + eps * np.eye(4))
    got_y = np.array([regs[r][:12] for r in range(4)])
    got_i = np.array([regs[r][12:] for r in range(4)])
    assert np.abs(got_y - Mi @ Y).max() < 1e-12
    assert np.abs(got_i - (np.eye(4) - Mi)).max() < 1e-12
    assert regs[4][0] > 0
    for r in range(12):
        want = acc0[r] + sum(X[j][r] * Yc[j] for j in range(12))
        assert np.abs(regs[12 + r] - want).max() < 1e-12


def test_lane_rows_q_block_emulated():
    """LaneRowsQ<12> (the Riccati step's V [A|B] product with the Q image's 12 reads
    riding in it): every output row is the same j-ordered chain as LaneDot<12>::fma
    (bitwise in the emulation), and q[r] is LDS row r at the lane's address + 128 r
    (CPU emulation of the instruction strings, tools/emu_dpp.py)."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import emu_dpp as E
    inc = open(os.path.join(REPO, "time_opt_ilqr_amd", "csrc", "dpp_blocks.inc")).read()
    rng = np.random.default_rng(43)
    n = 12
    acc0 = rng.standard_normal((n, 16))
    X = rng.standard_normal((n, 16))
    Y = rng.standard_normal((n, 16))
    lds = rng.standard_normal(4096)
    base = 8 * 100 + 8 * np.arange(16)  # lane c reads Q image row r at base + 128 r
    regs = {}
    for i in range(n):
        regs[i] = acc0[i].copy()
        regs[n + i] = np.full(16, np.nan)
        regs[2 * n + i] = X[i]
        regs[3 * n + i] = Y[i]
    regs[4 * n] = base.astype(float)
    E.run(E.extract(inc, "LaneRowsQ", "12"), regs, lds=lds)
    for i in range(n):
        want = acc0[i].copy()
        for j in range(n):  # LaneDot<12>::fma's order: acc += bcast_j(x) * y[j], j = 0..11
            want = want + np.full(16, X[i][j]) * Y[j]
        assert np.array_equal(regs[i], want)
        assert np.array_equal(regs[n + i], lds[(base + 128 * i) // 8])


def test_argmin_replay_rule_equals_the_fused_sequential_rule():
    """The rerun launch's non-finite triage replays the fused argmin as one wave
    reduction (lft_sweep_v2.hip nonfinite_resolve): "the first NaN of the window, else
    the first minimiser".  That equals the kernels' sequential rule (t_min initialises;
    later t <= t_max replace when best is not NaN and J is NaN or strictly smaller) on
    every window the C ABI accepts (1 <= t_min <= t_max <= N), NaN tails included."""
    rng = np.random.default_rng(11)
    for _ in range(3000):
        N = int(rng.integers(1, 40))
        J = rng.choice([-1.0, 0.0, 1.0, 2.0], size=N) + rng.integers(0, 3, size=N) * 0.5
        if rng.random() < 0.5:
            J[rng.integers(0, N, size=int(rng.integers(1, 4)))] = np.nan
        if rng.random() < 0.3:
            J[int(rng.integers(0, N)):] = np.nan  # the triage's NaN tail from h_nf
        t_min = int(rng.integers(1, N + 1))
        t_max = int(rng.integers(t_min, N + 1))
        best, tbest = 0.0, 0
        for t in range(1, N + 1):
            jk = J[t - 1]
            if t == t_min:
                best, tbest = jk, t
            elif t_min < t <= t_max and not np.isnan(best) and (np.isnan(jk) or jk < best):
                best, tbest = jk, t
        win = np.arange(t_min, t_max + 1)
        nans = [t for t in win if np.isnan(J[t - 1])]
        if nans:
            t2, b2 = nans[0], np.nan
        else:
            vals = J[win - 1]
            t2 = int(win[int(np.argmin(vals))])
            b2 = J[t2 - 1]
        assert t2 == tbest, (J, t_min, t_max)
        assert (np.isnan(b2) and np.isnan(best)) or b2 == best


def test_nonfinite_triage_rule_matches_oracle_semantics():
    """The rerun launch's non-finite triage (lft_sweep_v2.hip nonfinite_resolve) claims
    that with h_poison = 1 + the first stage whose Q_k / A_k / B_k is non-finite (1 for a
    non-finite z0 or R^-1), h_qt = the first horizon whose QT block is non-finite and
    h_nf = min of the two, h_poison <= h_qt + 1 implies: the reference association's J is
    finite before h_nf and NaN from h_nf on, and its status is ST_NONFINITE alone.  The
    oracle (pinned to the reference's outputs, utils.py:77's finiteness semantics) holds
    it on random NaN / inf placements; when the rule does not apply the triage leaves
    the problem to the recompute (nothing to check)."""
    rng = np.random.default_rng(77)
    s, m, N = 4, 2, 12
    checked = 0
    for case in range(400):
        A, Bm, Q, R, Ri, z0, QT = orc.synth_lft_problem(900 + case, s, m, N)
        A, Bm, Q, QT, z0, Ri = A.copy(), Bm.copy(), Q.copy(), QT.copy(), z0.copy(), Ri.copy()
        for _ in range(int(rng.integers(1, 3))):
            what = int(rng.integers(0, 6))
            k = int(rng.integers(0, N))
            val = [np.nan, np.inf, -np.inf][int(rng.integers(0, 3))]
            i, j = int(rng.integers(0, s)), int(rng.integers(0, s))
            if what == 0:
                Q[k, i, j] = val
            elif what == 1:
                A[k, i, j] = val
            elif what == 2:
                Bm[k, i, j % m] = val
            elif what == 3:
                QT[k, i, j] = val
            elif what == 4 and rng.random() < 0.2:
                z0[i] = val
            elif what == 5 and rng.random() < 0.2:
                Ri[i % m, j % m] = val
        bad = lambda x: not np.isfinite(x).all()  # noqa: E731
        INF = N + 1
        stage = [k for k in range(N) if bad(Q[k]) or bad(A[k]) or bad(Bm[k])]
        h_poison = 1 if (bad(z0) or bad(Ri)) else (stage[0] + 1 if stage else INF)
        qts = [k + 1 for k in range(N) if bad(QT[k])]
        h_qt = qts[0] if qts else INF
        h_nf = min(h_poison, h_qt)
        if not (h_nf <= N and h_poison <= h_qt + 1):
            continue
        with np.errstate(invalid="ignore", over="ignore", divide="ignore"):
            o = orc.lft_sweep(A, Bm, Q, Ri, z0, QT, N)
        J = o["J"]
        assert np.isfinite(J[:h_nf - 1]).all(), (case, h_nf, J)
        assert np.isnan(J[h_nf - 1:]).all(), (case, h_nf, J)
        assert int(o["status"]) == 4, (case, o["status"])
        checked += 1
    assert checked > 100


def test_handover_word_is_defined_once_in_hop_h(small_host):
    """The hand-over word (status bit 16 + the first flagged horizon at bits
    HOP_HANDOVER_SHIFT.., include/hop.h) has one definition: the host build encodes /
    decodes it with hop.h's macros (round trip, clamp below the sign bit), and no
    kernel source packs or unpacks the field by hand (a literal shift by 13 or a
    reason shift by 5 outside hop.h would be a second definition)."""
    import re
    for h in (0, 1, 2, 99, 100, 4096, 262142, 262143):
        w = small_host.small_host_handover_word(h)
        assert w & 16 and w >= 0
        assert small_host.small_host_handover_horizon(w) == h
    for h in (262144, 1 << 20, (1 << 31) - 1):
        w = small_host.small_host_handover_word(h)
        assert w >= 0 and small_host.small_host_handover_horizon(w) == 262143
    csrc = os.path.join(REPO, "time_opt_ilqr_amd", "csrc")
    for fn in os.listdir(csrc):
        if not fn.endswith((".hip", ".hpp", ".cpp")):
            continue
        with open(os.path.join(csrc, fn)) as f:
            src = f.read()
        assert not re.search(r"(<<|>>)\s*13\b", src), fn
        assert not re.search(r"why\s*<<\s*5\b", src), fn


def test_handover_horizon_of_small_cond_math_vs_oracle_first_nonfinite(small_host):
    """The conditioned small-s math (small_math.hpp, the COND kernels' arithmetic) hands
    a problem with non-finite inputs over with the first flagged horizon in the word;
    decoded with hop.h's definition it is the reference association's first non-finite
    horizon (the oracle's J curve, pinned to the reference), and the conditioned J
    before it is finite.  This is the field the s = 13 rerun launch's triage reads
    (HOP_TRIAGE_ACCEPTS: it requires h >= the first poisoned horizon)."""
    rng = np.random.default_rng(91)
    s, m, N = 3, 1, 16
    p = lambda x: x.ctypes.data_as(C.c_void_p)  # noqa: E731
    checked = 0
    for case in range(300):
        A, Bm, Q, R, Ri, z0, QT = orc.synth_lft_problem(1300 + case, s, m, N)
        A, Bm, Q, QT, z0, Ri = A.copy(), Bm.copy(), Q.copy(), QT.copy(), z0.copy(), Ri.copy()
        what = int(rng.integers(0, 4))
        k = int(rng.integers(0, N))
        i, j = int(rng.integers(0, s)), int(rng.integers(0, s))
        val = np.nan if rng.random() < 0.5 else np.inf * (1 if rng.random() < 0.5 else -1)
        if what == 0:
            Q[k, i, j] = val
        elif what == 1:
            A[k, i, j] = val
        elif what == 2:
            Bm[k, i, 0] = val
        else:
            QT[k, i, j] = val
        with np.errstate(invalid="ignore", over="ignore", divide="ignore"):
            o = orc.lft_sweep(A, Bm, Q, Ri, z0, QT, N)
        nf = np.nonzero(~np.isfinite(o["J"]))[0]
        if not len(nf):
            continue
        h_ref = int(nf[0]) + 1
        J = np.zeros((1, N))
        st, ts = np.zeros(1, np.int32), np.zeros(1, np.int32)
        args = [np.ascontiguousarray(x, dtype=np.float64) for x in (A, Bm, Q, Ri[None], QT, z0[None])]
        with np.errstate(invalid="ignore", over="ignore"):
            assert small_host.small_host_cond_sweep_f64(*[p(x) for x in args], C.c_int64(1), N, s,
                                                        m, 1, N, p(J), p(st), p(ts)) == 0
        assert st[0] & 16, (case, what, val, h_ref)
        h = small_host.small_host_handover_horizon(int(st[0]))
        assert h == h_ref, (case, what, val, h, h_ref)
        assert np.isfinite(J[0, :h - 1]).all(), (case, J[0])
        # the triage's verdict on this shape: a poisoned stage k (h_poison = k + 1) makes
        # every later horizon NaN and is accepted; a lone non-finite terminal block
        # (h_qt = k + 1, later horizons finite again) is left to the recompute
        h_poison = k + 1 if what < 3 else N + 1
        h_qt = k + 1 if what == 3 else N + 1
        want = 1 if (what < 3 or k == N - 1) else 0
        assert small_host.small_host_triage_accepts(h, h_poison, h_qt, N) == want
        assert small_host.small_host_triage_accepts(h - 1, h_poison, h_qt, N) == 0
        checked += 1
    assert checked > 150


def test_lu_slot_registers_equal_per_column_solves(small_host):
    """small_math.hpp's LU slot (lu_sym_solve_regs: one factorisation, the identity's
    columns carried through the elimination, every index a constant so the arrays
    stay in registers) against lu_pivot.hpp's per-column lu_sym_solve: bit for bit,
    for blocks the jitter ladder cannot make positive definite (indefinite, a zero
    leading entry that needs the row exchange); quad_inverse's one-column slot the same"""
    inv = small_host.small_host_spd_inverse_s5_f64
    inv.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    quad = small_host.small_host_quad_inverse_s5_f64
    quad.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
    quad.restype = C.c_double
    col = small_host.small_host_lu_sym_solve_f64
    col.argtypes = [C.c_void_p, C.c_int, C.c_double, C.c_void_p, C.c_void_p]
    col.restype = C.c_int
    rng = np.random.default_rng(11)
    cases = []
    for _ in range(40):
        Qo, _ = np.linalg.qr(rng.standard_normal((5, 5)))
        ev = rng.uniform(0.5, 3.0, 5)
        ev[rng.integers(5)] = -rng.uniform(1.0, 5.0)       # beyond the ladder's 0.1
        cases.append(Qo @ np.diag(ev) @ Qo.T)
    Z = np.diag([0.0, 1.0, 1.0, 1.0, 1.0]) - 2.0 * np.eye(5)   # zero-pivot-free only with
    Z[0, 1] = Z[1, 0] = 1.0                                    # the row exchange
    Z[0, 0] = -0.1
    cases.append(Z)
    for M in cases:
        M = np.ascontiguousarray(M)
        out = np.zeros((5, 5))
        st = C.c_uint(0)
        inv(M.ctypes.data, 8, out.ctypes.data, C.byref(st))
        assert st.value & 2, st.value  # the LU slot ran
        eps = 1e-9 * 10.0 ** 8
        ref = np.zeros((5, 5))
        for c in range(5):
            b = np.zeros(5)
            b[c] = 1.0
            x = np.zeros(5)
            assert col(M.ctypes.data, 5, eps, b.ctypes.data, x.ctypes.data) == 0
            ref[:, c] = x
        iu = np.triu_indices(5)
        assert np.array_equal(out[iu], ref[iu])
        np_ref = np.linalg.solve(M + eps * np.eye(5), np.eye(5))
        assert np.max(np.abs(out[iu] - np_ref[iu])) <= 1e-12 * np.max(np.abs(np_ref))
        z = rng.standard_normal(5)
        q = quad(M.ctypes.data, z.ctypes.data, 8, C.byref(st))
        x = np.zeros(5)
        assert col(M.ctypes.data, 5, eps, z.ctypes.data, x.ctypes.data) == 0
        assert st.value & 2 and q == float(sum(z[i] * x[i] for i in range(5)))
