"""Per-section cycle breakdown of the Riccati kernel (HOP_OPT_STAMPS instantiation of a developer build).

    python tools/stamps_riccati.py [--batch 4096] [--N 100] [--mode 0]
"""
import argparse
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
FAST = ["top wait", "stores (prev step)", "read [A|B], x, u", "e, du, lx, lu, qab",
        "V [A|B]", "Qxx, Qux, Quu", "Quu^T", "regularised solve", "gains K, k",
        "value update", "V^T, symmetrize", "checks, commit"]
NAMES = ["prefetch copy, e/du, ballot", "lx, lu, l0, Q column", "Qx, Qu, Vxx A, Vxx B",
         "Qxx, Quu, Qux", "Quu^T + regularised solve", "gains K, k", "value update",
         "symmetrize V, checks", "stores"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--N", type=int, default=100)
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--generic", action="store_true",
                    help="stamp the generic kernel (n != 12 or m != 4 shapes)")
    args = ap.parse_args()
    import torch
    from time_opt_ilqr_amd import _lib, engine
    lib = _lib.load()
    lib.hop_debug_ric_stamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    lib.hop_debug_ricf_stamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    Bn, n, m, N = args.batch, 12, 4, args.N
    kw = dict(device=dev, dtype=torch.float64, generator=g)
    eye = torch.eye(n, device=dev, dtype=torch.float64)
    A = eye + 0.05 * torch.randn((Bn, N, n, n), **kw)
    Bm = 0.1 * torch.randn((Bn, N, n, m), **kw)
    X = 0.5 * torch.randn((Bn, N + 1, n), **kw)
    U = 0.1 * torch.randn((Bn, N, m), **kw)
    M = torch.randn((n, n), **kw)
    Q = M @ M.T / n + 0.5 * eye
    R = torch.eye(m, device=dev, dtype=torch.float64)
    flags = _lib.OPT_STAMPS | (_lib.OPT_FORCE_GENERIC if args.generic else 0)
    _lib.check(_lib.load().hop_set_options(flags, 0))  # developer build
    rd = lib.hop_debug_ric_stamps if args.generic else lib.hop_debug_ricf_stamps
    names = NAMES if args.generic else FAST
    buf = (C.c_ulonglong * 16)()
    run = lambda: engine.riccati(A, Bm, X, U, torch.zeros(n, **{k: v for k, v in kw.items() if k != "generator"}),  # noqa: E731
                                 torch.zeros(m, device=dev, dtype=torch.float64), Q, R, 10 * eye, N,
                                 1e-3, mode=args.mode)
    run()
    torch.cuda.synchronize()
    rd(buf, 1)
    run()
    torch.cuda.synchronize()
    rd(buf, 1)
    waves = buf[15]
    tot = 0.0
    for j in range(len(names)):
        cyc = buf[j] / waves / N
        tot += cyc
        print(f"{j} {names[j]:32s} {cyc:9.1f} cycles/wave/step")
    print(f"  total {tot:9.1f} cycles/wave/step  (waves {waves})")


if __name__ == "__main__":
    main()
