"""Per-section cycle breakdown of the LFT kernel (diagnostic variant 32 = default + stamps; 20 = SchedLdl).

    python tools/stamps.py [--batch 4096] [--N 100]

Prints shader-clock cycles per wave per step for each section of the step.
Stamps perturb the schedule (each s_memtime waits on lgkmcnt): read them as a
breakdown, not as the kernel's speed.
"""
import argparse
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
NAMES = ["top wait + J store + diag offsets / traj build", "E/Xt inverses", "A/B reads + DMA issue",
         "F, G products", "W inverse", "compose products", "query: X0 (LDL, or Wt inverse)", "V, X0 products (non-LDL)",
         "bordered elimination", "traj: top wait + J store", "traj: LDS loads + selects",
         "traj: wrap", "traj: Q e, P e, B du", "traj: row sums", "traj: image writes"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--N", type=int, default=100)
    ap.add_argument("--variant", type=int, default=32)
    ap.add_argument("--cond", action="store_true",
                    help="conditioned-prefix kernel (variant 42)")
    ap.add_argument("--traj", action="store_true",
                    help="trajectory-form sweep (in-kernel builders, variant 24)")
    args = ap.parse_args()
    import torch
    from time_opt_ilqr_amd import _lib, engine, synth
    lib = _lib.load()
    lib.hop_debug_stamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    dev = torch.device("cuda", 0)
    A, Bm, Q, Ri, z0, QT = synth.device_batch(args.batch, 13, 4, args.N, seed=5, device=dev)
    run = lambda: engine.propagate(A, Bm, Q, Ri, z0, QT)  # noqa: E731
    if args.traj:
        args.variant = 24
        n, m, N, Bn = 12, 4, args.N, args.batch
        g = torch.Generator(device=dev)
        g.manual_seed(5)
        kw = dict(device=dev, dtype=torch.float64, generator=g)
        eye = torch.eye(n, device=dev, dtype=torch.float64)
        M = torch.randn((n, n), **kw)
        targs = (eye + 0.05 * torch.randn((Bn, N, n, n), **kw), 0.1 * torch.randn((Bn, N, n, m), **kw),
                 0.02 * torch.randn((Bn, N, n), **kw), 0.5 * torch.randn((Bn, N + 1, n), **kw),
                 0.3 * torch.randn((Bn, N, m), **kw), 0.2 * torch.randn((n,), **kw),
                 0.1 * torch.randn((m,), **kw), M @ M.T / n + 0.5 * eye,
                 torch.eye(m, device=dev, dtype=torch.float64), 5.0 * eye, 0.5)
        run = lambda: engine.propagate_traj(*targs)  # noqa: E731
    if args.cond:
        args.variant = 42 if args.variant == 32 else args.variant  # 46: the SYM2 form
        NAMES[:8] = ["top wait (DMA of step k)", "J store + diag offsets", "Q/QT image reads (sym)",
                     "E/Xt sweeps", "A/B reads + DMA issue", "update (CondLdl)", "predict products",
                     "query (ElimQ)"]
    _lib.check(_lib.load().hop_set_options(0, int(args.variant)))  # developer build
    buf = (C.c_ulonglong * 16)()
    run()
    torch.cuda.synchronize()
    lib.hop_debug_stamps(buf, 1)
    run()
    torch.cuda.synchronize()
    lib.hop_debug_stamps(buf, 1)
    waves = buf[15]
    tot = 0.0
    for j in range(15):
        if (j == 7 and not args.cond) or (j >= 8 and buf[j] == 0):
            continue
        cyc = buf[j] / waves / args.N
        tot += cyc
        print(f"{j} {NAMES[j]:36s} {cyc:9.1f} cycles/wave/step")
    print(f"  total {tot:9.1f} cycles/wave/step  (waves {waves})")


if __name__ == "__main__":
    main()
