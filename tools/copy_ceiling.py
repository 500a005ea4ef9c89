"""HBM ceilings of the traffic mixes the kernels here run (what
a Riccati mode-1 pass, ~50 % reads and ~50 % writes, can reach against the 8 TB/s
read figure):

  read   torch.sum over a 4 GiB fp64 tensor (read-only stream)
  write  fill_ of a 4 GiB tensor (write-only stream)
  copy   copy_ 2 GiB -> 2 GiB (half reads, half writes: mode 1's mix)
  read2_write1  torch.add of two 1.3 GiB views into a third (2:1 reads to writes;
         mode 0's mix is 4:1, the LFT sweep's read-only)

Each: 3 warm-ups, then the median of 20 launches (HIP events), bytes = algorithmic.
With --riccati, the Riccati mode-1 pass (tools/bench_riccati.py's inputs, B = 4096,
T = 100) is timed in the same process, so its rate is compared with the copy on the
same box and clocks (rounds alternate copy and mode 1).

    python tools/copy_ceiling.py [--riccati] [out.json]
"""
import json
import statistics
import sys

import torch


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e-3)
    return statistics.median(ts)


def riccati_vs_copy(dev, dst, src, rounds=7):
    """Riccati mode 1 (value expansions, horizon_selection.py:97-212) and the 2 GiB copy,
    interleaved: median ms of each, the mode-1 algorithmic rate and its ratio to the copy."""
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import riccati_bytes
    from time_opt_ilqr_amd import engine
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    Bn, n, m, N = 4096, 12, 4, 100
    kw = dict(device=dev, dtype=torch.float64, generator=g)
    A = torch.eye(n, device=dev, dtype=torch.float64) + 0.05 * torch.randn((Bn, N, n, n), **kw)
    Bm = 0.1 * torch.randn((Bn, N, n, m), **kw)
    X = 0.5 * torch.randn((Bn, N + 1, n), **kw)
    U = 0.1 * torch.randn((Bn, N, m), **kw)
    xg, ur = 0.2 * torch.randn((n,), **kw), 0.05 * torch.randn((m,), **kw)
    M = torch.randn((n, n), **kw)
    Q = M @ M.T / n + 0.5 * torch.eye(n, device=dev, dtype=torch.float64)
    R = torch.diag(0.5 + 1.5 * torch.rand((m,), **kw))
    Qf = 10.0 * torch.eye(n, device=dev, dtype=torch.float64)
    ric = lambda: engine.riccati(A, Bm, X, U, xg, ur, Q, R, Qf, N, 1e-3, mode=1)  # noqa: E731
    cp = lambda: dst.copy_(src)  # noqa: E731
    tr, tc = [], []
    for _ in range(rounds):
        tr.append(timed(ric, iters=10))
        tc.append(timed(cp, iters=10))
    ms_r, ms_c = statistics.median(tr) * 1e3, statistics.median(tc) * 1e3
    gbs_r = Bn * riccati_bytes(n, m, N, 1) / (ms_r * 1e-3) / 1e9
    gbs_c = 2 * dst.numel() * 8 / (ms_c * 1e-3) / 1e9
    return {"mode1_ms": ms_r, "mode1_GB/s": gbs_r, "copy_ms": ms_c, "copy_GB/s": gbs_c,
            "mode1_over_copy": gbs_r / gbs_c}


def main():
    dev = torch.device("cuda", 0)
    n = (4 << 30) // 8
    a = torch.empty(n, dtype=torch.float64, device=dev).normal_()
    out = {}
    t = timed(lambda: a.sum())
    out["read"] = {"GB/s": a.numel() * 8 / t / 1e9, "ms": t * 1e3}
    t = timed(lambda: a.fill_(1.0))
    out["write"] = {"GB/s": a.numel() * 8 / t / 1e9, "ms": t * 1e3}
    h = n // 2
    src, dst = a[:h], a[h:]
    t = timed(lambda: dst.copy_(src))
    out["copy"] = {"GB/s": 2 * h * 8 / t / 1e9, "ms": t * 1e3}
    # 2:1 -- two sources summed into one destination
    q = n // 3
    s1, s2, d = a[:q], a[q:2 * q], a[2 * q:3 * q]
    t = timed(lambda: torch.add(s1, s2, out=d))
    out["read2_write1"] = {"GB/s": 3 * q * 8 / t / 1e9, "ms": t * 1e3}
    if "--riccati" in sys.argv:
        out["riccati_mode1_vs_copy"] = riccati_vs_copy(dev, dst, src)
    for v in out.values():
        if "GB/s" in v:
            v["frac_of_8TBs"] = v["GB/s"] / 8000.0
    print(json.dumps(out), flush=True)
    files = [x for x in sys.argv[1:] if not x.startswith("--")]
    if files:
        with open(files[0], "w") as f:
            json.dump(out, f)


if __name__ == "__main__":
    main()
