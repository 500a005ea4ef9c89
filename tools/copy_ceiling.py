"""HBM ceilings of the traffic mixes the kernels here run (what
a Riccati mode-1 pass, ~50 % reads and ~50 % writes, can reach against the 8 TB/s
read figure):

  read   torch.sum over a 4 GiB fp64 tensor (read-only stream)
  write  fill_ of a 4 GiB tensor (write-only stream)
  copy   copy_ 2 GiB -> 2 GiB (half reads, half writes: mode 1's mix)
  read2_write1  torch.add of two 1.3 GiB views into a third (2:1 reads to writes;
         mode 0's mix is 4:1, the LFT sweep's read-only)

Each: 3 warm-ups, then the median of 20 launches (HIP events), bytes = algorithmic.

    python tools/copy_ceiling.py [out.json]
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
    for v in out.values():
        v["frac_of_8TBs"] = v["GB/s"] / 8000.0
    print(json.dumps(out), flush=True)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(out, f)


if __name__ == "__main__":
    main()
