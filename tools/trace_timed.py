"""Per-launch durations of a kernel over bench.py's timed launches, from a rocprofv3
--kernel-trace CSV: the K launches of the given grid size that precede the first launch
of a different grid size (the N = 1 config-2 run times its 20 steps, then the
config-4-shard anchor), or the last K when none follows.

    python tools/trace_timed.py <run_kernel_trace.csv> <kernel substring> [K]
"""
import csv
import sys


def timed(path, name, k):
    rows = [r for r in csv.DictReader(open(path)) if name in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    g = [int(r["Grid_Size_X"]) for r in rows]
    end = len(d)
    for i in range(1, len(d)):
        if g[i] != g[0]:
            end = i
            break
    sel = d[max(0, end - k):end]
    return sel, len(d)


if __name__ == "__main__":
    path, name = sys.argv[1], sys.argv[2]
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    sel, n = timed(path, name, k)
    print(f"{name}: {n} launches in the trace; the {len(sel)} timed ones average "
          f"{sum(sel) / len(sel):.4f} ms (min {min(sel):.4f}, max {max(sel):.4f})")
