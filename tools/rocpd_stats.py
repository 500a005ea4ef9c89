"""Kernel statistics from a rocprofv3 database (the default rocpd output, `-o NAME`
-> NAME_results.db): count, average / min / max duration per kernel, split by
code object (one per loaded library), as `--stats` prints for csv output.

    python tools/rocpd_stats.py <results.db> [name-substring ...]
"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    pats = sys.argv[2:]
    c = sqlite3.connect(db)
    q = ("select code_object_id, name, count(*), avg(end - start), min(end - start), "
         "max(end - start), sum(end - start) from kernels group by code_object_id, name "
         "order by sum(end - start) desc")
    print(f"{'code_obj':>8} {'calls':>6} {'avg_us':>10} {'min_us':>10} {'max_us':>10} {'total_ms':>10}  kernel")
    for co, name, n, avg, lo, hi, tot in c.execute(q):
        if pats and not any(p in name for p in pats):
            continue
        print(f"{co:>8} {n:>6} {avg / 1e3:>10.2f} {lo / 1e3:>10.2f} {hi / 1e3:>10.2f} "
              f"{tot / 1e6:>10.3f}  {name[:150]}")


if __name__ == "__main__":
    main()
