"""Where a multi-launch step's time goes: per-kernel durations and the idle gaps between
consecutive dispatches, from a rocprofv3 kernel trace (run_kernel_trace.csv).

    python tools/launch_gaps.py <run_kernel_trace.csv> <first-kernel-substring> [--skip N]

A step starts at each dispatch whose name contains the first substring (the step's
first kernel); every dispatch up to the next such one belongs to it.  Reported
(medians over the steps after --skip warm-up steps): the step period (start to next
start), each kernel's duration, each gap (end of one dispatch to the start of the
next, including the gap that closes the step), and the busy fraction.  Used for
VERDICT r05 item 7 (the select + gains block: would one fused launch pay?).
"""
import csv
import json
import statistics
import sys


def short(name):
    n = name.split("(")[0]
    for key in ("lft_cond_cf_kernel", "lft_rerun_pipe_kernel", "riccati_fast_kernel",
                "lft_cond_kernel", "lft_small_kernel", "lft_sweep_v2_kernel"):
        if key in n:
            return key
    return n[-40:]


def main(argv):
    path, first = argv[1], argv[2]
    skip = int(argv[argv.index("--skip") + 1]) if "--skip" in argv else 5
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    rows = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
             first in r["Kernel_Name"]) for r in rows]
    steps, cur = [], None
    for r in rows:
        if r[3]:
            if cur:
                steps.append(cur)
            cur = [r]
        elif cur is not None:
            cur.append(r)
    # the bench's timed steps: the most common dispatch count per step (side figures
    # and warm-up launches of other shapes drop out)
    common = statistics.mode([tuple(nm for nm, _, _, _ in s) for s in steps])
    steps = [s for s in steps if tuple(nm for nm, _, _, _ in s) == common][skip:]
    if len(steps) < 2:
        raise SystemExit("fewer than two complete steps")
    per = {"period_us": [], "busy_us": []}
    for i in range(len(steps) - 1):
        s, nxt = steps[i], steps[i + 1]
        if nxt[0][1] - s[-1][2] > 1e6:  # not consecutive (another phase in between)
            continue
        per["period_us"].append((nxt[0][1] - s[0][1]) / 1e3)
        per["busy_us"].append(sum(e - b for _, b, e, _ in s) / 1e3)
        for j, (nm, b, e, _) in enumerate(s):
            per.setdefault(f"k{j}_{nm}_us", []).append((e - b) / 1e3)
            nb = s[j + 1][1] if j + 1 < len(s) else nxt[0][1]
            per.setdefault(f"gap_after_k{j}_us", []).append((nb - e) / 1e3)
    out = {k: round(statistics.median(v), 2) for k, v in per.items()}
    out["busy_frac"] = round(out["busy_us"] / out["period_us"], 4)
    out["steps"] = len(steps) - 1
    out["kernels_per_step"] = [nm for nm, _, _, _ in steps[0]]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv)
