"""Summarise rocprofv3 counter CSVs for one kernel: per-dispatch means, per-wave figures."""
import collections
import csv
import glob
import sys

root, pat = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "lft_sweep")
agg = collections.defaultdict(list)
waves = None
for f in sorted(glob.glob(f"{root}/pmc_*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
if "SQ_WAVES" in agg:
    waves = sum(agg["SQ_WAVES"]) / len(agg["SQ_WAVES"])
for k in sorted(agg):
    v = sum(agg[k]) / len(agg[k])
    extra = f"  per-wave {v / waves:,.0f}" if waves and k.startswith("SQ_") and k != "SQ_WAVES" else ""
    print(f"{k:24s} dispatches={len(agg[k]):3d} mean={v:,.1f}{extra}")
