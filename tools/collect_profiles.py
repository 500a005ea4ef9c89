"""Copy one tools/archive/prof_r02.sh pass into profiles/ (tracked): bench lines, rocprofv3
kernel stats per workload, a PMC summary per kernel, and the PMC traffic entries of
profiles/traffic.json.

    python tools/collect_profiles.py gpurun_out/<tag> <round-prefix, e.g. r02>
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(root, d, pat):
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(root, d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def main():
    root, pre = sys.argv[1], sys.argv[2]
    prof = os.path.join(REPO, "profiles")
    lines = []
    for name in ("bench", "bench_config3", "bench_config5", "bench_config5_padded", "bench_sg",
                 "bench_c4shard"):
        p = os.path.join(root, name + ".out")
        if os.path.exists(p):
            d = json.loads(open(p).read().strip().splitlines()[-1])
            d["_run"] = name
            lines.append(d)
    with open(os.path.join(prof, f"{pre}_bench_lines.jsonl"), "w") as f:
        for d in lines:
            f.write(json.dumps(d) + "\n")
    shutil.copy(os.path.join(root, "ric.out"), os.path.join(prof, f"{pre}_riccati.jsonl"))
    for t in ("config2", "config3", "config5", "sg", "ric"):
        src = os.path.join(root, f"tr_{t}", "run_kernel_stats.csv")
        if os.path.exists(src):
            shutil.copy(src, os.path.join(prof, f"{pre}_kernel_stats_{t}.csv"))
    # PMC summaries: per kernel (full template name), per-wave figures for SQ counters
    out = []
    specs = [("pmc_fetch_c2", "lft_cond_kernel<hop::v2::SchedCondL"),
             ("pmc_write_c2", "lft_cond_kernel<hop::v2::SchedCondL"),
             ("pmc_sq_c2", "lft_cond_kernel<hop::v2::SchedCondL"),
             ("pmc_fetch_c3", "lft_small_kernel<float, 5, 1, true, 64, 0, 2>"),
             ("pmc_write_c3", "lft_small_kernel<float, 5, 1, true, 64, 0, 2>"),
             ("pmc_sq_c3", "lft_small_kernel<float, 5, 1, true, 64, 0, 2>"),
             ("pmc_fetch_c3", "lft_small_kernel<float, 5, 1, false, 64, 0, 1>"),
             ("pmc_write_c3", "lft_small_kernel<float, 5, 1, false, 64, 0, 1>"),
             ("pmc_sq_c3", "lft_small_kernel<float, 5, 1, false, 64, 0, 1>"),
             ("pmc_sq_ric", "riccati_fast_kernel<0"), ("pmc_sq_ric", "riccati_fast_kernel<1")]
    traffic = {}
    for d, pat in specs:
        mean, cnt = counters(root, d, pat)
        waves = mean.get("SQ_WAVES")
        for k in sorted(mean):
            extra = ""
            if waves and k.startswith("SQ_") and k != "SQ_WAVES":
                extra = f"  per-wave {mean[k] / waves:,.0f}"
            out.append(f"{pat:48s} {d:14s} {k:22s} n={cnt[k]:3d} mean={mean[k]:,.1f}{extra}")
            if k in ("FETCH_SIZE", "WRITE_SIZE"):
                traffic.setdefault(pat, {})[k] = mean[k]
    out.append("")
    out.append("HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB counters; gfx950 correction, "
               "calibrated for 16-B/lane coalesced streaming reads -- the batch-major small-s stream "
               "(LY 1) is not such a read and its FETCH figure is uncalibrated)")
    for pat, t in traffic.items():
        if "FETCH_SIZE" in t and "WRITE_SIZE" in t:
            out.append(f"{pat:48s} {(2 * t['FETCH_SIZE'] + t['WRITE_SIZE']) * 1024 / 1e9:.4f} GB")
    open(os.path.join(prof, f"{pre}_pmc_summary.txt"), "w").write("\n".join(out) + "\n")
    # bench.py reads profiles/traffic.json by workload key
    tj_path = os.path.join(prof, "traffic.json")
    tj = json.load(open(tj_path)) if os.path.exists(tj_path) else {}
    keymap = {"lft_cond_kernel<hop::v2::SchedCondL": "lft_s13_m4_N100_B4096_f64",
              "lft_small_kernel<float, 5, 1, true, 64, 0, 2>": "config3_s5_m1_N200_B65536_f32_tile64"}
    for pat, key in keymap.items():
        t = traffic.get(pat, {})
        if "FETCH_SIZE" in t and "WRITE_SIZE" in t:
            tj[key] = {"hbm_bytes_per_launch": (2 * t["FETCH_SIZE"] + t["WRITE_SIZE"]) * 1024,
                       "fetch_size_kib": t["FETCH_SIZE"], "write_size_kib": t["WRITE_SIZE"],
                       "correction": "2 x FETCH_SIZE + WRITE_SIZE (gfx950)",
                       "source": f"profiles/{pre}_pmc_summary.txt ({os.path.relpath(root, REPO)})"}
    json.dump(tj, open(tj_path, "w"), indent=1, sort_keys=True)
    print("\n".join(out))


if __name__ == "__main__":
    main()
