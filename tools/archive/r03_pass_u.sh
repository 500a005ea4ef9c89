#!/bin/bash
# Round 3 final: config 5's PMC passes (its s = 13 kernel now reads under the sweeps) and the
# rocprofv3 kernel traces of the bench commands (tools/prof_r03_bench.sh).
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
B="python3 bench.py --workload config5 --steps 5 --warmup 1 --no-cpu-baseline --no-h2d --no-anchor --no-alt --prewarm-s 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/config5/trace -o run --output-format csv -- $B > $OUT/config5.trace.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/config5/pmc_fetch -o run --output-format csv -- $B > $OUT/config5.fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/config5/pmc_write -o run --output-format csv -- $B > $OUT/config5.write.log 2>&1 && \
bash tools/prof_r03_bench.sh $1pb
rc=$?; echo "rc=$rc"; exit $rc
