#!/bin/bash
# Round 3: the EXEC-mask issue micro-benchmark and the bruteforce PMC passes
# (kernel trace, FETCH_SIZE, WRITE_SIZE) of the two-wave J curve.
#   gpurun -- bash tools/r03_pass_j.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
B="python3 bench.py --workload bruteforce --steps 5 --warmup 1 --no-cpu-baseline --no-h2d --no-anchor --no-alt --prewarm-s 0"
timeout -k 10 60 ./tools/bin/ubench_exec > $OUT/ubench_exec.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/bf/trace -o run --output-format csv -- $B > $OUT/bf.trace.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/bf/pmc_fetch -o run --output-format csv -- $B > $OUT/bf.fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/bf/pmc_write -o run --output-format csv -- $B > $OUT/bf.write.log 2>&1
rc=$?; echo "rc=$rc"; exit $rc
