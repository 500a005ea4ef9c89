#!/bin/bash
# Round 3: FETCH_SIZE / WRITE_SIZE passes (separate runs, no trace domains) for every
# bench workload, so each bench line carries roofline.traffic (tools/make_traffic.py
# writes profiles/traffic.json from the outputs on the CPU side).
#   gpurun -- bash tools/prof_r03_pmc.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, bench args
  local n=$1; shift
  local B="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-h2d --no-anchor --no-alt --prewarm-s 0 $*"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$n/trace -o run --output-format csv -- $B > $OUT/$n.trace.log 2>&1 && \
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/$n/pmc_fetch -o run --output-format csv -- $B > $OUT/$n.fetch.log 2>&1 && \
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/$n/pmc_write -o run --output-format csv -- $B > $OUT/$n.write.log 2>&1
}
run config2 && run c4shard --batch 32768 && run config3 --workload config3 && \
run config5 --workload config5 && run sg --workload select_gains && run bf --workload bruteforce
rc=$?; echo "pmc rc=$rc"; exit $rc
