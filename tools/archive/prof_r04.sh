#!/bin/bash
# Round 4: rocprofv3 --kernel-trace --stats of the bench commands themselves (config 2,
# config 3 with its raw-linearisation side figure, select + gains at rho_reg = 1e-12,
# brute force), then FETCH_SIZE / WRITE_SIZE passes (separate runs, no trace domains)
# for the workloads whose kernels changed this round (tools/make_traffic.py writes
# profiles/traffic.json from them on the CPU side).
#   gpurun -- bash tools/prof_r04.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/c2.json 2> $OUT/c2.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c3 -o run --output-format csv -- python3 bench.py --workload config3 --no-cpu-baseline > $OUT/c3.json 2> $OUT/c3.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/sg -o run --output-format csv -- python3 bench.py --workload select_gains --no-cpu-baseline > $OUT/sg.json 2> $OUT/sg.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/bf -o run --output-format csv -- python3 bench.py --workload bruteforce --steps 5 --no-cpu-baseline > $OUT/bf.json 2> $OUT/bf.err || exit $?
run() {  # name, bench args
  local n=$1; shift
  local B="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-h2d --no-anchor --no-alt --prewarm-s 0 $*"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_$n/pmc_fetch -o run --output-format csv -- $B > $OUT/$n.fetch.log 2>&1 && \
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_$n/pmc_write -o run --output-format csv -- $B > $OUT/$n.write.log 2>&1
}
run config2 && run c4shard --batch 32768 && run sg --workload select_gains && run config3 --workload config3
rc=$?; echo "prof_r04 rc=$rc"; exit $rc
