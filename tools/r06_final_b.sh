#!/bin/bash
# Round 6 evidence pass B: rocprofv3 kernel traces of the bench commands (config 2, select
# + gains, config 3, the quadrotor line search), the FETCH_SIZE / WRITE_SIZE and SQ PMC passes of config 2 (separate
# runs, no trace domains), the rerun bench under a kernel trace, the Riccati passes.
#   gpurun --timeout 1200 -- bash tools/r06_final_b.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/c2.json 2> $OUT/c2.err || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/sg -o run --output-format csv -- python3 bench.py --workload select_gains --no-cpu-baseline > $OUT/sg.json 2> $OUT/sg.err || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/c3 -o run --output-format csv -- python3 bench.py --workload config3 --no-cpu-baseline > $OUT/c3.json 2> $OUT/c3.err || exit $?
B="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-h2d --no-anchor --no-alt --prewarm-s 0"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- $B > $OUT/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- $B > $OUT/pmc_write.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM -d $OUT/pmc_sq -o run --output-format csv -- $B > $OUT/pmc_sq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/rerun -o run --output-format csv -- python3 tools/bench_rerun.py time_opt_ilqr_amd/libhop_amd.so --rounds 5 > $OUT/rerun.jsonl 2> $OUT/rerun.err || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/fwd -o run --output-format csv -- python3 tools/bench_forward.py --system quadrotor --no-loop --cpu-seconds 1 > $OUT/fwd.jsonl 2> $OUT/fwd.err || exit $?
timeout -k 10 200 python tools/bench_riccati.py > $OUT/riccati.jsonl 2> $OUT/riccati.err
rc=$?; echo "r06_final_b rc=$rc"; exit $rc
