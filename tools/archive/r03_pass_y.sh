#!/bin/bash
# Round 3: SQ counters of the two-lane quadrotor line search (tools/bench_forward.py --no-loop).
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
SQ1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_LDS SQ_BUSY_CYCLES"
timeout -s KILL 120 rocprofv3 --pmc $SQ1 -d $OUT/ls/pmc_sq -o run --output-format csv -- python3 tools/bench_forward.py --system quadrotor --no-loop --cpu-seconds 0 --rounds 1 --iters 2 > $OUT/ls.pmc.log 2>&1
rc=$?
python3 tools/pmc_summary.py $OUT/ls "linesearch_kernel" > $OUT/summary.txt 2>&1
echo "rc=$rc"; exit $rc
