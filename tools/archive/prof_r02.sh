#!/bin/bash
# Round-2 evidence pass (GPU box, repo root): bench lines of every workload,
# rocprofv3 --kernel-trace --stats of each, PMC traffic / SQ passes (separate runs).
#   bash tools/prof_r02.sh <tag>          -> gpurun_out/<tag>/
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
B="python3 bench.py --no-cpu-baseline --steps 10 --warmup 2"
run() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$n.out 2> $OUT/$n.err || { echo "FAILED $n"; exit 1; }
}
run bench 300 python3 bench.py && \
run bench_config3 300 $B --workload config3 && \
run bench_config5 300 $B --workload config5 && \
run bench_config5_padded 300 $B --workload config5 --layout padded && \
run bench_sg 300 $B --workload select_gains && \
run bench_c4shard 300 $B --batch 32768 && \
run ric 180 python3 tools/bench_riccati.py && \
run tr_config2 300 rocprofv3 --kernel-trace --stats -d $OUT/tr_config2 -o run --output-format csv -- $B && \
run tr_config3 300 rocprofv3 --kernel-trace --stats -d $OUT/tr_config3 -o run --output-format csv -- $B --workload config3 && \
run tr_config5 300 rocprofv3 --kernel-trace --stats -d $OUT/tr_config5 -o run --output-format csv -- $B --workload config5 && \
run tr_sg 300 rocprofv3 --kernel-trace --stats -d $OUT/tr_sg -o run --output-format csv -- $B --workload select_gains && \
run tr_ric 300 rocprofv3 --kernel-trace --stats -d $OUT/tr_ric -o run --output-format csv -- python3 tools/bench_riccati.py --rounds 3 && \
run pmc_fetch_c2 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch_c2 -o run --output-format csv -- $B --prewarm-s 0 && \
run pmc_write_c2 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write_c2 -o run --output-format csv -- $B --prewarm-s 0 && \
run pmc_fetch_c3 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch_c3 -o run --output-format csv -- $B --workload config3 --prewarm-s 0 && \
run pmc_write_c3 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write_c3 -o run --output-format csv -- $B --workload config3 --prewarm-s 0 && \
run pmc_sq_c3 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_SALU -d $OUT/pmc_sq_c3 -o run --output-format csv -- $B --workload config3 --prewarm-s 0 && \
run pmc_sq_c2 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_SALU -d $OUT/pmc_sq_c2 -o run --output-format csv -- $B --prewarm-s 0 && \
run pmc_sq_ric 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_SALU -d $OUT/pmc_sq_ric -o run --output-format csv -- python3 tools/bench_riccati.py --rounds 2 --iters 3 --prewarm-s 0
echo "prof_r02 rc=$?"
