#!/bin/bash
# Round 3: the line search and outer loops after the two-lane rollout (tools/bench_forward.py),
# and SQ counters of the two-wave kernels (J curve at the bench shape, Riccati mode 0 at
# B = 32,768, the packed conditioned kernel at the config-4 shard).
#   gpurun -- bash tools/r03_pass_q.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
SQ1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_LDS SQ_BUSY_CYCLES"
timeout -k 10 400 python -u tools/bench_forward.py --system quadrotor --methods propagator,bruteforce --cpu-seconds 3 > $OUT/fwd.jsonl 2> $OUT/fwd.err && \
timeout -s KILL 120 rocprofv3 --pmc $SQ1 -d $OUT/bf/pmc_sq -o run --output-format csv -- python3 bench.py --workload bruteforce --steps 2 --warmup 1 --no-cpu-baseline --no-h2d --no-anchor --no-alt --prewarm-s 0 > $OUT/bf.pmc.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc $SQ1 -d $OUT/ric/pmc_sq -o run --output-format csv -- python3 tools/bench_riccati.py --batch 32768 --rounds 1 --iters 2 --prewarm-s 0 > $OUT/ric.pmc.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc $SQ1 -d $OUT/c4/pmc_sq -o run --output-format csv -- python3 bench.py --batch 32768 --steps 2 --warmup 1 --no-cpu-baseline --no-h2d --no-anchor --no-alt --prewarm-s 0 > $OUT/c4.pmc.log 2>&1
rc=$?
(echo "== riccati_fast_jcurve (bruteforce bench)"; python3 tools/pmc_summary.py $OUT/bf "riccati_fast_jcurve"; echo "== riccati_fast_kernel<0 (B = 32768)"; python3 tools/pmc_summary.py $OUT/ric "riccati_fast_kernel<0"; echo "== lft_cond_kernel<SchedCondLSymP (B = 32768)"; python3 tools/pmc_summary.py $OUT/c4 "SchedCondLSymP") > $OUT/summary.txt 2>&1
echo "rc=$rc"; exit $rc
