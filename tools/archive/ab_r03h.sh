#!/bin/bash
# Round 3: the J curve at two waves per SIMD (developer variant 85: one step image,
# batch-shared Q image, Q rows from LDS; 247 VGPRs, 77,824 B LDS per workgroup) vs
# the product schedule: interleaved timing + bitwise check, then SQ counters of both.
#   gpurun -- bash tools/ab_r03h.sh <tag>     (ships libhop_amd_dev.so)
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp HOP_DEV_BUILD=1 HOP_LIB=$PWD/time_opt_ilqr_amd/libhop_amd_dev.so
SQ1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_LDS SQ_BUSY_CYCLES"
timeout -k 10 300 python -u tools/ab_jcurve.py --variants 0,85 --rounds 8 > $OUT/ab_jc.log 2>&1 && \
timeout -k 10 300 python -u tools/ab_jcurve.py --variants 0,85 --rounds 4 --batch 1000 > $OUT/ab_jc_1000.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc $SQ1 -d $OUT/v85/pmc_sq -o run --output-format csv -- python3 tools/ab_jcurve.py --variants 85 --rounds 1 --iters 1 > $OUT/pmc_v85.log 2>&1
rc=$?
python3 tools/pmc_summary.py $OUT/v85 "riccati_fast_jcurve" > $OUT/summary.txt 2>&1
echo "ab rc=$rc"; exit $rc
