#!/bin/bash
# Round-3 developer A/B pass of the conditioned kernel (ships libhop_amd_dev.so:
# run with the dev library un-ignored).  Outputs under gpurun_out/$1/.
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export HOP_DEV_BUILD=1 HOP_LIB=$PWD/time_opt_ilqr_amd/libhop_amd_dev.so
V=${2:-41,45,40,44}
timeout -k 10 300 python -u tools/ab_bench.py --variants $V --rounds 9 --iters 10 > $OUT/ab.log 2>&1 && \
timeout -k 10 300 python -u tools/ab_bench.py --variants $V --rounds 5 --iters 3 --batch 32768 > $OUT/ab_32k.log 2>&1 && \
timeout -k 10 120 python -u tools/stamps.py --cond > $OUT/stamps42.log 2>&1 && \
timeout -k 10 120 python -u tools/stamps.py --cond --variant 46 > $OUT/stamps46.log 2>&1
rc=$?; echo "ab rc=$rc"; exit $rc
