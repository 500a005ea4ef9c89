#!/bin/bash
# Round 3: J-curve XCD grouping A/B (developer variant 83) with its FETCH_SIZE per variant.
#   gpurun -- bash tools/ab_r03f.sh <tag>     (ships libhop_amd_dev.so)
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp HOP_DEV_BUILD=1 HOP_LIB=$PWD/time_opt_ilqr_amd/libhop_amd_dev.so
timeout -k 10 300 python -u tools/ab_jcurve.py --variants 0,83 --rounds 8 > $OUT/ab_jc.log 2>&1 && \
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 tools/ab_jcurve.py --variants 0,83 --rounds 1 --iters 1 > $OUT/pmc.log 2>&1
rc=$?; echo "ab rc=$rc"; exit $rc
