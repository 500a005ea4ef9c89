#!/bin/bash
# Round 3: the GPU suite on the product library with the two-wave J curve default,
# the J-curve A/B against the one-wave layout (developer variant 86), and the
# bruteforce bench line.   gpurun -- bash tools/ab_r03i.sh <tag>   (ships libhop_amd_dev.so)
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 && \
HOP_DEV_BUILD=1 HOP_LIB=$PWD/time_opt_ilqr_amd/libhop_amd_dev.so timeout -k 10 300 python -u tools/ab_jcurve.py --variants 0,86 --rounds 8 > $OUT/ab_jc.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload bruteforce > $OUT/bench_bf.log 2>&1
rc=$?; echo "rc=$rc"; exit $rc
