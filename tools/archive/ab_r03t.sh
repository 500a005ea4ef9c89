#!/bin/bash
# Round 3: the J curve (two waves per SIMD) with the Qxx start read in the V [A|B] block
# (default) vs with the step's reads (developer variant 96); Riccati / J-curve GPU tests on
# the product library first.   (ships libhop_amd_dev.so)
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_forward.py -m gpu -x -v --timeout 120 --timeout-method thread -k "riccati or jcurve or bruteforce or value or select" > $OUT/pytest.log 2>&1 && \
HOP_DEV_BUILD=1 HOP_LIB=$PWD/time_opt_ilqr_amd/libhop_amd_dev.so timeout -k 10 300 python -u tools/ab_jcurve.py --variants 0,96 --rounds 10 > $OUT/ab_jc.log 2>&1 && \
HOP_DEV_BUILD=1 HOP_LIB=$PWD/time_opt_ilqr_amd/libhop_amd_dev.so timeout -k 10 300 python -u tools/bench_riccati.py --batch 32768 --rounds 7 --iters 3 > $OUT/ric_32768.jsonl 2>&1
rc=$?; echo "rc=$rc"; exit $rc
