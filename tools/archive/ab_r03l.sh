#!/bin/bash
# Round 3: the J-curve GPU tests on the product library (two waves per SIMD + XCD-grouped
# horizons by default), the A/B against round-robin XCDs (developer variant 88) and the
# one-wave layout (86), and the bruteforce bench line.   (ships libhop_amd_dev.so)
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_configs.py -m gpu -x -v --timeout 120 --timeout-method thread -k "bruteforce or jcurve or plots" > $OUT/pytest.log 2>&1 && \
HOP_DEV_BUILD=1 HOP_LIB=$PWD/time_opt_ilqr_amd/libhop_amd_dev.so timeout -k 10 300 python -u tools/ab_jcurve.py --variants 0,88,86 --rounds 8 > $OUT/ab_jc.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload bruteforce > $OUT/bench_bf.log 2>&1
rc=$?; echo "rc=$rc"; exit $rc
