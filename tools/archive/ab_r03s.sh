#!/bin/bash
# Round 3: the Riccati step's Q image read inside the V [A|B] product block (QL, default)
# vs with the step's other reads (developer variant 96): the Riccati / J-curve GPU tests on
# the product library, then the interleaved A/B at B = 4,096.   (ships libhop_amd_dev.so)
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_forward.py -m gpu -x -v --timeout 120 --timeout-method thread -k "riccati or jcurve or bruteforce or value or select" > $OUT/pytest.log 2>&1 && \
HOP_DEV_BUILD=1 HOP_LIB=$PWD/time_opt_ilqr_amd/libhop_amd_dev.so timeout -k 10 300 python -u tools/bench_riccati.py --batch 4096 --variants 0,96 --rounds 11 > $OUT/ab_ric.jsonl 2>&1
rc=$?; echo "rc=$rc"; exit $rc
