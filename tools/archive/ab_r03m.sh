#!/bin/bash
# Round 3: the exact-size Riccati kernel at two waves per SIMD for batches above one
# wave per SIMD (batch-shared Q): the Riccati / J-curve GPU tests on the product
# library, then the A/B on the developer library at B = 32,768 (0 = default = two
# waves, 89 = one wave) and B = 4,096 (0 = one wave, 90 = forced two waves).
#   gpurun -- bash tools/ab_r03m.sh <tag>     (ships libhop_amd_dev.so)
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_forward.py -m gpu -x -v --timeout 120 --timeout-method thread -k "riccati or jcurve or bruteforce or value" > $OUT/pytest.log 2>&1 && \
HOP_DEV_BUILD=1 HOP_LIB=$PWD/time_opt_ilqr_amd/libhop_amd_dev.so timeout -k 10 300 python -u tools/bench_riccati.py --batch 32768 --variants 0,89 --rounds 7 --iters 3 > $OUT/ab_ric_32768.jsonl 2>&1 && \
HOP_DEV_BUILD=1 HOP_LIB=$PWD/time_opt_ilqr_amd/libhop_amd_dev.so timeout -k 10 300 python -u tools/bench_riccati.py --batch 4096 --variants 0,90 --rounds 7 > $OUT/ab_ric_4096.jsonl 2>&1
rc=$?; echo "rc=$rc"; exit $rc
