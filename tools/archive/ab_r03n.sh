#!/bin/bash
# Round 3: the conditioned kernel at two waves per SIMD (packed images, SchedCondLSymP)
# for batches above one wave per SIMD: the LFT GPU tests on the product library, then
# the A/B on the developer library at B = 32,768 (0 = packed default, 92 = forced one
# wave) and B = 4,096 (0 = one wave, 91 = forced packed).   (ships libhop_amd_dev.so)
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 && \
HOP_DEV_BUILD=1 HOP_LIB=$PWD/time_opt_ilqr_amd/libhop_amd_dev.so timeout -k 10 300 python -u tools/ab_bench.py --variants 0,92 --batch 32768 --rounds 7 --iters 3 > $OUT/ab_32768.log 2>&1 && \
HOP_DEV_BUILD=1 HOP_LIB=$PWD/time_opt_ilqr_amd/libhop_amd_dev.so timeout -k 10 300 python -u tools/ab_bench.py --variants 0,91 --batch 4096 --rounds 9 --iters 10 > $OUT/ab_4096.log 2>&1
rc=$?; echo "rc=$rc"; exit $rc
