#!/bin/bash
# Round 3: SYM2 on the fp32-block conditioned kernel (config 5's s = 13 part; developer
# variant 95 = plain converting reads) and the packed-layout hand-over test; the LFT / config
# GPU tests on the product library, then the A/B.   (ships libhop_amd_dev.so)
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 && \
HOP_DEV_BUILD=1 HOP_LIB=$PWD/time_opt_ilqr_amd/libhop_amd_dev.so timeout -k 10 300 python -u tools/ab_bench.py --variants 0,95 --rounds 9 --iters 10 --dtype f32 --N 128 --batch 5462 > $OUT/ab_c5_s13.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload config5 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err
rc=$?; echo "rc=$rc"; exit $rc
