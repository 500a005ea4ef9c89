#!/bin/bash
# Round-3 developer A/B: the conditioned-kernel schedules at config 2 (41 default
# without rerun, 52 SYM2 + reciprocal Newton, 47, 48) and the fp32-block kernel with
# its predict on the f32 matrix cores (57 MFMA vs 41, no rerun) at the config-5 s = 13
# bucket (5,462 problems) and the padded 16,384 launch; the MFMA variant's golden test;
# a kernel trace naming the MFMA kernel.  Ships libhop_amd_dev.so (un-ignore it).
#   gpurun -- bash tools/ab_r03c.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp HOP_DEV_BUILD=1 HOP_LIB=$PWD/time_opt_ilqr_amd/libhop_amd_dev.so
timeout -k 10 300 python -u tools/ab_bench.py --variants 0,60,58,52 --rounds 10 --iters 10 > $OUT/ab_c2.log 2>&1 && \
timeout -k 10 300 python -u tools/ab_bench.py --variants 41,57 --rounds 9 --iters 10 --dtype f32 --N 128 --batch 5462 > $OUT/ab_c5_s13.log 2>&1 && \
timeout -k 10 300 python -u tools/ab_bench.py --variants 0,56,41,57 --rounds 7 --iters 5 --dtype f32 --N 128 --batch 16384 > $OUT/ab_c5_pad.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 120 --timeout-method thread -k "mfma or config5" > $OUT/pytest_mfma.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_mfma -o run --output-format csv -- python3 -u tools/ab_bench.py --variants 57,41 --rounds 3 --iters 5 --dtype f32 --N 128 --batch 5462 > $OUT/trace_mfma.log 2>&1
rc=$?; echo "ab rc=$rc"; exit $rc
