#!/bin/bash
# Round-6 GPU pass h: one-process A/Bs of two candidate changes against the product
# library: the congruence query's row offsets as three-address v_fma_f64 (fma3,
# config 2) and the small-s row-group kernel's two stage sweeps as one interleaved
# block (sw2, fp64 s = 5); parity of sw2 on the small-s and real-input tests.
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
HOP_LIB=tools/exp/libhop_sw2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_small_rowgroup.py tests/test_gpu_real_lin.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_sw2.log 2>&1 && \
timeout -k 10 600 python tools/ab_libs.py tools/exp/libhop_sw2.so tools/exp/libhop_head.so --only small_s5_f64_4096 --rounds 12 > $OUT/ab_sw2.jsonl 2> $OUT/ab_sw2.err && \
timeout -k 10 600 python tools/ab_libs.py tools/exp/libhop_fma3.so tools/exp/libhop_head.so --only config2 --rounds 12 > $OUT/ab_fma3.jsonl 2> $OUT/ab_fma3.err
rc=$?; echo "r06h_pass rc=$rc"
exit $rc
