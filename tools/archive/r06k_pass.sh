#!/bin/bash
# Round-6 GPU pass k: the s = 13 conditioned kernel with its two sweeps as one
# interleaved block behind one Q/QT read (HOP_COND_SWEEP2, tools/exp/libhop_c2sw.so):
# parity, then a one-process A/B against the product library.
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
HOP_LIB=tools/exp/libhop_c2sw.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_real_lin.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_c2sw.log 2>&1 && \
timeout -k 10 600 python tools/ab_libs.py tools/exp/libhop_c2sw.so time_opt_ilqr_amd/libhop_amd.so --only config2 --rounds 12 > $OUT/ab_c2sw.jsonl 2> $OUT/ab.err
rc=$?; echo "r06k_pass rc=$rc"
exit $rc
