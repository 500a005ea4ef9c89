#!/bin/bash
# Round-6 GPU pass g: the config-2 kernel with the step's LDS-DMA pieces spread through
# the update block (HOP_COND_DMAI, tools/exp/libhop_dmai.so): parity, then a one-process
# A/B against the product library.
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
HOP_LIB=tools/exp/libhop_dmai.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_real_lin.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_dmai.log 2>&1 && \
timeout -k 10 600 python tools/ab_libs.py tools/exp/libhop_dmai.so time_opt_ilqr_amd/libhop_amd.so --only config2 --rounds 12 > $OUT/ab_dmai.jsonl 2> $OUT/ab.err
rc=$?; echo "r06g_pass rc=$rc"
exit $rc
