#!/bin/bash
# Round-6 GPU pass l: the s = 13 fp64 predict on v_mfma_f64_16x16x4_f64
# (HOP_COND_MFMA64, tools/exp/libhop_mf64.so): parity, a one-process A/B against the
# product library, and the MFMA counters of the variant's config-2 kernel.
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
HOP_LIB=tools/exp/libhop_mf64.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_real_lin.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_mf64.log 2>&1 && \
timeout -k 10 600 python tools/ab_libs.py tools/exp/libhop_mf64.so time_opt_ilqr_amd/libhop_amd.so --only config2 --rounds 12 > $OUT/ab_mf64.jsonl 2> $OUT/ab.err && \
export HOP_LIB=tools/exp/libhop_mf64.so && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_F64 SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES -d $OUT/pmc_mf64 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-h2d --no-anchor --no-alt --prewarm-s 0 > $OUT/pmc_mf64.log 2>&1
rc=$?; echo "r06l_pass rc=$rc"
exit $rc
