#!/bin/bash
# Round 3: packed [Qux | Quu] Riccati rows (default of the developer build) vs the
# separate rows (developer variant 84): the GPU suite on the developer library, the
# interleaved Riccati / J-curve timing and SQ counters per variant.
#   gpurun -- bash tools/ab_r03g.sh <tag>     (ships libhop_amd_dev.so)
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp HOP_DEV_BUILD=1 HOP_LIB=$PWD/time_opt_ilqr_amd/libhop_amd_dev.so
SQ1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_SALU"
timeout -k 10 400 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_riccati.py --variants 0,84 --jcurve --rounds 9 > $OUT/ab_ric.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc $SQ1 -d $OUT/v0/pmc_sq -o run --output-format csv -- python3 tools/bench_riccati.py --variants 0 --jcurve --rounds 1 --iters 2 --prewarm-s 0 > $OUT/pmc_v0.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc $SQ1 -d $OUT/v84/pmc_sq -o run --output-format csv -- python3 tools/bench_riccati.py --variants 84 --jcurve --rounds 1 --iters 2 --prewarm-s 0 > $OUT/pmc_v84.log 2>&1
rc=$?
for v in v0 v84; do for k in "riccati_fast_kernel<0, false" "riccati_fast_kernel<1, true" "riccati_fast_jcurve"; do echo "== $v $k"; python3 tools/pmc_summary.py $OUT/$v "$k"; done; done > $OUT/summary.txt 2>&1
echo "ab rc=$rc"; exit $rc
