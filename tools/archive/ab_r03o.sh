#!/bin/bash
# Round 3: the quadrotor line search at two lanes per rollout (default) vs one lane
# (developer variant 93): the forward GPU tests on the product library, then the
# interleaved A/B with a bitwise check.   (ships libhop_amd_dev.so)
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 && \
HOP_DEV_BUILD=1 HOP_LIB=$PWD/time_opt_ilqr_amd/libhop_amd_dev.so timeout -k 10 300 python -u tools/ab_linesearch.py --variants 0,93 > $OUT/ab_ls.log 2>&1
rc=$?; echo "rc=$rc"; exit $rc
