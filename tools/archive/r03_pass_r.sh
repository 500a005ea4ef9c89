#!/bin/bash
# Round 3: forward / configs GPU tests after the two-lane gating (one wave per SIMD).
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_configs.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "rc=$rc"; exit $rc
