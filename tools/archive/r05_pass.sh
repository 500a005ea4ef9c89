#!/bin/bash
# Round-5 GPU pass: real-input capture, GPU tests, same-process library A/B.
#   gpurun -- bash tools/r05_pass.sh <tag> [ab libs...]     (outputs under gpurun_out/<tag>/)
set -o pipefail
OUT=gpurun_out/$1
shift
mkdir -p $OUT
timeout -k 10 300 python -u tools/real_lin_capture.py $OUT 64 32 > $OUT/capture.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest.log
if [ $# -gt 0 ] && [ $rc -ne 124 ] && [ $rc -ne 137 ] && [ $rc -ne 134 ] && [ $rc -ne 139 ]; then
  timeout -k 10 600 python -u tools/ab_libs.py "$@" --rounds 7 > $OUT/ab.jsonl 2> $OUT/ab.err
  echo "ab rc=$?" >> $OUT/ab.err
fi
exit $rc
