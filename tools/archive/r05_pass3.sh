#!/bin/bash
# Round-5 GPU pass 3: the rerun tests, a kernel trace of the rerun bench.
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rerun.py tests/test_gpu_real_lin.py -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest.log
if [ $rc -ne 124 ] && [ $rc -ne 137 ] && [ $rc -ne 134 ] && [ $rc -ne 139 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o rerun -- python3 tools/bench_rerun.py tools/exp/libhop_r05_sym2.so time_opt_ilqr_amd/libhop_amd.so --rounds 3 > $OUT/rerun.jsonl 2> $OUT/rerun.err
  echo "prof rc=$?" >> $OUT/pytest.log
fi
exit $rc
