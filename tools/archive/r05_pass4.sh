#!/bin/bash
# Round-5 GPU pass 4: rerun + select tests on the equilibrated sweep, the escalated
# problem dumped for the 50-digit check, a kernel trace of the rerun bench.
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_rerun.py tests/test_gpu_real_lin.py tests/test_gpu_parity.py tests/test_gpu_nonfinite.py -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest.log
case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 120 python tools/dump_escalation_case.py $OUT/esc.npz 5e-7 > $OUT/esc.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o rerun -- python3 tools/bench_rerun.py tools/exp/libhop_r05_sym2.so time_opt_ilqr_amd/libhop_amd.so --rounds 5 > $OUT/rerun.jsonl 2> $OUT/rerun.err
echo "prof rc=$?" >> $OUT/pytest.log
exit $rc
