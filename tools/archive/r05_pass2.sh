#!/bin/bash
# Round-5 GPU pass 2: capture, GPU tests, rerun cost, symmetrisation-interval A/B.
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 300 python -u tools/real_lin_capture.py $OUT 64 32 > $OUT/capture.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest.log
if [ $rc -ne 124 ] && [ $rc -ne 137 ] && [ $rc -ne 134 ] && [ $rc -ne 139 ]; then
  timeout -k 10 300 python -u tools/bench_rerun.py tools/exp/libhop_r05_sym2.so time_opt_ilqr_amd/libhop_amd.so > $OUT/rerun.jsonl 2> $OUT/rerun.err && \
  timeout -k 10 900 python -u tools/ab_libs.py tools/exp/libhop_r05_sym8.so tools/exp/libhop_r05_sym4.so tools/exp/libhop_r05_sym2.so tools/exp/libhop_r05_sym2ns.so tools/exp/libhop_r05_sym1.so --only config2,select_traj_cf,config4_shard --rounds 9 > $OUT/ab_sym.jsonl 2> $OUT/ab_sym.err
  echo "post rc=$?" >> $OUT/pytest.log
fi
exit $rc
