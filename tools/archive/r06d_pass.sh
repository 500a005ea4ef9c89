#!/bin/bash
# Round-6 GPU pass d: the gain and small-s tests on the rsq-equilibrated Riccati solve
# and HOP_OPT_SMALL_LANE, a one-process A/B against round 5's library (8 rounds, both
# orders), and the small-s batch sweep with the trajectory form.
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_gains.py tests/test_gpu_small_rowgroup.py -v -s --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 && \
timeout -k 10 900 python tools/ab_libs.py time_opt_ilqr_amd/libhop_amd.so time_opt_ilqr_amd/libhop_ab_base.so --only config2,riccati_mode0,riccati_mode1,bruteforce_jcurve,select_traj_cf,small_s5_f64_4096 --rounds 8 > $OUT/ab_vs_r05.jsonl 2> $OUT/ab.err && \
timeout -k 10 600 python tools/bench_small_rg.py --out $OUT/small_rg.jsonl > $OUT/small_rg.log 2>&1
rc=$?; echo "r06d_pass rc=$rc"
exit $rc
