#!/bin/bash
# Round-5 GPU pass 10: the closed-form kernel's symmetrisation reads sharing their
# round trip: the trajectory / real-input / rerun tests, then the A/B.
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_traj.py tests/test_gpu_real_lin.py tests/test_gpu_rerun.py tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 500 python tools/ab_libs.py time_opt_ilqr_amd/libhop_amd.so tools/exp/libhop_r05_m0.so time_opt_ilqr_amd/libhop_ab_base.so --only select_traj_cf,config2 --rounds 15 --iters 5 > $OUT/ab.jsonl 2> $OUT/ab.err
echo "ab rc=$?" >> $OUT/pytest.log
