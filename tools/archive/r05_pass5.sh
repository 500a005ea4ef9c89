#!/bin/bash
# Round-5 GPU pass 5: parity / rerun / configs tests, the rerun diagnosis, and the
# same-process A/B of the hot kernels against the round-3 and round-4 libraries and
# the query / symmetrisation variants.
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rerun.py tests/test_gpu_nonfinite.py tests/test_gpu_configs.py tests/test_gpu_traj.py -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest.log
case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 120 python tools/diag_rerun3.py > $OUT/diag.log 2>&1 || exit $?
timeout -k 10 400 python tools/ab_libs.py time_opt_ilqr_amd/libhop_amd.so time_opt_ilqr_amd/libhop_ab_base.so tools/exp/libhop_r04final.so tools/exp/libhop_r05_nowq.so tools/exp/libhop_r05_nosym.so tools/exp/libhop_r05_nowq_nosym.so tools/exp/libhop_r05_cq32.so --only config2,config3_tile64,select_traj_cf --rounds 7 > $OUT/ab.jsonl 2> $OUT/ab.err
echo "ab rc=$?" >> $OUT/pytest.log
exit $rc
