#!/bin/bash
# Round-5 GPU pass 6: the rerun tests, DMA-placement A/B on config 2.
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rerun.py -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest.log
case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 400 python tools/ab_libs.py time_opt_ilqr_amd/libhop_amd.so tools/exp/libhop_r05_nodma.so tools/exp/libhop_r05_dmasplit.so tools/exp/libhop_r05_nowq_nosym.so time_opt_ilqr_amd/libhop_ab_base.so --only config2,select_traj_cf --rounds 9 > $OUT/ab.jsonl 2> $OUT/ab.err
echo "ab rc=$?" >> $OUT/pytest.log
exit $rc
