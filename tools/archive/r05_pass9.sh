#!/bin/bash
# Round-5 GPU pass 9: the LDS-DMA pieces sharing M0 (instruction offsets): the GPU suite,
# then the A/B against the previous library.
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest_gpu.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 600 python tools/ab_libs.py time_opt_ilqr_amd/libhop_amd.so tools/exp/libhop_r05_elide1.so --only config2,select_traj_cf,config4_shard,riccati_mode0,riccati_mode1,bruteforce_jcurve --rounds 11 --iters 5 > $OUT/ab.jsonl 2> $OUT/ab.err
echo "ab rc=$?" >> $OUT/pytest_gpu.log
