#!/bin/bash
# Round-5 GPU pass 8: the library built with the DPP hazard pads elided
# (tools/nop_elide.py): GPU suite, then the A/B against the plain build.
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest_gpu.log
case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 700 python tools/ab_libs.py time_opt_ilqr_amd/libhop_amd.so tools/exp/libhop_r05_noelide.so time_opt_ilqr_amd/libhop_ab_base.so --only config2,select_traj_cf,config3_tile64,riccati_mode0,riccati_mode1,bruteforce_jcurve,linesearch_quad --rounds 11 --iters 5 > $OUT/ab.jsonl 2> $OUT/ab.err
echo "ab rc=$?" >> $OUT/pytest_gpu.log
exit $rc
