#!/bin/bash
# Round-3 pass B: product library A/B (libhop_ab_base.so = before the lane-sum
# change) on the Riccati / J-curve / trajectory workloads, the affected GPU tests,
# the developer A/B of tools/ab_r03c.sh, and the SQ / stamp profile of tools/prof_r03_ric.sh.
#   gpurun -- bash tools/r03_pass_b.sh <tag>     (ships libhop_amd_dev.so and libhop_ab_base.so)
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 400 python -u tools/ab_libs.py time_opt_ilqr_amd/libhop_ab_base.so time_opt_ilqr_amd/libhop_amd.so --rounds 5 --only bruteforce_jcurve,riccati_mode0,riccati_mode1,select_traj_cf,config2 > $OUT/ab_libs.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "riccati or bruteforce or traj or jcurve or select or legacy" > $OUT/pytest_sub.log 2>&1 && \
bash tools/ab_r03c.sh $1/dev && \
bash tools/prof_r03_ric.sh $1/prof
rc=$?; echo "pass_b rc=$rc"; exit $rc
