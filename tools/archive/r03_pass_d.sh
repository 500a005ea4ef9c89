#!/bin/bash
# Round-3 pass D: developer A/B (tools/ab_r03c.sh), SQ counters + Riccati stamps
# (tools/prof_r03_ric.sh), product A/B against libhop_ab_base.so with alternating order.
#   gpurun -- bash tools/r03_pass_d.sh <tag>     (ships libhop_amd_dev.so, libhop_ab_base.so)
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
bash tools/ab_r03c.sh $1/dev; r1=$?
bash tools/prof_r03_ric.sh $1/prof; r2=$?
timeout -k 10 600 python -u tools/ab_libs.py time_opt_ilqr_amd/libhop_amd.so time_opt_ilqr_amd/libhop_ab_base.so --rounds 10 --only bruteforce_jcurve,riccati_mode0,riccati_mode1,select_traj_cf,config2 > $OUT/ab_libs.log 2>&1; r3=$?
echo "pass_d rc=$r1 $r2 $r3"; exit $(( r1 | r2 | r3 ))
