#!/bin/bash
# Round-3 pass C: full product GPU tests, product A/B against libhop_ab_base.so
# (round-3 start: halved-sum default, butterfly row sums), the developer A/B
# (tools/ab_r03c.sh: schedules, MFMA predict) and the SQ / stamp profile
# (tools/prof_r03_ric.sh).  Each group runs only if the one before passed.
#   gpurun -- bash tools/r03_pass_c.sh <tag>     (ships libhop_amd_dev.so, libhop_ab_base.so)
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 && \
timeout -k 10 600 python -u tools/ab_libs.py time_opt_ilqr_amd/libhop_amd.so time_opt_ilqr_amd/libhop_ab_base.so --rounds 9 --only bruteforce_jcurve,riccati_mode0,riccati_mode1,select_traj_cf,config2 > $OUT/ab_libs.log 2>&1 && \
bash tools/ab_r03c.sh $1/dev && \
bash tools/prof_r03_ric.sh $1/prof
rc=$?; echo "pass_c rc=$rc"; exit $rc
