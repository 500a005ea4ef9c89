#!/bin/bash
# Round 4 pass A: GPU tests + smoke + bench lines (tools/gpu_pass.sh), real-linearisation
# parity at batch scale, the symmetrisation / query A/Bs (developer library) and the real
# quadrotor select timing.   gpurun --timeout 1200 -- bash tools/r04_passA.sh <tag>
set -o pipefail
T=$1
OUT=gpurun_out/$T
mkdir -p $OUT
bash tools/gpu_pass.sh $T && \
timeout -k 10 300 python tools/real_lin_parity.py 4096 $OUT/real_lin.jsonl > $OUT/real_lin.log 2>&1 && \
timeout -k 10 300 python tools/ab_traj.py --system quadrotor --variants 0 --rounds 5 > $OUT/ab_traj_quad.log 2>&1 && \
HOP_LIB=time_opt_ilqr_amd/libhop_amd_dev.so timeout -k 10 300 python tools/ab_bench.py --variants 0,96,0,96 > $OUT/ab_sym.log 2>&1 && \
HOP_LIB=time_opt_ilqr_amd/libhop_amd_dev.so timeout -k 10 300 python tools/ab_traj.py --system synthetic --variants 0,95,94 --rounds 9 > $OUT/ab_traj_syn.log 2>&1
rc=$?; echo "r04_passA rc=$rc"; exit $rc
