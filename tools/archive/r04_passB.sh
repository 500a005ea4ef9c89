#!/bin/bash
# Round 4 pass B (after tools/r04_passA.sh): the Riccati passes, the outer loop, the
# rocprofv3 kernel traces and PMC traffic passes (tools/prof_r04.sh) and the MFMA
# utilisation PMC pass of the config-5 MFMA predict variant (tools/mfma_pmc.py, developer
# library).
#   gpurun --timeout 1200 -- bash tools/r04_passB.sh <tag>
set -o pipefail
T=$1
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/bench_riccati.py > $OUT/riccati.jsonl 2> $OUT/riccati.err && \
timeout -k 10 400 python tools/bench_forward.py --system quadrotor --cpu-seconds 0 > $OUT/fwd.jsonl 2> $OUT/fwd.err && \
bash tools/prof_r04.sh $T/prof && \
HOP_LIB=time_opt_ilqr_amd/libhop_amd_dev.so timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/mfma -o run --output-format csv -- python3 tools/mfma_pmc.py > $OUT/mfma.log 2>&1
rc=$?; echo "r04_passB rc=$rc"; exit $rc
