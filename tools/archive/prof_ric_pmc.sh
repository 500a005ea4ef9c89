#!/bin/bash
# PMC pass over the Riccati bench (tools/bench_riccati.py, default lib only).
#   bash tools/prof_ric_pmc.sh <tag>      -> gpurun_out/<tag>/
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
B="python3 tools/bench_riccati.py --rounds 2 --iters 3 --prewarm-s 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B > $OUT/trace.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_SALU -d $OUT/pmc_sq -o run --output-format csv -- $B > $OUT/pmc_sq.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_BUSY_CYCLES -d $OUT/pmc_sq2 -o run --output-format csv -- $B > $OUT/pmc_sq2.log 2>&1
rc=$?
for k in "riccati_fast_kernel<0, false" "riccati_fast_kernel<1, true"; do echo "== $k"; python3 tools/pmc_summary.py $OUT "$k"; done
echo "prof rc=$rc"
exit $rc
