#!/bin/bash
# PMC passes (separate runs, no trace domains) for one bench configuration.
#   bash tools/prof_pmc.sh <tag> <bench args...>
OUT=gpurun_out/$1
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --prewarm-s 0 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B > $OUT/trace.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_SALU -d $OUT/pmc_sq -o run --output-format csv -- $B > $OUT/pmc_sq.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- $B > $OUT/pmc_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- $B > $OUT/pmc_write.log 2>&1
echo "prof rc=$?"
