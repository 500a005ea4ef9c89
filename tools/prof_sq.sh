#!/bin/bash
# SQ PMC pass (issue vs wait breakdown) of one command, plus its kernel-trace stats.
#   bash tools/prof_sq.sh <outdir> <cmd...>
set -o pipefail
OUT=$1; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- "$@" > $OUT/trace.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM -d $OUT/pmc_sq -o run --output-format csv -- "$@" > $OUT/pmc_sq.log 2>&1
