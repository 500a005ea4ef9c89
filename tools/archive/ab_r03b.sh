#!/bin/bash
# Round-3 A/B: library A (before) vs library B (after) on every bench workload, and
# the conditioned-kernel schedules of the developer library.  gpurun_out/$1/.
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 400 python -u tools/ab_libs.py time_opt_ilqr_amd/libhop_ab_base.so time_opt_ilqr_amd/libhop_ab_al8.so --rounds 7 > $OUT/ab_libs.log 2>&1 && \
HOP_DEV_BUILD=1 HOP_LIB=$PWD/time_opt_ilqr_amd/libhop_amd_dev.so timeout -k 10 300 python -u tools/ab_bench.py --variants ${2:-41,45,47,48,49,50,51} --rounds 9 --iters 10 > $OUT/ab.log 2>&1 && \
HOP_DEV_BUILD=1 HOP_LIB=$PWD/time_opt_ilqr_amd/libhop_amd_dev.so timeout -k 10 300 python -u tools/ab_bench.py --variants ${2:-41,45,47,48,49,50,51} --rounds 5 --iters 3 --batch 32768 > $OUT/ab_32k.log 2>&1
rc=$?; echo "ab rc=$rc"
[ $rc -eq 0 ] && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "legacy or edge_cases" > $OUT/pytest_new.log 2>&1; rc=$?; echo "tests rc=$rc"; exit $rc
