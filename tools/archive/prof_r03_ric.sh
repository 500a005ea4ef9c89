#!/bin/bash
# Round 3: SQ counters of the Riccati family and the hot kernel (product library),
# then section stamps of the exact-size Riccati kernel in modes 0 and 1 (developer
# library, shipped only for this pass).
#   gpurun -- bash tools/prof_r03_ric.sh <tag>        (outputs under gpurun_out/<tag>/)
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
SQ1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_SALU"
pmc() {  # name, command...
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc $SQ1 -d $OUT/$n/pmc_sq -o run --output-format csv -- "$@" > $OUT/$n.pmc.log 2>&1
}
pmc ric python3 tools/bench_riccati.py --rounds 2 --iters 3 --prewarm-s 0 && \
pmc bf python3 bench.py --workload bruteforce --steps 2 --warmup 1 --no-cpu-baseline --no-h2d --no-anchor --no-alt --prewarm-s 0 && \
pmc c2 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-h2d --no-anchor --no-alt --prewarm-s 0 && \
HOP_DEV_BUILD=1 HOP_LIB=$PWD/time_opt_ilqr_amd/libhop_amd_dev.so timeout -k 10 120 python3 -u tools/stamps_riccati.py --mode 0 > $OUT/stamps_ric0.log 2>&1 && \
HOP_DEV_BUILD=1 HOP_LIB=$PWD/time_opt_ilqr_amd/libhop_amd_dev.so timeout -k 10 120 python3 -u tools/stamps_riccati.py --mode 1 > $OUT/stamps_ric1.log 2>&1
rc=$?
for k in "riccati_fast_kernel<0, false" "riccati_fast_kernel<1, true"; do echo "== $k"; python3 tools/pmc_summary.py $OUT/ric "$k"; done > $OUT/summary.txt
echo "== riccati_fast_jcurve_kernel" >> $OUT/summary.txt; python3 tools/pmc_summary.py $OUT/bf "riccati_fast_jcurve" >> $OUT/summary.txt
echo "== lft_cond_kernel" >> $OUT/summary.txt; python3 tools/pmc_summary.py $OUT/c2 "lft_cond_kernel" >> $OUT/summary.txt
echo "prof rc=$rc"
exit $rc
