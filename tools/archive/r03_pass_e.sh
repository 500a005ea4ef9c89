#!/bin/bash
# Round-3 pass E: full product GPU tests (fused hand-over default), then pass D
# (developer A/B incl. the fused / unfused config-2 launch, MFMA predict, SQ counters,
# Riccati stamps, product A/B against libhop_ab_base.so).
#   gpurun -- bash tools/r03_pass_e.sh <tag>     (ships libhop_amd_dev.so, libhop_ab_base.so)
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
bash tools/r03_pass_d.sh $1
rc=$?; echo "pass_e rc=$rc"; exit $rc
