#!/bin/bash
# One GPU-box pass: full GPU tests, smoke, default bench (with CPU baseline), rocprofv3 passes.
#   gpurun -- bash tools/round_gpu.sh <tag>      (outputs under gpurun_out/<tag>/)
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -q > $OUT/pytest.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err && \
bash tools/prof1.sh $1/prof
echo "round_gpu rc=$?"
