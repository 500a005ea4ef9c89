#!/bin/bash
# Round-6 GPU pass b: the GPU suite, smoke, the default bench line, the fp64 s <= 5
# crossover table (tools/bench_small_rg.py).
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
prc=$?
echo "pytest rc=$prc" >> $OUT/pytest.log
if [ $prc -ne 0 ] && [ $prc -ne 1 ]; then exit $prc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err && \
timeout -k 10 600 python tools/bench_small_rg.py --out $OUT/small_rg.jsonl > $OUT/small_rg.log 2>&1
rc=$?; echo "r06b_pass rc=$rc pytest=$prc"
exit $rc
