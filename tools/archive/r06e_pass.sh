#!/bin/bash
# Round-6 GPU pass e: the whole GPU suite after routing fp64 small-s trajectory-form
# batches through hop_augment + the row-group kernel, the small-s batch sweep, and
# the select + gains and default bench lines.
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu --maxfail 15 -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 && \
timeout -k 10 300 python tools/bench_small_rg.py --out $OUT/small_rg.jsonl > $OUT/small_rg.log 2>&1 && \
timeout -k 10 300 python bench.py --workload select_gains --no-cpu-baseline > $OUT/bench_sg.json 2> $OUT/bench_sg.err
rc=$?; echo "r06e_pass rc=$rc"
exit $rc
