#!/bin/bash
# Round 3: rocprofv3 --kernel-trace --stats of the bench commands themselves (warm clocks:
# bench.py's own pre-warm and warm-up), so the committed kernel averages and the bench
# line's HIP-event kernel_ms come from the same run.  gpurun -- bash tools/prof_r03_bench.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/c2.json 2> $OUT/c2.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/bf -o run --output-format csv -- python3 bench.py --workload bruteforce --steps 5 --no-cpu-baseline > $OUT/bf.json 2> $OUT/bf.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/sg -o run --output-format csv -- python3 bench.py --workload select_gains --no-cpu-baseline > $OUT/sg.json 2> $OUT/sg.err && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py -m gpu -x -v --timeout 120 --timeout-method thread -k "integration_md or legacy" > $OUT/pytest.log 2>&1
rc=$?; echo "prof_bench rc=$rc"; exit $rc
