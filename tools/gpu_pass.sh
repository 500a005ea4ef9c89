#!/bin/bash
# One GPU-box pass: GPU tests, smoke, the bench workloads.
#   gpurun -- bash tools/gpu_pass.sh <tag> [pytest -k expr]    (outputs under gpurun_out/<tag>/)
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
K=${2:+-k "$2"}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $K > $OUT/pytest.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err && \
timeout -k 10 300 python bench.py --workload config3 --no-cpu-baseline > $OUT/bench_config3.json 2> $OUT/bench_config3.err && \
timeout -k 10 300 python bench.py --workload config5 --no-cpu-baseline > $OUT/bench_config5.json 2> $OUT/bench_config5.err && \
timeout -k 10 300 python bench.py --workload select_gains --no-cpu-baseline > $OUT/bench_sg.json 2> $OUT/bench_sg.err && \
timeout -k 10 300 python bench.py --batch 32768 --no-cpu-baseline > $OUT/bench_c4shard.json 2> $OUT/bench_c4shard.err && \
timeout -k 10 300 python bench.py --workload bruteforce --steps 5 > $OUT/bench_bf.json 2> $OUT/bench_bf.err
rc=$?; echo "gpu_pass rc=$rc"
# a 1-GPU box must refuse --gpus 2 (exit 2) instead of timing one rank
timeout -k 10 120 python bench.py --gpus 2 --no-cpu-baseline > $OUT/bench_gpus2.out 2> $OUT/bench_gpus2.err; echo "gpus2 rc=$?" >> $OUT/bench_gpus2.err
exit $rc
