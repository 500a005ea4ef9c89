#!/bin/bash
# Forward pass / outer loop / linearisation measurements on the GPU box (repo root):
#   bash tools/prof_forward.sh <tag>  -> gpurun_out/<tag>/{fwd.jsonl, lin.jsonl, ric.jsonl, fwd_trace/}
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python3 tools/bench_forward.py --cpu-seconds 5 > $OUT/fwd.jsonl 2> $OUT/fwd.err && \
timeout -k 10 300 python3 tools/bench_linearize.py --system all --both --cpu-seconds 3 > $OUT/lin.jsonl 2> $OUT/lin.err && \
timeout -k 10 300 python3 tools/bench_riccati.py > $OUT/ric.jsonl 2> $OUT/ric.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/fwd_trace -o run --output-format csv -- \
  python3 tools/bench_forward.py --system quadrotor --cpu-seconds 0 > $OUT/fwd_trace.log 2>&1
echo "prof_forward rc=$?"
