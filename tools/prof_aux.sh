#!/bin/bash
# rocprofv3 kernel-trace stats of the secondary paths (GPU box, repo root):
#   config 3 (small-s kernel), trajectory form (fused / builder; config 2 and 3 shapes), Riccati passes.
#   bash tools/prof_aux.sh <tag>     -> gpurun_out/<tag>/{cfg3,traj,traj3,riccati}/
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/cfg3 -o run --output-format csv -- \
  python3 bench.py --s 5 --m 1 --N 200 --batch 65536 --dtype f32 --t-min 20 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/cfg3.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/traj -o run --output-format csv -- \
  python3 tools/bench_traj.py --rounds 3 > $OUT/traj.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/traj3 -o run --output-format csv -- \
  python3 tools/bench_traj.py --n 4 --m 1 --N 200 --batch 65536 --dtype f32 --rounds 3 > $OUT/traj3.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/riccati -o run --output-format csv -- \
  python3 tools/bench_riccati.py > $OUT/riccati.log 2>&1
echo "prof_aux rc=$?"
