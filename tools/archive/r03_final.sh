#!/bin/bash
# Round 3 final pass on the product library: GPU tests + smoke + every bench line
# (tools/gpu_pass.sh), the Riccati passes and J curve (tools/bench_riccati.py), the
# quadrotor line search and outer loop with both select methods (tools/bench_forward.py).
#   gpurun -- bash tools/r03_final.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
bash tools/gpu_pass.sh $1 && \
timeout -k 10 300 python -u tools/bench_riccati.py --jcurve --rounds 9 > $OUT/riccati.jsonl 2> $OUT/riccati.err && \
timeout -k 10 400 python -u tools/bench_forward.py --system quadrotor --methods propagator,bruteforce --cpu-seconds 3 > $OUT/fwd.jsonl 2> $OUT/fwd.err
rc=$?; echo "final rc=$rc"; exit $rc
