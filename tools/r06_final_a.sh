#!/bin/bash
# Round 6 evidence pass A: the whole GPU suite, smoke, the bench lines.
#   gpurun --timeout 1200 -- bash tools/r06_final_a.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest_gpu.log
case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $OUT/bench_config2.json 2> $OUT/bench_config2.err || exit $?
for w in config3 config5 select_gains; do
  timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline > $OUT/bench_$w.json 2> $OUT/bench_$w.err || exit $?
done
timeout -k 10 200 python bench.py --workload bruteforce --steps 10 --no-cpu-baseline > $OUT/bench_bruteforce.json 2> $OUT/bench_bruteforce.err || exit $?
timeout -k 10 200 python tools/bench_forward.py --system quadrotor --no-loop --cpu-seconds 1 > $OUT/fwd.jsonl 2> $OUT/fwd.err || exit $?
exit $rc
