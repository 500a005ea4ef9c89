#!/bin/bash
# Round-6 GPU pass f: kernel traces of the select + gains and config-2 bench steps
# (launch gaps: is a fused select + gains launch worth building?), the rerun cost
# against round 5's library in one process, and the default bench line.
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/tr_sg -o run --output-format csv -- python3 bench.py --workload select_gains --steps 400 --no-cpu-baseline --no-h2d --event-every 1000000 > $OUT/tr_sg.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/tr_c2 -o run --output-format csv -- python3 bench.py --steps 400 --no-cpu-baseline --no-h2d --no-anchor --no-alt --event-every 1000000 > $OUT/tr_c2.log 2>&1 && \
timeout -k 10 600 python tools/bench_rerun.py time_opt_ilqr_amd/libhop_amd.so time_opt_ilqr_amd/libhop_ab_base.so --rounds 8 > $OUT/rerun.jsonl 2> $OUT/rerun.err && \
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "r06f_pass rc=$rc"
exit $rc
