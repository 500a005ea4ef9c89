#!/bin/bash
# usage: ric_run.sh tag
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "riccati or value_exp or backward or bruteforce or plots or dropin or outer_loop or gains" > $OUT/pytest.log 2>&1 && \
timeout -k 10 120 python tools/bench_riccati.py --libs ${LIBS:-$PWD/ab/base.so} > $OUT/ric.json 2>&1
rc=$?
tail -3 $OUT/pytest.log; cat $OUT/ric.json | grep -v amdgpu.ids
exit $rc
