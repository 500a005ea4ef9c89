#!/bin/bash
# Round-6 GPU pass: the whole GPU suite (no -x: every failure in one pass), smoke, and
# the default bench line.  gpurun -- bash tools/r06_pass.sh <tag> [pytest -k expr]
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
K=${2:+-k "$2"}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread $K > $OUT/pytest.log 2>&1
prc=$?
echo "pytest rc=$prc" >> $OUT/pytest.log
# a fault / abort / timeout ends the pass here (pytest's own failures do not)
if [ $prc -ne 0 ] && [ $prc -ne 1 ]; then exit $prc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "r06_pass rc=$rc pytest=$prc"
exit $rc
