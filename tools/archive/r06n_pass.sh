#!/bin/bash
# Round-6 GPU pass n: the small-s row-group kernel with each step's query under the
# next step's sweeps (HOP_SMALL_QPIPE, tools/exp/libhop_qpipe.so): parity on the small-s
# and real-input tests, a one-process A/B against the product library (bitwise equal
# expected), and the batch sweep of the augmented and trajectory forms.
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
HOP_LIB=tools/exp/libhop_qpipe.so timeout -k 10 600 python -u -m pytest tests/test_gpu_small_rowgroup.py tests/test_gpu_real_lin.py tests/test_gpu_traj.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_qpipe.log 2>&1 && \
timeout -k 10 600 python tools/ab_libs.py tools/exp/libhop_qpipe.so time_opt_ilqr_amd/libhop_amd.so --only small_s5_f64_4096 --rounds 12 > $OUT/ab_qpipe.jsonl 2> $OUT/ab.err
rc=$?; echo "r06n_pass rc=$rc"
exit $rc
