#!/bin/bash
# Round-6 GPU pass i: the small-s row-group kernel with two image slots (the DMA two
# steps ahead): parity on the small-s, real-input and trajectory tests, then a
# one-process A/B against the library before it (tools/exp/libhop_head.so).
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_small_rowgroup.py tests/test_gpu_real_lin.py tests/test_gpu_traj.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 && \
timeout -k 10 600 python tools/ab_libs.py time_opt_ilqr_amd/libhop_amd.so tools/exp/libhop_head.so --only small_s5_f64_4096,config2 --rounds 12 > $OUT/ab_db.jsonl 2> $OUT/ab_db.err
rc=$?; echo "r06i_pass rc=$rc"
exit $rc
