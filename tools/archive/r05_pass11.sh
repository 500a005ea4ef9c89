#!/bin/bash
# Round-5 GPU pass 11: small-s tile64 LDS-DMA pieces grouped under shared M0: tests,
# the A/B and the config-3 line.
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_traj.py tests/test_gpu_parity.py tests/test_gpu_real_lin.py -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 400 python tools/ab_libs.py time_opt_ilqr_amd/libhop_amd.so tools/exp/libhop_r05_cfsym.so --only config3_tile64 --rounds 11 --iters 5 > $OUT/ab.jsonl 2> $OUT/ab.err || exit $?
timeout -k 10 200 python bench.py --workload config3 --no-cpu-baseline > $OUT/bench_config3.json 2> $OUT/bench_config3.err
