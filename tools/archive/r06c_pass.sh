#!/bin/bash
# Round-6 GPU pass c: the new gain tests, a one-process A/B against round 5's library
# (tools/ab_libs.py), SQ counters of the two small-s kernels, the select + gains line,
# the per-step aten ops and event-record A/B of the bench steps.
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_gains.py tests/test_gpu_small_rowgroup.py -v -s --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 && \
timeout -k 10 300 python tools/trace_aten_ops.py --workload select_gains > $OUT/aten_sg.txt 2>&1 && \
timeout -k 10 300 python tools/ab_step_events.py --workload lft > $OUT/step_events_lft.json 2> $OUT/step_events.err && \
timeout -k 10 300 python tools/ab_step_events.py --workload select_gains --steps 1000 > $OUT/step_events_sg.json 2>> $OUT/step_events.err && \
timeout -k 10 900 python tools/ab_libs.py time_opt_ilqr_amd/libhop_amd.so time_opt_ilqr_amd/libhop_ab_base.so --only config2,riccati_mode0,riccati_mode1,bruteforce_jcurve,select_traj_cf,small_s5_f64_4096 --rounds 7 > $OUT/ab_vs_r05.jsonl 2> $OUT/ab.err && \
bash tools/prof_sq.sh $OUT/sq_rowgroup python3 tools/small_rg_probe.py --path rowgroup && \
bash tools/prof_sq.sh $OUT/sq_lane python3 tools/small_rg_probe.py --path lane && \
timeout -k 10 300 python bench.py --workload select_gains --no-cpu-baseline > $OUT/bench_sg.json 2> $OUT/bench_sg.err
rc=$?; echo "r06c_pass rc=$rc"
exit $rc
