#!/bin/bash
# Round-5 GPU pass 7: the default bench line (with the fp64 s = 5 augmented-block side
# figure), the fixture statistics of every select path, the warmed A/B.
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 200 python tools/real_lin_fixture_stats.py $OUT/fixture_stats.jsonl > $OUT/fixture_stats.log 2>&1 || exit $?
timeout -k 10 500 python tools/ab_libs.py time_opt_ilqr_amd/libhop_amd.so time_opt_ilqr_amd/libhop_ab_base.so tools/exp/libhop_r04final.so tools/exp/libhop_r05_nowq_nosym.so tools/exp/libhop_r05_dmasplit.so --only config2,select_traj_cf,config3_tile64 --rounds 11 --iters 5 > $OUT/ab.jsonl 2> $OUT/ab.err
