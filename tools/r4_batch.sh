#!/bin/bash
# Round-4 verification batch on one GPU box (each step under its own time limit, chained).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_brute_mfma.py tests/test_gpu_top.py > $O/mfma_tests.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/top_diag.py 100000000 > $O/diag.log 2>&1 || exit 1
PKD_BRUTE_MFMA_STATS=1 timeout -k 10 120 python3 tools/bench_query.py --queries 100 --reps 2 > $O/mfma_stats.log 2>&1 || exit 1
timeout -k 10 120 python3 tools/bench_query.py --queries 100 > $O/mfma_bench.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_mf -o mf --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_query.py --queries 100 > $GRAFT_REPO_ROOT/$O/prof_mf.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$O/prof_emu -o emu --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/emulate_rank.py --reps 3 > $GRAFT_REPO_ROOT/$O/prof_emu.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
bash tools/top_knobs.sh > $O/top_knobs.log 2>&1 || exit 1
timeout -k 10 200 python3 tools/bench_reference.py --n 10000000 > $O/refbench.log 2>&1 || exit 1
