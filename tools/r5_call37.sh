#!/bin/bash
# Round 5, call 37: 4096 partition blocks per level at >= 64 M points: tests, bench 100M, 1B.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 600 python3 -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_build.py tests/test_gpu_g3.py tests/test_gpu_top.py > $O/r5_lb_tests.log 2>&1; echo "tests rc=$?"
tail -n 1 $O/r5_lb_tests.log
grep -q " passed" $O/r5_lb_tests.log && ! grep -q "failed\|rror" $O/r5_lb_tests.log || exit 1
PKD_SKIP_BUILD=1 timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 > $O/r5_bench_lb.log 2>&1; echo "bench rc=$?"
grep -o '"ms_per_step": [0-9.]*' $O/r5_bench_lb.log
PKD_SKIP_BUILD=1 timeout -k 10 300 python3 -u bench.py --points 1000000000 --dim 3 --steps 3 --warmup 1 > $O/r5_bench_lb_1b.log 2>&1; echo "bench1b rc=$?"
grep -o '"ms_per_step": [0-9.]*' $O/r5_bench_lb_1b.log
