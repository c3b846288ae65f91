#!/bin/bash
# Round 5, call 41: partition grid by size (4096 >= 40M, 2048 >= 20M, 1024 below): build tests at
# these sizes, benches 25M / 50M / 100M.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 600 python3 -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_build.py tests/test_gpu_g3.py > $O/r5_lb2_tests.log 2>&1; echo "tests rc=$?"
tail -n 1 $O/r5_lb2_tests.log
grep -q " passed" $O/r5_lb2_tests.log && ! grep -q "failed\|rror" $O/r5_lb2_tests.log || exit 1
for n in 25000000 50000000 100000000; do
  PKD_SKIP_BUILD=1 timeout -k 10 200 python3 -u bench.py --points $n --dim 3 --steps 20 --warmup 5 > $O/r5_b_$n.log 2>&1 || exit 1
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' $O/r5_b_$n.log)"
done
