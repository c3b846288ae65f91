#!/bin/bash
# Round 5, call 38: the full GPU suite (builders discarded after a miss), the bench, the smoke.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 900 python3 -u -m pytest -q -x -m gpu --timeout 300 --timeout-method thread tests/ > $O/r5_gpu_suite.log 2>&1; echo "suite rc=$?"
tail -n 2 $O/r5_gpu_suite.log
grep -q " passed" $O/r5_gpu_suite.log && ! grep -q "failed\|rror" $O/r5_gpu_suite.log || exit 1
PKD_SKIP_BUILD=1 timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 > $O/r5_bench_final.log 2>&1; echo "bench rc=$?"
grep -o '"ms_per_step": [0-9.]*' $O/r5_bench_final.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/r5_smoke.log 2>&1; echo "smoke rc=$?"
tail -n 1 $O/r5_smoke.log
