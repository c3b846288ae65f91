#!/bin/bash
# Round 5, call 30: high-dim prep with batched tile loads: build tests, eval-config timings + profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 400 python3 -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_build.py > $O/r5_prep_tests.log 2>&1; echo "tests rc=$?"
tail -n 1 $O/r5_prep_tests.log
timeout -k 10 120 python3 -u tools/bench_reference.py --n 500000 --dim 128 --reps 10 > $O/r5_ref_128c.log 2>&1; echo "ref128 rc=$?"
PKD_SKIP_BUILD=1 timeout -k 10 120 python3 -u bench.py --points 500000 --dim 128 --steps 20 --warmup 5 > $O/r5_bench_128.log 2>&1; echo "bench rc=$?"
bash tools/prof_reference.sh r5k128b 500000 128; echo "profref rc=$?"
