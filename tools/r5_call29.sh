#!/bin/bash
# Round 5, call 29: reference mode's element-parallel output gather (permutation path): tests, timings.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python3 -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_reference.py > $O/r5_ref_tests.log 2>&1; echo "tests rc=$?"
tail -n 1 $O/r5_ref_tests.log
timeout -k 10 120 python3 -u tools/bench_reference.py --n 500000 --dim 128 --reps 10 > $O/r5_ref_128b.log 2>&1; echo "ref128 rc=$?"
timeout -k 10 120 python3 -u tools/bench_reference.py --n 1000000 --dim 16 --reps 10 > $O/r5_ref_16b.log 2>&1; echo "ref16 rc=$?"
