#!/bin/bash
# Round 5, call 35: reference mode with one partition chunk per block (partials sized per block):
# tests, 10M x 3D timing, profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python3 -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_reference.py > $O/r5_ref_tests.log 2>&1; echo "tests rc=$?"
tail -n 1 $O/r5_ref_tests.log
grep -q " passed" $O/r5_ref_tests.log && ! grep -q "failed\|rror" $O/r5_ref_tests.log || exit 1
timeout -k 10 120 python3 -u tools/bench_reference.py --n 10000000 100000000 --reps 10 > $O/r5_ref_final.log 2>&1; echo "bench rc=$?"
bash tools/prof_reference.sh r5l 10000000 3; echo "profref rc=$?"
