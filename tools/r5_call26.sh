#!/bin/bash
# Round 5, call 26: the full GPU suite at the head, reference mode at high dims (perm path).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 900 python3 -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests/ > $O/r5_gpu_suite.log 2>&1; echo "suite rc=$?"
tail -n 3 $O/r5_gpu_suite.log
timeout -k 10 120 python3 -u tools/bench_reference.py --n 500000 --dim 128 --reps 5 > $O/r5_ref_128.log 2>&1; echo "ref128 rc=$?"
timeout -k 10 120 python3 -u tools/bench_reference.py --n 1000000 --dim 16 --reps 5 > $O/r5_ref_16.log 2>&1; echo "ref16 rc=$?"
