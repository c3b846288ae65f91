#!/bin/bash
# Round 5, call 14: sampled triples across second-stage levels (the 1 B plan), reference-mode
# histograms from stored block partials: tests, the 1 B / 100 M A/B, reference bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
step() {  # step SECONDS LOG cmd...: a test failure (rc 1) goes on, anything else ends the call
  local t=$1 log=$2; shift 2
  timeout -k 10 $t "$@" > $O/$log 2>&1
  local rc=$?
  echo "$log rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step 400 r5_g3_tests6.log python3 -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_g3.py
step 300 r5_ref_tests6.log python3 -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_reference.py
step 200 r5_ref_bench6.log python3 -u tools/bench_reference.py --n 10000000 1000000 --dim 3
step 500 r5_g3_ab_1b.log python3 -u tools/g3_ab.py --n 1000000000 100000000 --steps 2 --reps 2 --sets "PKD_G3=0" ""
