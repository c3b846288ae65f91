#!/bin/bash
# Round 5, call 21: 12-item k_tail3 with two key sets + ids in registers (no spills): tail tests,
# interleaved A/B at 100M.
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
step 300 r5_tail_tests.log python3 -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_build.py -k tail_levels
step 500 r5_tail_ab2.log python3 -u tools/g3_ab.py --n 100000000 --reps 5 --sets "" "PKD_TAIL_SLIM12=2" "PKD_TAIL_SLIM12=1"
