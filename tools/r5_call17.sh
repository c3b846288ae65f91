#!/bin/bash
# Round 5, call 17: reference mode with the select fused into the histogram block (one block per
# segment) and the next level's descriptors written by the select (no seg_init launches); the
# skewed stage2 tests on the paired path plus the checked sampled path.
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
step 300 r5_ref_tests.log python3 -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_reference.py

bash tools/prof_reference.sh r5h 10000000 3; echo "profref rc=$?"
