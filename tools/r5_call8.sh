#!/bin/bash
# Round 5, call 8: sampled-triple tests, then the G3 knob A/B (tools/g3_ab.py).
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
step 400 r5_g3_tests2.log python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_g3.py
step 400 r5_g3_ab1.log python3 -u tools/g3_ab.py --n 100000000 12500000 --sets "PKD_G3=0" "" \
  "PKD_PART3_ATOMIC=0" "PKD_PART3_ATOMIC=1" "PKD_G3_MIN_ROWS=262144" "PKD_G3_MIN_ROWS=262144,PKD_PART3_ATOMIC=1" \
  "PKD_G3_MIN_ROWS=262144,PKD_G3_SAMPLE=131072" "PKD_G3_MIN_ROWS=262144,PKD_G3_SAMPLE=32768" \
  "PKD_G3_MIN_ROWS=262144,PKD_G3_Z=5" "PKD_G3_SAMPLE=16384"
