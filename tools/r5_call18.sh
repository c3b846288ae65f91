#!/bin/bash
# Round 5, call 18: reference-mode finish with wave-by-wave last levels (readlane ranks): tests,
# A/B of PKD_REF_WAVE_ROWS, profile.
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
for w in 0 64 0 64 32; do
  PKD_REF_WAVE_ROWS=$w step 120 r5_ref_ab_$w.log python3 -u tools/bench_reference.py --n 10000000 --reps 10
  cat $O/r5_ref_ab_$w.log >> $O/r5_ref_ab.log
done
bash tools/prof_reference.sh r5i 10000000 3; echo "profref rc=$?"
