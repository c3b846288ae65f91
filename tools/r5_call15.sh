#!/bin/bash
# Round 5, call 15: k_tail3 with two key register sets and on-demand ids (16 items always, 12 by
# knob): build tests, A/B at 100M (12 items) and 1B (16 items), reference-mode profile.
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
step 500 r5_build_tests.log python3 -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_build.py
step 400 r5_tail_ab.log python3 -u tools/g3_ab.py --n 100000000 12500000 --reps 4 --sets "" "PKD_TAIL_SLIM12=1"
step 300 r5_tail_ab_1b.log python3 -u tools/g3_ab.py --n 1000000000 --steps 2 --reps 1 --sets ""
bash tools/prof_reference.sh r5f 10000000 3; echo "profref rc=$?"
