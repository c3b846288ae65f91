#!/bin/bash
# Round 5, call 11: new defaults (sampled triples from 16 segments, z = 5; top z = 6): G3 + top
# tests, then an interleaved A/B (4 rounds, median) at 100M x 3D, 12.5M x 3D and 100M x 8D.
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
step 500 r5_g3_tests5.log python3 -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_g3.py tests/test_gpu_top.py
step 500 r5_g3_ab4.log python3 -u tools/g3_ab.py --n 100000000 12500000 --reps 4 --sets \
  "PKD_G3=0,PKD_TOP_Z=9" "PKD_TOP_Z=9" "" "PKD_G3_MIN_SEGS=128" "PKD_G3_MULTI_BELOW=1024"
step 400 r5_g3_ab4_8d.log python3 -u tools/g3_ab.py --n 100000000 --dim 8 --reps 3 --sets "PKD_G3=0,PKD_TOP_Z=9" ""
