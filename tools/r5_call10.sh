#!/bin/bash
# Round 5, call 10: sampled-triple tests (single- and multi-block resolve), then the A/B of the
# band widths (top z, triple z), the multi-block resolve at level 7, sampled triples from level 4,
# and the sample grid.
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
step 500 r5_g3_tests4.log python3 -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_g3.py
step 500 r5_g3_ab3.log python3 -u tools/g3_ab.py --n 100000000 --sets \
  "PKD_G3=0" "" "PKD_G3_Z=5" "PKD_TOP_Z=6" "PKD_TOP_Z=5" "PKD_G3_MULTI_BELOW=1024" \
  "PKD_G3_MIN_SEGS=16" "PKD_G3_MIN_SEGS=16,PKD_G3_MULTI_BELOW=1024" "PKD_G3_SAMPLE_BLOCKS=512" \
  "PKD_G3_SAMPLE_BLOCKS=1024" "PKD_G3_MIN_SEGS=16,PKD_G3_Z=5,PKD_TOP_Z=6"
step 300 r5_ref_tests5.log python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_reference.py
step 200 r5_ref_bench4.log python3 -u tools/bench_reference.py --n 10000000 1000000 --dim 3
bash tools/prof_reference.sh r5d 10000000 3; echo "profref rc=$?"
