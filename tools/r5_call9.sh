#!/bin/bash
# Round 5, call 9: sampled-triple + top tests, the partition-rank / G3 A/B at 100M and 12.5M
# (first set = LDS-atomic ranks everywhere, the independent reference tree), a kernel trace of
# the 100M x 3D build, reference-mode profile + bench, MFMA scratch allocator check.
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
step 300 r5_g3_tests3.log python3 -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_g3.py
step 400 r5_g3_ab2.log python3 -u tools/g3_ab.py --n 100000000 12500000 --sets \
  "PKD_PART3_ATOMIC=1,PKD_PART_ATOMIC=1,PKD_G3=0" "PKD_G3=0" "" "PKD_G3_Z=5" \
  "PKD_G3_MIN_ROWS=65536,PKD_G3_DIV_MIN=8" "PKD_G3_MIN_ROWS=65536,PKD_G3_DIV_MIN=4"
bash tools/prof_build_dim.sh r5g3b 100000000 3; echo "prof rc=$?"
bash tools/prof_reference.sh r5c 10000000 3; echo "profref rc=$?"
step 200 r5_ref_bench3.log python3 -u tools/bench_reference.py --n 10000000 1000000 --dim 3
bash tools/mfma_alloc_check.sh r5 > /dev/null 2>&1; echo "mfma rc=$?"
step 500 r5_top_tests.log python3 -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_top.py
