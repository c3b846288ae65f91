#!/bin/bash
# Round 5, call 25: the sampled top's per-node selections fused into the last blocks of the passes
# before them: top tests, interleaved A/B (PKD_TOP_FUSE) at 12.5M / 100M, the emulated P = 8 rank.
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
step 400 r5_fuse_tests.log python3 -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_top.py
grep -q " passed" $O/r5_fuse_tests.log && ! grep -q "failed" $O/r5_fuse_tests.log || exit 1
step 400 r5_fuse_ab.log python3 -u tools/g3_ab.py --n 12500000 100000000 --reps 5 --sets "PKD_TOP_FUSE=0" ""

