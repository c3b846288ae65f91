#!/bin/bash
# Round 5, call 7: sampled triples (G3) tests, reference-mode tests, G3 on/off build A/B and a
# kernel-trace profile of the 100M x 3D build.
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
step 400 r5_g3_tests.log python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_g3.py
step 300 r5_ref_tests4.log python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_reference.py
step 200 r5_g3_bench_on.log python3 -u tools/bench_build.py --n 100000000 12500000 --dim 3 --steps 5
PKD_AB=1 PKD_G3=0 step 200 r5_g3_bench_off.log python3 -u tools/bench_build.py --n 100000000 12500000 --dim 3 --steps 5
bash tools/prof_build_dim.sh r5g3 100000000 3; echo "prof rc=$?"
