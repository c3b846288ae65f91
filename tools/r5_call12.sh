#!/bin/bash
# Round 5, call 12: the whole GPU suite at the head, the reference-mode bench + profile, then the
# BASELINE refresh (tools/r5_baseline.sh: bench.py at the quoted sizes, 100M x 8D, 1B x 3D).
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
step 900 r5_gpu_suite.log python3 -u -m pytest -q -m gpu --timeout 200 --timeout-method thread tests/
step 200 r5_ref_bench5.log python3 -u tools/bench_reference.py --n 10000000 1000000 --dim 3
bash tools/prof_reference.sh r5e 10000000 3; echo "profref rc=$?"
bash tools/r5_baseline.sh; echo "baseline rc=$?"
