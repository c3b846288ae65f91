#!/bin/bash
# Round 5, call 19: reference-mode LDS finish by rank propagation: tests, A/B against the
# row-moving finish (PKD_REF_FIN=0), profile.
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
step 300 r5_ref_tests.log python3 -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_reference.py
: > $O/r5_ref_ab.log
for f in 0 1 0 1; do
  PKD_REF_FIN=$f step 120 r5_ref_ab_$f.log python3 -u tools/bench_reference.py --n 10000000 --reps 10
  sed "s/^/fin=$f /" $O/r5_ref_ab_$f.log >> $O/r5_ref_ab.log
done
bash tools/prof_reference.sh r5j 10000000 3; echo "profref rc=$?"
