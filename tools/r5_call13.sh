#!/bin/bash
# Round 5, call 13: the new top tests (level-0 entry points of a sampled-top builder, a 12 M
# heavy-duplicate input), kernel traces of the default 100M x 3D and 1B x 3D builds, k_tail3 and
# subtree stamps at 100M.
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
step 300 r5_top_tests2.log python3 -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_top.py -k "level0 or heavy"
bash tools/prof_build_dim.sh r5final 100000000 3; echo "prof rc=$?"
PKD_TAIL_STAMPS=1 PKD_SUBTREE_STAMPS=1 step 200 r5_stamps.log python3 -u tools/bench_build.py --n 100000000 --dim 3 --steps 3
export TMPDIR=/tmp
mkdir -p $O/prof_r5_1b
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_r5_1b -o kt --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/tools/bench_build.py --n 1000000000 --dim 3 --steps 1 > $GRAFT_REPO_ROOT/$O/prof_r5_1b/run.log 2>&1); echo "1b rc=$?"
python3 tools/trace_summary.py $O/prof_r5_1b/kt_kernel_trace.csv > $O/prof_r5_1b/summary.txt; echo "sum rc=$?"
