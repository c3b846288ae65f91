#!/bin/bash
# Round 5, call 23: 100M x 3D with smaller subtree capacities (one more global level: tail 14-16)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python3 -u tools/bench_build.py --n 100000000 --subtree 0 4096 0 4096 --steps 5 > $O/r5_sub4096.log 2>&1 || exit 1
export TMPDIR=/tmp
mkdir -p $O/prof_sub4096
cd /tmp
PKD_SPLIT=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_sub4096 -o kt --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/tools/bench_build.py --n 100000000 --subtree 4096 --steps 3 > $GRAFT_REPO_ROOT/$O/prof_sub4096/run.log 2>&1 || exit 1
python3 $GRAFT_REPO_ROOT/tools/trace_summary.py $GRAFT_REPO_ROOT/$O/prof_sub4096/kt_kernel_trace.csv > $GRAFT_REPO_ROOT/$O/prof_sub4096/summary.txt
