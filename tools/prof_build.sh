#!/bin/bash
# One-stream 100M x 3D build under rocprofv3 kernel trace + the subtree kernel's per-level stamps.
# Usage: prof_build.sh TAG [N]
set -e
export TMPDIR=/tmp
TAG=$1; N=${2:-100000000}
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp
PKD_SPLIT=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT -o kt --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/tools/bench_build.py --n $N --dim 3 --steps 3 > $OUT/run.log 2>&1
PKD_SPLIT=0 PKD_SUBTREE_STAMPS=1 timeout -k 10 120 python3 $GRAFT_REPO_ROOT/tools/bench_build.py --n $N --dim 3 --steps 1 > $OUT/stamps.log 2>&1
