#!/bin/bash
# One-stream build of N x DIM under rocprofv3 kernel trace. Usage: prof_build_dim.sh TAG N DIM
set -e
export TMPDIR=/tmp
TAG=$1; N=$2; DIM=$3
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp
PKD_SPLIT=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT -o kt --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/tools/bench_build.py --n $N --dim $DIM --steps 3 > $OUT/run.log 2>&1
python3 $GRAFT_REPO_ROOT/tools/trace_summary.py $OUT/kt_kernel_trace.csv > $OUT/summary.txt
