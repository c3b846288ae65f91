#!/bin/bash
# Per-kernel HBM traffic and bandwidth of one 100M x 3D build: rocprofv3 kernel trace (times) plus
# one counter pass each for FETCH_SIZE and WRITE_SIZE (tools/bench_build.py --steps 1 = 2 builds).
# Usage: traffic_table.sh TAG [N] [DIM]
set -e
export TMPDIR=/tmp
TAG=$1; N=${2:-100000000}; DIM=${3:-3}
OUT=$GRAFT_REPO_ROOT/gpurun_out/traffic_$TAG
mkdir -p $OUT
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace -d $OUT/kt -o kt --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/tools/bench_build.py --n $N --dim $DIM --steps 1 > $OUT/kt.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/f -o f --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/tools/bench_build.py --n $N --dim $DIM --steps 1 > $OUT/f.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $OUT/w -o w --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/tools/bench_build.py --n $N --dim $DIM --steps 1 > $OUT/w.log 2>&1
python3 $GRAFT_REPO_ROOT/tools/traffic_table.py $OUT 2 > $OUT/table.txt
