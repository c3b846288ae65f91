#!/bin/bash
# HBM-side byte counters of the global-level kernels of one 100M x 3D build (tools/bench_build.py, 1 step):
# one rocprofv3 pass per TCC counter group. Usage: pmc_partition.sh TAG
set -e
export TMPDIR=/tmp
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmcp_$TAG
mkdir -p $OUT
cd /tmp
run() {
  timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-include-regex 'k_partition|k_scan|k_prep|k_subtree' \
    -d $OUT/$1 -o $1 --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_build.py --n 100000000 --dim 3 --steps 1
}
run FETCH_SIZE
run WRITE_SIZE
run TCC_HIT_sum TCC_MISS_sum
