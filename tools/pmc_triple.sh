#!/bin/bash
# Counters of the scatter / key-sweep kernels of one 100M x 3D one-stream build (pairs + triples):
# one rocprofv3 pass per counter group. Usage: pmc_triple.sh TAG
set -e
export TMPDIR=/tmp
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmct_$TAG
mkdir -p $OUT
cd /tmp
run() {
  local name=$1
  shift
  PKD_SPLIT=0 timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-include-regex 'k_partition|k_scan' \
    -d $OUT/$name -o $name --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_build.py --n 100000000 --dim 3 --steps 1
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run sq SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD
