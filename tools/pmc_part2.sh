#!/bin/bash
# Wave-state counters of the paired scatter (k_partition2) in one 100M x 3D build. Usage: pmc_part2.sh TAG
set -e
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmcq_$1
mkdir -p $OUT
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
  --kernel-include-regex 'k_partition2|k_scan' -d $OUT/a -o a --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/tools/bench_build.py --n 100000000 --dim 3 --steps 1
timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC \
  --kernel-include-regex 'k_partition2|k_scan' -d $OUT/b -o b --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/tools/bench_build.py --n 100000000 --dim 3 --steps 1
