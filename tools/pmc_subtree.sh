#!/bin/bash
# PMC passes over the LDS subtree kernel of one 100M x 3D build (tools/bench_build.py, 1 step):
# each pass is its own rocprofv3 run with at most 8 SQ counters. Usage: pmc_subtree.sh TAG [DIM]
set -e
export TMPDIR=/tmp
TAG=$1; DIM=${2:-3}
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_BRANCH \
  --kernel-include-regex 'k_subtree|k_tail' -d $OUT/p1 -o p1 --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/tools/bench_build.py --n 100000000 --dim $DIM --steps 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS \
  --kernel-include-regex 'k_subtree|k_tail' -d $OUT/p2 -o p2 --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/tools/bench_build.py --n 100000000 --dim $DIM --steps 1
