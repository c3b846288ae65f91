#!/bin/bash
# PMC passes over the sampled top pass's kernels (k_scatter, k_res_*, k_samp_*) of one 100M x 3D
# build (tools/bench_build.py, 1 step). One rocprofv3 run per counter group (no multi-pass).
# Usage: pmc_top.sh TAG [N]
set -e
export TMPDIR=/tmp
TAG=$1; N=${2:-100000000}
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmctop_$TAG
mkdir -p $OUT
cd /tmp
run() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-include-regex 'k_scatter|k_res_|k_samp_|k_partition3' \
    -d $OUT/$name -o $name --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_build.py --n $N --dim 3 --steps 1
}
run p1 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_BRANCH
run p2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD
run p3 FETCH_SIZE
run p4 WRITE_SIZE
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $(find $OUT -name '*counter_collection.csv') > $OUT/summary.txt
