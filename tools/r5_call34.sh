#!/bin/bash
# Round 5, call 34: reference-mode partition grid sweep (PKD_REF_BLOCKS), 10M x 3D, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
: > $O/r5_ref_blocks.log
for rep in 1 2; do
for b in 8192 12288 16384 1536 6144; do
  PKD_REF_BLOCKS=$b timeout -k 10 120 python3 -u tools/bench_reference.py --n 10000000 --reps 10 > $O/r5_rb.log 2>&1 || exit 1
  grep -v amdgpu $O/r5_rb.log | sed "s/^/blocks=$b /" >> $O/r5_ref_blocks.log
done
done
cat $O/r5_ref_blocks.log
