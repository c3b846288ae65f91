#!/bin/bash
# Round 5, call 36: exact builder partition grid at 100M (PKD_LEVEL_BLOCKS), interleaved A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 600 python3 -u tools/g3_ab.py --n 100000000 --reps 6 --sets "" "PKD_LEVEL_BLOCKS=4096" "PKD_LEVEL_BLOCKS=6144" > $O/r5_level_blocks.log 2>&1; echo "rc=$?"
grep median $O/r5_level_blocks.log
