#!/bin/bash
# Round 5, call 40: partition grid below 64 M points (12.5M, 25M, 50M), interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 600 python3 -u tools/g3_ab.py --n 12500000 25000000 50000000 --reps 4 --sets "" "PKD_LEVEL_BLOCKS=2048" "PKD_LEVEL_BLOCKS=4096" > $O/r5_lb_small.log 2>&1; echo "rc=$?"
grep median $O/r5_lb_small.log
