#!/bin/bash
# Round 5, call 27: 100M x 8D with subtree capacity 2048 (one global level fewer: no pair pass)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python3 -u tools/bench_build.py --n 100000000 --dim 8 --subtree 0 2048 0 2048 --steps 3 > $O/r5_8d_sub2048.log 2>&1; echo "rc=$?"
