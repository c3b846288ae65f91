#!/bin/bash
# Round 5, call 22: sampled triples at more levels: 100M with level 10 sampled (small samples),
# 12.5M with level 4 sampled (the P = 8 leaf size).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 500 python3 -u tools/g3_ab.py --n 100000000 --reps 3 --sets "" "PKD_G3_MIN_ROWS=65536,PKD_G3_SAMPLE=8192" "PKD_G3_MIN_ROWS=65536,PKD_G3_SAMPLE=4096" > $O/r5_g3_l10.log 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/g3_ab.py --n 12500000 --reps 5 --sets "" "PKD_G3_MIN_N=0" "PKD_G3_MIN_N=0,PKD_G3_SAMPLE=16384" "PKD_G3_MIN_N=0,PKD_G3_MULTI_BELOW=1" > $O/r5_g3_12m.log 2>&1 || exit 1
