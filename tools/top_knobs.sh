#!/bin/bash
# Sampled-top band knobs at 100 M x 3D: z (band half-width in sample-rank sigmas) x sample size.
# Usage: top_knobs.sh  (prints one JSON line per setting from tools/top_check.py --time)
for cfg in "9 20" "6 20" "6 21" "5 21" "7 21"; do
  set -- $cfg
  PKD_AB=1 PKD_TOP_Z=$1 PKD_TOP_SAMPLE=$2 timeout -k 10 120 python3 -u $GRAFT_REPO_ROOT/tools/top_check.py --quick --time 100000000 2>&1 \
    | grep '"top": "1"' | sed "s/^/{\"z\": $1, \"sample_log2\": $2} /" || exit 1
done
