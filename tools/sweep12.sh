#!/bin/bash
# A/B/A/B of level-grid knobs on one-stream builds (bench_build, 30 steps): PKD_AB variants at 12.5 M and 100 M.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/sweep12.txt
: > $O
for r in 1 2; do
  for n in 12500000 100000000; do
    for v in "X=0" "PKD_SCAN_DIV=1" "PKD_SCAN_DIV=1,PKD_LEVEL_BLOCKS=2048" "PKD_LEVEL_BLOCKS=2048"; do
      echo "== round $r n $n $v" >> $O
      env PKD_AB=1 PKD_SPLIT=0 $(echo "$v" | tr , " ") timeout -k 10 100 python3 tools/bench_build.py --n $n --dim 3 --steps 30 2>&1 | grep '^{' >> $O || exit 1
    done
  done
done
