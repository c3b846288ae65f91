#!/bin/bash
# A/B/A/B of A/B knobs on one-stream builds (bench_build, 30 steps) at N (default 12.5 M):
#   VARIANTS="X=0 PKD_FOO=1,PKD_BAR=2 ..." bash tools/sweep12.sh [N]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/sweep12.txt
N=${1:-12500000}
: > $O
for r in 1 2; do
  for v in $VARIANTS; do
    echo "== round $r n $N $v" >> $O
    env PKD_AB=1 PKD_SPLIT=0 $(echo "$v" | tr , " ") timeout -k 10 100 python3 tools/bench_build.py --n $N --dim ${DIM:-3} --steps ${STEPS:-30} 2>&1 | grep '^{' >> $O || exit 1
  done
done
