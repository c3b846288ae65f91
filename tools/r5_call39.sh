#!/bin/bash
# Round 5, call 39: 1B x 3D and 100M x 8D at the head (4096 partition blocks per level >= 64 M points)
# against PKD_LEVEL_BLOCKS=2048 (the previous default), interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 400 python3 -u tools/g3_ab.py --n 1000000000 --steps 2 --reps 2 --sets "" "PKD_LEVEL_BLOCKS=2048" > $O/r5_lb_1b.log 2>&1; echo "1b rc=$?"
grep median $O/r5_lb_1b.log
timeout -k 10 400 python3 -u tools/g3_ab.py --n 100000000 --dim 8 --steps 3 --reps 2 --sets "" "PKD_LEVEL_BLOCKS=2048" > $O/r5_lb_8d.log 2>&1; echo "8d rc=$?"
grep median $O/r5_lb_8d.log
