#!/bin/bash
# Round 5, call 42: knob sweep at 100M x 3D (histogram and sample grids), interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 800 python3 -u tools/g3_ab.py --n 100000000 --reps 3 --sets "" "PKD_HIST_DIV=1" "PKD_HIST_DIV=4" "PKD_G3_SAMPLE_BLOCKS=4096" "PKD_G3_SAMPLE_BLOCKS=1024" "PKD_SCAN_DIV=2" > $O/r5_knobs.log 2>&1; echo "rc=$?"
grep median $O/r5_knobs.log
