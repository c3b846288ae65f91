#!/bin/bash
# Round 5, call 43: closing profiles: 100M x 3D kernel timeline and the subtree / tail PMC passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/prof_build_dim.sh r5head 100000000 3; echo "prof rc=$?"
bash tools/pmc_subtree.sh r5head 3; echo "pmc rc=$?"
python3 tools/pmc_summary.py gpurun_out/pmc_r5head/p1/*counter_collection.csv gpurun_out/pmc_r5head/p2/*counter_collection.csv > gpurun_out/pmc_r5head/summary.txt 2>&1; echo "sum rc=$?"
