#!/bin/bash
# Round 5, call 20: per-kernel HBM traffic of one 100M x 3D build at the round-5 head.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/traffic_table.sh r5 100000000 3; echo "traffic rc=$?"
