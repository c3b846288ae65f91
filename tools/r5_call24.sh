#!/bin/bash
# Round 5, call 24: 100M x 8D kernel timeline at the round-5 head
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/prof_build_dim.sh r5_8d 100000000 8; echo "prof rc=$?"
