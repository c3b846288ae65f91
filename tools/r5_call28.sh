#!/bin/bash
# Round 5, call 28: reference-mode kernel profile at the eval config (500k x 128D, permutation path)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/prof_reference.sh r5k128 500000 128; echo "profref rc=$?"
