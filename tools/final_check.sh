#!/bin/bash
# Round-end verification on one GPU box: the whole GPU suite, smoke(), the 1-GPU bench; each
# step under its own time limit, chained.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py > $O/bench.log 2>&1 || exit 1
