#!/bin/bash
# Round 5, call 33: the full GPU suite and the driver's smoke at the head.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 900 python3 -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests/ > $O/r5_gpu_suite.log 2>&1; echo "suite rc=$?"
tail -n 2 $O/r5_gpu_suite.log
grep -q " passed" $O/r5_gpu_suite.log && ! grep -q "failed\|rror" $O/r5_gpu_suite.log || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/r5_smoke.log 2>&1; echo "smoke rc=$?"
tail -n 3 $O/r5_smoke.log
