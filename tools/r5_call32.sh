#!/bin/bash
# Round 5, call 32: selects that do not find their median rank (only after a reported miss) now
# leave empty zones instead of uninitialised LDS values; the refine stops inside its zone. The
# reuse-after-miss repro first, then the build / top / g3 tests, then the 100M bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python3 -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_top.py -k reused_after_misses > $O/r5_reuse_test.log 2>&1; echo "repro rc=$?"
tail -n 1 $O/r5_reuse_test.log
grep -q " passed" $O/r5_reuse_test.log && ! grep -q "failed\|rror" $O/r5_reuse_test.log || exit 1
timeout -k 10 600 python3 -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_build.py tests/test_gpu_top.py tests/test_gpu_g3.py > $O/r5_clamp_tests.log 2>&1; echo "tests rc=$?"
tail -n 1 $O/r5_clamp_tests.log
grep -q " passed" $O/r5_clamp_tests.log && ! grep -q "failed\|rror" $O/r5_clamp_tests.log || exit 1
PKD_SKIP_BUILD=1 timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 > $O/r5_bench_head.log 2>&1; echo "bench rc=$?"
grep -o '"ms_per_step": [0-9.]*' $O/r5_bench_head.log
