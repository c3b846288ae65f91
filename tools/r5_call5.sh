set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_reference.py > $O/r5_ref_tests2.log 2>&1 || exit 1
bash tools/prof_reference.sh r5b 10000000 3 || exit 1
timeout -k 10 200 python3 -u tools/bench_reference.py --n 10000000 1000000 --dim 3 > $O/r5_ref_bench2.log 2>&1 || exit 1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_build.py tests/test_gpu_top.py > $O/r5_build_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py > $O/r5_bench_tail.log 2>&1
