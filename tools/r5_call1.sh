set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python3 -u bench.py > $O/r5_bench0.log 2>&1 || exit 1
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_global_native.py tests/test_gpu_top.py > $O/r5_t1.log 2>&1 || exit 1
bash tools/prof_build_dim.sh r5base 100000000 3
