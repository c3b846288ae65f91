set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_reference.py > $O/r5_ref_tests.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/bench_reference.py --n 10000000 1000000 --dim 3 > $O/r5_ref_bench.log 2>&1 || exit 1
PKD_SUBTREE_STAMPS=1 PKD_TAIL_STAMPS=1 PKD_SPLIT=0 timeout -k 10 200 python3 -u tools/bench_build.py --n 100000000 12500000 --dim 3 --steps 2 > $O/r5_stamps.log 2>&1
