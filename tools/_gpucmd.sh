export TMPDIR=/tmp
python tools/gpu_steps.py \
  t 300 'python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_build.py tests/test_gpu_cli.py -m gpu -k "queries or traversal or cli"' \
  qp 200 'cd /tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/profq3 -o q -- python3 $GRAFT_REPO_ROOT/tools/bench_query.py' \
  q4 120 'python tools/bench_query.py --n 500000 --dim 128 --queries 100; python tools/bench_query.py --n 1000000 --dim 64 --queries 10'
