export TMPDIR=/tmp
python tools/gpu_steps.py \
  t 600 'python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_build.py -m gpu' \
  ab 300 'PKD_SUBTREE_STAMPS=1 python tools/bench_build.py --n 100000000 --steps 3; PKD_SUBTREE_STAMPS=1 python tools/bench_build.py --n 100000000 --dim 8 --steps 3; PKD_SUBTREE_IMPL=rank python tools/bench_build.py --n 100000000 --steps 3'
