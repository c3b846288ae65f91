export TMPDIR=/tmp
python tools/gpu_steps.py \
  buildtests 300 'python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_build.py tests/test_gpu_cli.py -m gpu' \
  d128 200 'python tools/bench_build.py --n 500000 2000000 --dim 128 --steps 5' \
  d16 200 'python tools/bench_build.py --n 10000000 --dim 16 --steps 5' \
  d3 200 'python tools/bench_build.py --n 12500000 100000000 --dim 3 --steps 5' \
  eval 120 'echo 42 | bin/kdtree_gpu --metrics-json'
