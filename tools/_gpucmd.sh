export TMPDIR=/tmp
python tools/gpu_steps.py \
  buildtests 300 'python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_build.py -m gpu' \
  dims 300 'python tools/bench_build.py --n 10000000 --dim 4 5 6 8 16 --steps 3 && python tools/bench_build.py --n 100000000 --dim 3 8 --steps 3'
