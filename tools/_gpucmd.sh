export TMPDIR=/tmp
python tools/gpu_steps.py \
  gputests 600 'python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu' \
  sizes 120 'python tools/bench_build.py --n 12500000 25000000 100000000 --steps 10'
