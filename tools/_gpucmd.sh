export TMPDIR=/tmp
python tools/gpu_steps.py \
  gputests 600 'python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu' \
  bench 300 'python bench.py'
