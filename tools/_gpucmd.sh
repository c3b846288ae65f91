export TMPDIR=/tmp
python tools/gpu_steps.py \
  gputests 600 'python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu'
