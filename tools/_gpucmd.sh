export TMPDIR=/tmp
python tools/gpu_steps.py \
  clitests 300 'python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_cli.py -m gpu'
