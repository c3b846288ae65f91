export TMPDIR=/tmp
python tools/gpu_steps.py \
  mr 500 'python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multirank.py -m gpu'
