export TMPDIR=/tmp
python tools/gpu_steps.py \
  gputests 600 'python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu' \
  smoke 120 'python -c "import __graft_entry__ as g; g.smoke()"' \
  bench 300 'python bench.py'
