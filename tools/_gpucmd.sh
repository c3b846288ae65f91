export TMPDIR=/tmp
python tools/gpu_steps.py \
  graph 200 'python tools/graph_check.py 100000 4000000 12500000 25000000 100000000' \
  t 900 'python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/ -m gpu' \
  b 200 'python bench.py --steps 20 --warmup 5'
