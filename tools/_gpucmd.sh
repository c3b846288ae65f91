export TMPDIR=/tmp
python tools/gpu_steps.py \
  graphtest 300 'python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_build.py -m gpu -k graphed' \
  graphbench 200 'python tools/bench_graph.py 100000 1000000 4000000 12500000 100000000'
