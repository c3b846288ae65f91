export TMPDIR=/tmp
python tools/gpu_steps.py \
  tests 300 'python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_build.py tests/test_gpu_cli.py -m gpu' \
  q 200 'python tools/bench_query.py && python tools/bench_query.py --queries 1000 && python tools/bench_query.py --dim 3 --n 10000000 --queries 1000 && python tools/bench_query.py --dim 5 --n 1000000 --queries 1000'
