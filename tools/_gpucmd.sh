export TMPDIR=/tmp
python tools/gpu_steps.py \
  t 900 'python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/ -m gpu' \
  q 200 'python tools/bench_query.py 2>&1 | tail -20' \
  cli 100 'echo 42 | timeout 60 bin/kdtree_gpu --metrics-json 2>gpurun_out/cli_err.log | head -12; tail -5 gpurun_out/cli_err.log'
