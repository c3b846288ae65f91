export TMPDIR=/tmp
python tools/gpu_steps.py \
  gputests 600 'python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu' \
  marker 200 'rocprofv3 --marker-trace --kernel-trace --stats --output-format csv -d gpurun_out/marker -o run -- python3 tools/bench_build.py --n 12500000 --steps 2' \
  bench 300 'python bench.py'
