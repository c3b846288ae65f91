export TMPDIR=/tmp
python tools/gpu_steps.py \
  gentest 300 'python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_generator.py -m gpu' \
  genbench 200 'python tools/bench_gen.py 100000000 && python tools/bench_gen.py 12500000' \
  genprof 200 'rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/genprof -o run -- python3 tools/bench_gen.py 100000000'
