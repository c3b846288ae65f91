export TMPDIR=/tmp
python tools/gpu_steps.py \
  t 600 'python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_build.py -m gpu' \
  b 200 'python tools/bench_build.py --n 500000 --dim 128 --steps 20 --data reference && python tools/bench_build.py --n 1000000 --dim 16 32 64 --steps 10' \
  p 100 'rocprofv3 --kernel-trace --output-format csv -d gpurun_out/p128b -o run -- python3 tools/bench_build.py --n 500000 --dim 128 --steps 3 --data reference'
