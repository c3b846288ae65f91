export TMPDIR=/tmp
python tools/gpu_steps.py \
  buildtests 300 'python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_build.py -m gpu' \
  sizes 200 'python tools/bench_build.py --n 12500000 100000000 --steps 10 && python tools/bench_build.py --n 10000000 --dim 5 8 --steps 5' \
  prof 200 'rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profD -o run -- python3 tools/bench_build.py --n 100000000 --steps 3'
