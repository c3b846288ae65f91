export TMPDIR=/tmp
python tools/gpu_steps.py \
  t 600 'python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/ -m gpu' \
  p1 100 'PKD_IMPLICIT_IDS=0 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pi0 -o run -- python3 tools/bench_build.py --n 100000000 --dim 3 --steps 3' \
  p2 100 'rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pi1 -o run -- python3 tools/bench_build.py --n 100000000 --dim 3 --steps 3' \
  b 200 'python3 tools/bench_build.py --n 100000000 12500000 --dim 3 --steps 20 && PKD_IMPLICIT_IDS=0 python3 tools/bench_build.py --n 100000000 12500000 --dim 3 --steps 20 && python3 tools/bench_build.py --n 100000000 12500000 --dim 3 --steps 20'
