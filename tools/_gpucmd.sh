export TMPDIR=/tmp
python tools/gpu_steps.py \
  t 600 'python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_build.py -m gpu -k "not wave"' \
  ab 300 'for v in 0 1 0 1; do PKD_PART_PREFETCH=$v python tools/bench_build.py --n 12500000 100000000 --steps 10 | grep -v amdgpu; done'
