export TMPDIR=/tmp
python tools/gpu_steps.py \
  t 900 'python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/ -m gpu' \
  smoke 200 'python -c "import __graft_entry__ as g; g.smoke()"' \
  bench 200 'python bench.py --steps 20 --warmup 3' \
  sizes 300 'python tools/bench_build.py --n 12500000 25000000 50000000 100000000 --dim 3 --steps 10 && python tools/bench_build.py --n 100000000 --dim 8 --steps 5 && python tools/bench_build.py --n 500000 --dim 128 --steps 20 --data reference && python tools/bench_build.py --n 1000000000 --dim 3 --steps 3'
