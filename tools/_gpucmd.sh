export TMPDIR=/tmp
python tools/gpu_steps.py \
  new 200 'python -u tools/bench_build.py --n 100000000 12500000 --dim 8 3 --steps 10' \
  old 200 'cd old_wt && python -u tools/bench_build.py --n 100000000 12500000 --dim 8 3 --steps 10' \
  new2 200 'python -u tools/bench_build.py --n 100000000 12500000 --dim 8 3 --steps 10'
