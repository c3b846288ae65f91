export TMPDIR=/tmp
python tools/gpu_steps.py \
  t 600 'python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/ -m gpu' \
  b 200 'python bench.py --steps 20 --warmup 5' \
  p 200 'cd /tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r2a -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2'
