export TMPDIR=/tmp
python tools/gpu_steps.py \
  prof100 200 'rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof100b -o run -- python3 tools/bench_build.py --n 100000000 --steps 3 --data reference' \
  prof12 200 'rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof12b -o run -- python3 tools/bench_build.py --n 12500000 --steps 3 --data reference'
