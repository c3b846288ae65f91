export TMPDIR=/tmp
python tools/gpu_steps.py \
  p1 100 'PKD_SCAN_DIV=1 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pa1 -o run -- python3 tools/bench_build.py --n 100000000 --dim 3 --steps 3' \
  p2 100 'PKD_SCAN_DIV=2 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pa2 -o run -- python3 tools/bench_build.py --n 100000000 --dim 3 --steps 3' \
  p3 100 'PKD_SCAN_DIV=1 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pa3 -o run -- python3 tools/bench_build.py --n 100000000 --dim 3 --steps 3' \
  p4 100 'PKD_SCAN_DIV=2 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pa4 -o run -- python3 tools/bench_build.py --n 100000000 --dim 3 --steps 3'
