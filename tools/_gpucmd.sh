export TMPDIR=/tmp
for d in 1 2 4 1 2 4; do
  PKD_HIST_DIV=$d timeout -k 10 100 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ph$d -o run$RANDOM -- python3 tools/bench_build.py --n 100000000 --dim 3 --steps 3 > /dev/null 2>&1 || exit 1
done
