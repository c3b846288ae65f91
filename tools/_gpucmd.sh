export TMPDIR=/tmp
for g in 8 16 32 8 16 32; do
PKD_COLGROUP=$g timeout -k 10 100 python tools/bench_build.py --n 500000 --dim 128 --steps 20 --data reference > gpurun_out/cg_$g.log 2>&1 || exit 1
PKD_COLGROUP=$g timeout -k 10 100 python tools/bench_build.py --n 1000000 --dim 16 64 --steps 10 >> gpurun_out/cg_$g.log 2>&1 || exit 1
echo "cg $g"; grep -o '"dim": [0-9]*\|"ms": [0-9.]*' gpurun_out/cg_$g.log | paste - - | tail -3
done
