#!/bin/bash
# bench.py over the sizes README / BASELINE.md quote (every run checks its tree). Usage: size_sweep.sh OUT
set -e
OUT=$1
for cfg in "1000000 3" "10000000 3" "12500000 3" "25000000 3" "50000000 3" "10000000 8" "500000 128"; do
  set -- $cfg
  echo "== $1 x $2D" >> "$OUT"
  PKD_SKIP_BUILD=1 timeout -k 10 150 python bench.py --points "$1" --dim "$2" --steps 20 --warmup 5 2>&1 \
    | grep -v amdgpu.ids >> "$OUT"
done
