#!/bin/bash
# Round-5 refresh of BASELINE.md's single-GPU column: bench.py (every run checks its tree on the
# device) at the quoted sizes, 100 M x 8D and 1 B x 3D; then a kernel trace of one 1 B build.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_baseline
mkdir -p $O
run() {  # tag, then bench.py arguments
  local tag=$1; shift
  PKD_SKIP_BUILD=1 timeout -k 10 240 python3 -u bench.py "$@" > $O/$tag.log 2>&1 || return 1
  grep -h '"metric"' $O/$tag.log | sed "s/^/$tag /" >> $O/all.txt
}
: > $O/all.txt
run b100M_3d --steps 20 --warmup 5 || exit 1
run b100M_8d --points 100000000 --dim 8 --steps 10 --warmup 3 || exit 1
for cfg in "1000000 3" "10000000 3" "12500000 3" "25000000 3" "50000000 3" "10000000 8" "500000 128"; do
  set -- $cfg
  run b$1_$2d --points $1 --dim $2 --steps 20 --warmup 5 || exit 1
done
run b1B_3d --points 1000000000 --dim 3 --steps 3 --warmup 1 || exit 1
cat $O/all.txt
