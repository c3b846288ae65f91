#!/bin/bash
# rocprofv3 kernel stats of the reference-mode GPU build (tools/bench_reference.py, 6 builds).
# Usage: prof_reference.sh TAG N DIM
set -e
export TMPDIR=/tmp
TAG=$1; N=$2; DIM=$3
OUT=$GRAFT_REPO_ROOT/gpurun_out/profref_$TAG
mkdir -p $OUT
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT -o kt --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/tools/bench_reference.py --n $N --dim $DIM --reps 5 > $OUT/run.log 2>&1
python3 - $OUT/kt_kernel_stats.csv > $OUT/summary.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    if "k_ref" in r["Name"] or "k_rr" in r["Name"] or "pkdtree" in r["Name"]:
        print(f'{r["Name"][:60]:60s} calls={r["Calls"]:>6s} total_ms/build={float(r["TotalDurationNs"])/6e6:8.3f} avg_us={float(r["AverageNs"])/1e3:8.1f}')
PY
