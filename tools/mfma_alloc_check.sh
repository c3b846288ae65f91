#!/bin/bash
# The MFMA brute force's scratch is persistent per (device, stream): a 10 k-query batch over
# 500 k x 128D must make no allocator call. rocprofv3 HIP API trace of tools/bench_query.py;
# prints the allocator-call counts and the timing lines. Usage: mfma_alloc_check.sh TAG
set -e
export TMPDIR=/tmp
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/mfma_$TAG
mkdir -p $OUT
cd /tmp
timeout -k 10 120 python3 $GRAFT_REPO_ROOT/tools/bench_query.py --queries 100 --dim 128 --reps 20 > $OUT/q100.log 2>&1
timeout -k 10 150 rocprofv3 --hip-trace --stats -d $OUT -o api --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/tools/bench_query.py --queries 10000 --dim 128 --reps 3 > $OUT/q10k.log 2>&1
python3 - $OUT <<'PY' > $OUT/summary.txt
import csv, glob, sys
out = sys.argv[1]
stats = glob.glob(out + "/**/api_hip_api_stats.csv", recursive=True)
rows = list(csv.DictReader(open(stats[0]))) if stats else []
alloc = {r["Name"]: r["Calls"] for r in rows if "Malloc" in r["Name"] or "Free" in r["Name"]}
print("HIP allocator calls over the whole process (setup included):", alloc)
tr = glob.glob(out + "/**/api_hip_api_trace.csv", recursive=True)
if tr:
    t = list(csv.DictReader(open(tr[0])))
    k = [r for r in t if "LaunchKernel" in r.get("Function", r.get("Name", ""))]
    a = [r for r in t if r.get("Function", r.get("Name", "")) in ("hipMallocAsync", "hipFreeAsync")]
    print("kernel launches:", len(k), "hipMallocAsync/hipFreeAsync calls:", len(a))
for f in ("q100.log", "q10k.log"):
    print(f, open(out + "/" + f).read().strip().splitlines()[-1])
PY
cat $OUT/summary.txt
