#!/usr/bin/env python3
"""Per-kernel timeline (start offset, duration in us) of the last emulated rank chain in a
rocprofv3 kernel-trace CSV: the kernels from the last k_top_bbox* dispatch on.
Usage: chain_timeline.py kernel_trace.csv"""
import csv
import re
import sys

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        name = re.sub(r"^(void )?pkdtree::(\(anonymous namespace\)::)?", "", r["Kernel_Name"])
        name = re.sub(r"\(.*$", "", name)
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
rows.sort()
starts = [i for i, r in enumerate(rows) if r[2].startswith("k_top_bbox")]
if not starts:
    sys.exit("no k_top_bbox dispatch in the trace")
chain = rows[starts[-1]:]
t0 = chain[0][0]
for s, e, n in chain:
    print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:7.1f} {n}")
print(f"span {(chain[-1][1] - t0) / 1e3:.1f} us")
