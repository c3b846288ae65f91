#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace: per-kernel totals and the per-dispatch timeline of
the last build (from the last k_prep / k_bbox_init)."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))


def short(n):
    import re
    m = re.search(r"(k_[a-z_0-9]+(<[^>]*>)?)", n)
    return m.group(1) if m else n[:40]


first_kernel = next((k for k in ("k_samp_gather", "k_bbox_init", "k_bbox_reduce", "k_prep") if any(k in r["Kernel_Name"] for r in rows)), None)
starts = [i for i, r in enumerate(rows) if first_kernel and first_kernel in r["Kernel_Name"]]
last = rows[starts[-1]:] if starts else rows
# the build ends at its subtree kernel (later dispatches belong to the caller)
ends = [i for i, r in enumerate(last) if "k_subtree" in r["Kernel_Name"]]
if ends:
    last = last[:ends[0] + 1]
tot = defaultdict(float)
cnt = defaultdict(int)
print("timeline of the last build:")
t0 = int(last[0]["Start_Timestamp"])
for r in last:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    k = short(r["Kernel_Name"])
    tot[k] += d
    cnt[k] += 1
    if "--all" in sys.argv:
        print(f"  {(int(r['Start_Timestamp']) - t0) / 1e3:9.1f} {k:32s} {d:9.1f} us grid={r['Grid_Size_X']}")
span = (int(last[-1]["End_Timestamp"]) - t0) / 1e3
print(f"span {span:.1f} us; kernel sum {sum(tot.values()):.1f} us")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"  {k:32s} {v:10.1f} us  ({cnt[k]} dispatches, {100 * v / span:5.1f}% of span)")
