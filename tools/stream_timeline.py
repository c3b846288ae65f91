#!/usr/bin/env python3
"""Concurrency of the last build in a rocprofv3 kernel trace (split builds run on several
streams): span, busy time per stream / queue, time covered by 0 / 1 / 2+ kernels, and which
kernels run alone. Usage: stream_timeline.py kernel_trace.csv [--all]"""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
skey = next((k for k in ("Stream_Id", "Queue_Id") if k in rows[0]), None)


def short(n):
    m = re.search(r"(k_[a-z_0-9]+(<[^>]*>)?)", n)
    return m.group(1) if m else n[:40]


starts = [i for i, r in enumerate(rows) if "k_bbox_reduce" in r["Kernel_Name"]]
last = rows[starts[-1]:] if starts else rows
sub_end = max((int(r["End_Timestamp"]) for r in last if "k_subtree" in r["Kernel_Name"]), default=None)
if sub_end is not None:
    last = [r for r in last if int(r["Start_Timestamp"]) < sub_end]
t0 = min(int(r["Start_Timestamp"]) for r in last)
t1 = max(int(r["End_Timestamp"]) for r in last)
ev = []
busy = defaultdict(float)
for i, r in enumerate(last):
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    ev.append((s, 1, i))
    ev.append((e, -1, i))
    busy[r.get(skey, "?")] += (e - s) / 1e3
ev.sort(key=lambda x: (x[0], x[1]))
cover = defaultdict(float)
alone = defaultdict(float)
active = set()
prev = t0
for t, d, i in ev:
    dt = (t - prev) / 1e3
    cover[min(len(active), 2)] += dt
    if len(active) == 1:
        alone[short(last[next(iter(active))]["Kernel_Name"])] += dt
    prev = t
    if d > 0:
        active.add(i)
    else:
        active.discard(i)
print(f"build span {(t1 - t0) / 1e3:.1f} us, {len(last)} dispatches, kernel sum {sum(busy.values()):.1f} us")
print("busy per " + str(skey) + ": " + ", ".join(f"{k}: {v:.1f} us" for k, v in sorted(busy.items())))
print(f"covered by 0 kernels {cover[0]:.1f} us, 1 kernel {cover[1]:.1f} us, 2+ kernels {cover[2]:.1f} us")
print("time running alone, by kernel:")
for k, v in sorted(alone.items(), key=lambda kv: -kv[1])[:15]:
    print(f"  {k:36s} {v:9.1f} us")
if "--all" in sys.argv:
    for r in last:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"  {(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} q={r.get(skey, '?'):>4} {short(r['Kernel_Name']):36s} "
              f"{(e - s) / 1e3:8.1f} us grid={r.get('Grid_Size_X', r.get('Grid_Size', '?'))}")
