#!/usr/bin/env python3
"""Table of a build's kernels: dispatches, time, HBM-side read / write bytes (FETCH_SIZE /
WRITE_SIZE counters, KB units) and the implied bandwidth, per build.
Usage: traffic_table.py OUT_DIR BUILDS   (OUT_DIR from tools/traffic_table.sh)"""
import csv
import glob
import re
import sys
from collections import defaultdict

out, builds = sys.argv[1], int(sys.argv[2])


def short(n):
    m = re.search(r"(k_[a-z_0-9]+(<[^>]*>)?)", n)
    return m.group(1) if m else n[:40]


t = defaultdict(float)
cnt = defaultdict(int)
for p in glob.glob(f"{out}/kt/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        k = short(r["Kernel_Name"])
        t[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        cnt[k] += 1
byt = defaultdict(float)
for tag, name in (("f", "FETCH_SIZE"), ("w", "WRITE_SIZE")):
    for p in glob.glob(f"{out}/{tag}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            if r["Counter_Name"] == name:
                byt[(short(r["Kernel_Name"]), tag)] += float(r["Counter_Value"]) * 1024
rows = sorted(t, key=lambda k: -t[k])
tot_t = tot_r = tot_w = 0.0
print(f"per build ({builds} builds profiled): kernel, dispatches, time us, read GB, write GB, TB/s")
for k in rows:
    us = t[k] / builds
    rd = byt[(k, "f")] / builds / 1e9
    wr = byt[(k, "w")] / builds / 1e9
    tot_t += us
    tot_r += rd
    tot_w += wr
    bw = (rd + wr) / (us * 1e-6) / 1e3 if us > 0 else 0.0
    print(f"  {k:40s} {cnt[k] // builds:4d} {us:9.1f} {rd:8.3f} {wr:8.3f} {bw:6.2f}")
print(f"  {'total':40s}      {tot_t:9.1f} {tot_r:8.3f} {tot_w:8.3f}   HBM total {tot_r + tot_w:.2f} GB")
