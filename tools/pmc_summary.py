#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter collections: per kernel, counters summed over dispatches
(and the dispatch count), plus derived rates where the inputs are present.
Usage: pmc_summary.py run_counter_collection.csv [more.csv ...]"""
import csv
import re
import sys
from collections import defaultdict


def short(n):
    m = re.search(r"(k_[a-z_0-9]+(<[^>]*>)?)", n)
    return m.group(1) if m else n[:40]


tot = defaultdict(float)
disp = defaultdict(set)
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        tot[(k, r["Counter_Name"])] += float(r["Counter_Value"])
        disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
kernels = sorted({k for k, _ in tot})
for k in kernels:
    cs = sorted(c for kk, c in tot if kk == k)
    print(k)
    for c in cs:
        print(f"    {c:24s} {tot[(k, c)]:14.4g}   ({len(disp[(k, c)])} dispatches)")
    g = lambda c: tot.get((k, c))
    if g("SQ_INSTS_VALU") and g("SQ_INSTS_SALU"):
        print(f"    SALU / VALU instructions  {g('SQ_INSTS_SALU') / g('SQ_INSTS_VALU'):.2f}")
    if g("SQ_LDS_BANK_CONFLICT") is not None and g("SQ_INSTS_LDS"):
        print(f"    LDS bank-conflict cycles per LDS instruction  {g('SQ_LDS_BANK_CONFLICT') / g('SQ_INSTS_LDS'):.2f}")
    if g("SQ_BUSY_CYCLES") and g("SQ_WAVE_CYCLES"):
        print(f"    mean resident waves per busy cycle (whole chip)  {g('SQ_WAVE_CYCLES') / g('SQ_BUSY_CYCLES'):.1f}")
    if g("FETCH_SIZE"):
        print(f"    HBM/L2 fetch  {g('FETCH_SIZE') / 1e6:.1f} MB (FETCH_SIZE is in KB: {g('FETCH_SIZE') * 1024 / 1e9:.2f} GB)")
    if g("WRITE_SIZE"):
        print(f"    write         {g('WRITE_SIZE') * 1024 / 1e9:.2f} GB (WRITE_SIZE in KB)")
