#!/usr/bin/env python3
"""Timeline of the last build in a rocprofv3 kernel-trace CSV (`--kernel-trace --output-format csv`).

A build starts at a `k_samp_gather` (sampled top), `k_prep*` or `k_bbox*` dispatch and ends at its
`k_subtree_rank` dispatch. Prints every dispatch of the last complete build (start offset, duration,
gap to the previous dispatch's end), then per-kernel totals of that build and the span.

Usage: build_timeline.py kernel_trace.csv [--summary]   (--summary: totals and span only)
"""
import csv
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"^(void )?pkdtree::(\(anonymous namespace\)::)?((top4|subtree_detail)::)?"
                  r"(\(anonymous namespace\)::)?", "", name)
    return re.sub(r"\(.*$", "", name)


def main() -> None:
    rows = []
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    ends = [i for i, r in enumerate(rows) if r[2].startswith("k_subtree_rank")]
    if not ends:
        sys.exit("no k_subtree_rank dispatch in the trace")
    last = ends[-1]
    first = max(i for i, r in enumerate(rows[:last + 1]) if re.match(r"k_(samp_gather|prep|bbox)", r[2]))
    chain = rows[first:last + 1]
    t0 = chain[0][0]
    summary = "--summary" in sys.argv
    tot, cnt = defaultdict(float), defaultdict(int)
    prev_end = t0
    for s, e, n in chain:
        if not summary:
            print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} gap {(s - prev_end) / 1e3:6.1f}  {n}")
        prev_end = max(prev_end, e)
        key = re.sub(r"<.*$", "", n)
        tot[key] += (e - s) / 1e3
        cnt[key] += 1
    busy = sum(tot.values())
    print(f"span {(chain[-1][1] - t0) / 1e3:.1f} us, {len(chain)} dispatches, kernel busy {busy:.1f} us")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f"  {k:28s} {v:9.1f} us  {cnt[k]:4d}x")


if __name__ == "__main__":
    main()
