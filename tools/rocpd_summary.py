#!/usr/bin/env python3
"""Summarise a rocprofv3 database (rocpd SQLite, the default output of
`rocprofv3 --kernel-trace`): per-kernel totals over the whole run, and the per-dispatch
timeline of the last build (from its last `k_bbox*` / `k_prep*` dispatch to its subtree kernel).

Usage: rocpd_summary.py RUN_results.db [--all]   (--all prints every dispatch of the last build)
"""
import re
import sqlite3
import sys
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"(k_[A-Za-z_0-9]+(<[^>]*>)?)", name)
    return m.group(1) if m else name[:40]


def main():
    db = sqlite3.connect(sys.argv[1])
    rows = db.execute("select name, start, end, grid_x, workgroup_x, lds_size, vgpr_count, sgpr_count "
                      "from kernels order by start").fetchall()
    tot, cnt = defaultdict(float), defaultdict(int)
    for name, s, e, *_ in rows:
        tot[short(name)] += (e - s) / 1e3
        cnt[short(name)] += 1
    print(f"whole run: {len(rows)} dispatches")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:25]:
        print(f"  {k:40s} {v:10.1f} us  {cnt[k]:5d} dispatches  {v / cnt[k]:9.1f} us each")
    firsts = [i for i, r in enumerate(rows) if re.search(r"k_(prep|bbox)", r[0])]
    if not firsts:
        return
    # the last build starts at the first prep/bbox dispatch after the previous subtree kernel
    subs = [i for i, r in enumerate(rows) if "k_subtree" in r[0]]
    last_sub = subs[-1] if subs else len(rows) - 1
    prev_sub = max([i for i in subs if i < last_sub], default=-1)
    start = min(i for i in firsts if i > prev_sub) if any(i > prev_sub for i in firsts) else firsts[-1]
    last = rows[start:last_sub + 1]
    t0 = last[0][1]
    span = (last[-1][2] - t0) / 1e3
    bt, bc = defaultdict(float), defaultdict(int)
    print("\ntimeline of the last build:")
    for name, s, e, gx, wx, lds, vg, sg in last:
        k = short(name)
        d = (e - s) / 1e3
        bt[k] += d
        bc[k] += 1
        if "--all" in sys.argv:
            print(f"  {(s - t0) / 1e3:9.1f} {k:36s} {d:9.1f} us grid={gx // max(wx, 1)}x{wx} lds={lds} vgpr={vg}")
    busy = sum(bt.values())
    print(f"span {span:.1f} us; kernel sum {busy:.1f} us; gaps {span - busy:.1f} us over {len(last)} dispatches")
    for k, v in sorted(bt.items(), key=lambda kv: -kv[1]):
        print(f"  {k:40s} {v:10.1f} us  ({bc[k]} dispatches, {100 * v / span:5.1f}% of span)")


if __name__ == "__main__":
    main()
