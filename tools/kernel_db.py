"""Kernel timeline from a rocprofv3 sqlite output (rocpd `kernels` view):
per-kernel average durations, and the dispatch sequence with gaps.

    python tools/kernel_db.py gpurun_out/x/run_results.db [--seq N] [--skip S]
"""
from __future__ import annotations

import argparse
import re
import sqlite3
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"(\w+kernel\w*)", name)
    base = m.group(1) if m else name[:40]
    t = re.search(r"ILi(-?\d+)E(?:Li(\d+)E)?(?:Li(\d+)E)?", name)
    if t:
        base += "<" + ",".join(x for x in t.groups() if x) + ">"
    return base


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--seq", type=int, default=0, help="print N dispatches in order")
    ap.add_argument("--skip", type=int, default=0)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else "name"
    rows = list(c.execute(f"select {name_col}, start, end from kernels order by start"))
    agg = defaultdict(list)
    for n, s, e in rows:
        agg[short(n)].append((e - s) / 1e3)
    print(f"{'kernel':60s} {'calls':>6s} {'avg_us':>9s} {'min_us':>9s}")
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k:60s} {len(v):6d} {sum(v)/len(v):9.2f} {min(v):9.2f}")
    if a.seq:
        prev = None
        for n, s, e in rows[a.skip:a.skip + a.seq]:
            gap = (s - prev) / 1e3 if prev is not None else 0.0
            print(f"  gap {gap:7.2f}  dur {(e - s) / 1e3:7.2f}  {short(n)}")
            prev = e


if __name__ == "__main__":
    main()
