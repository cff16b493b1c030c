"""Per-kernel dispatch count, average duration and period of a rocprofv3
kernel trace (--kernel-trace --output-format csv): for each kernel, runs of
consecutive dispatches separated by an idle gap (> 50 us) are the submitted
batches; the period of a run is (last end - first start) / dispatches.

    python tools/trace_period.py <rocprofv3 output dir> [kernel substrings...]
"""
import collections
import csv
import glob
import json
import sys


def main():
    d = sys.argv[1]
    want = sys.argv[2:]
    rows = []
    for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if want and not any(w in name for w in want):
                continue
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name.split("(")[0]))
    rows.sort()
    by = collections.defaultdict(list)
    for s, e, n in rows:
        by[n].append((s, e))
    out = {}
    for n, v in by.items():
        runs, cur = [], [v[0]]
        for a, b in zip(v, v[1:]):
            if b[0] - max(x[1] for x in cur) > 50_000:
                runs.append(cur)
                cur = [b]
            else:
                cur.append(b)
        runs.append(cur)
        out[n] = {"dispatches": len(v),
                  "avg_us": round(sum(e - s for s, e in v) / len(v) / 1e3, 3),
                  "runs": [{"dispatches": len(r),
                            "period_us": round((max(e for _, e in r) - r[0][0]) / len(r) / 1e3, 3)}
                           for r in runs]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
