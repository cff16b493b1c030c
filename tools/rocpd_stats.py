"""Kernel statistics from a rocprofv3 SQLite output (run_results.db), in the
--stats CSV's columns (Name, Calls, TotalDurationNs, AverageNs, Percentage,
MinNs, MaxNs, StdDev). Not part of the product.

    python tools/rocpd_stats.py gpurun_out/<dir>/run_results.db [> out.csv]
"""
import csv
import sqlite3
import statistics
import sys


def main(path):
    c = sqlite3.connect(path)
    rows = {}
    for name, dur in c.execute("select name, duration from kernels"):
        rows.setdefault(name, []).append(int(dur))
    total = sum(sum(v) for v in rows.values()) or 1
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs",
                "StdDev"])
    for name, v in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([name, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / total, min(v), max(v),
                    statistics.pstdev(v)])


if __name__ == "__main__":
    main(sys.argv[1])
