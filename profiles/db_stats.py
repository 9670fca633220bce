"""Dump a rocprofv3 (rocpd SQLite) run's per-kernel summary as CSV — the same columns as
`rocprofv3 --stats` kernel_stats.csv (durations in ns).

usage: python profiles/db_stats.py RUN_results.db OUT.csv
"""
import csv
import sqlite3
import statistics
import sys


def main():
    db, out = sys.argv[1], sys.argv[2]
    c = sqlite3.connect(db)
    rows = {}
    for name, s, e in c.execute("select name, start, end from kernels"):
        rows.setdefault(name, []).append(e - s)
    total = sum(sum(v) for v in rows.values())
    with open(out, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
        for name, d in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([name, len(d), sum(d), sum(d) / len(d), 100.0 * sum(d) / total, min(d), max(d),
                        statistics.pstdev(d) if len(d) > 1 else 0.0])


if __name__ == "__main__":
    main()
