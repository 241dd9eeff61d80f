"""Kernel statistics (the `rocprofv3 --stats` kernel table) from a rocprofv3 SQLite output
(`results.db`): name, calls, total/average/min/max ns, percentage.   usage:
    python tools/rocpd_stats.py gpurun_out/<tag>/prof_c2/run_results.db > profiles/.../kernel_stats.csv
"""
import csv
import sqlite3
import statistics
import sys


def main(db):
    con = sqlite3.connect(db)
    rows = con.execute("select name, duration from kernels").fetchall()
    by = {}
    for name, dur in rows:
        by.setdefault(name, []).append(dur)
    total = sum(sum(v) for v in by.values()) or 1
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([name, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / total, min(v), max(v),
                    statistics.pstdev(v) if len(v) > 1 else 0.0])


if __name__ == "__main__":
    main(sys.argv[1])
