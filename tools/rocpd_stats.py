#!/usr/bin/env python3
"""Per-kernel stats CSV (rocprofv3 *_kernel_stats.csv columns) from a rocprofv3 rocpd SQLite DB.

    python tools/rocpd_stats.py gpurun_out/prof/run_results.db profiles/r01/x_kernel_stats.csv
"""
import csv
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, n, s, a, lo, hi in rows:
            w.writerow([name, n, s, f"{a:.1f}", f"{100.0 * s / tot:.4f}", lo, hi])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
