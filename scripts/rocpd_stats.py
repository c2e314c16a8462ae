#!/usr/bin/env python3
"""Kernel statistics (calls, total / average / min / max ns) from a rocprofv3 SQLite output
(``run_results.db``), as the CSV that ``--stats --output-format csv`` would write.

Usage: python scripts/rocpd_stats.py RESULTS_DB OUT_CSV
"""
import csv
import sqlite3
import sys


def main():
    db, out = sys.argv[1:3]
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, n, s, a, mn, mx in rows:
            w.writerow([name, n, s, round(a, 1), round(100.0 * s / tot, 2), mn, mx])
    for name, n, s, a, mn, mx in rows[:12]:
        print(f"{a / 1e3:10.1f} us avg  x{n:4d}  {name[:110]}")


if __name__ == "__main__":
    main()
