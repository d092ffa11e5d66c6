"""Kernel stats (rocprofv3 --stats layout) from a rocpd SQLite database.

rocprofv3 on ROCm 7.2 writes `<out>_results.db` unless `--output-format csv` is given; this
turns that database's `top_kernels` view into the kernel_stats.csv columns profiles/ uses.
usage: python tools/rocpd_stats.py RUN_results.db OUT.csv
"""
import csv
import sqlite3
import sys


def main(db: str, out: str) -> None:
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), "
                     "max(duration) from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, calls, tot, avg, mn, mx in rows:
            w.writerow([name, calls, tot, f"{avg:.1f}", f"{100.0 * tot / total:.4f}", mn, mx])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
