"""Per-kernel summary (the `--stats` kernel_stats.csv columns) from a rocprofv3 rocpd SQLite database.

rocprofv3 on ROCm 7 writes `<dir>/<name>_results.db` by default; this prints the same table that
`--output-format csv --stats` would have written to kernel_stats.csv.

    python tools/rocpd_stats.py gpurun_out/prof/run_results.db > profiles/rNN_kernel_stats.csv
"""
import csv
import sqlite3
import sys


def main(path):
    con = sqlite3.connect(path)
    rows = con.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
        "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, calls, tot, avg, mn, mx in rows:
        w.writerow([name, calls, tot, f"{avg:.1f}", f"{100.0 * tot / total:.2f}", mn, mx])


if __name__ == "__main__":
    main(sys.argv[1])
