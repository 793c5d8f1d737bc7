"""Kernel summary (the rocprofv3 --stats table) from a rocprofv3 rocpd database or a
kernel_stats.csv, written as CSV.  usage: python tools/rocpd_stats.py <run_results.db|dir> [out.csv]"""
import csv
import glob
import os
import sqlite3
import sys


def rows_from(path):
    if os.path.isdir(path):
        dbs = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
        if dbs:
            path = dbs[0]
        else:
            cs = glob.glob(os.path.join(path, "**", "*kernel_stats.csv"), recursive=True)
            with open(cs[0]) as f:
                return list(csv.reader(f))
    c = sqlite3.connect(path)
    cur = c.execute("select name, total_calls, total_duration, average, percentage from top_kernels")
    out = [["Name", "Calls", "TotalDurationUs", "AverageUs", "Percentage"]]
    for name, calls, tot, avg, pct in cur:
        out.append([name, calls, f"{tot:.3f}", f"{avg:.3f}", f"{pct:.3f}"])
    return out


if __name__ == "__main__":
    rows = rows_from(sys.argv[1])
    w = csv.writer(open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout)
    w.writerows(rows)
