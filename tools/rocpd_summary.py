"""Write the per-kernel summary (rocprofv3 --kernel-trace --stats, rocpd SQLite output) as CSV.

Usage: python tools/rocpd_summary.py gpurun_out/<dir>/run_results.db profiles/r01/<name>.csv
Columns: kernel name, calls, total ns, average ns, percent of GPU kernel time.
"""
import csv
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_us", "average_us", "percent"])
        for r in rows:
            w.writerow([r[0], r[1], round(r[2], 3), round(r[3], 3), round(r[4], 3)])
    print(f"{len(rows)} kernels -> {out}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
