"""Summarise a rocprofv3 rocpd database (kernel-trace) into a per-kernel stats CSV.

    python tools/rocpd_summary.py gpurun_out/r1/prof/run_results.db > profiles/r01_bench_kernel_stats.csv

Columns follow rocprofv3's own kernel_stats.csv: Name, Calls, TotalDurationNs,
AverageNs, Percentage.  (Later runs pass `-f csv` and commit kernel_stats.csv
directly; this exists for runs that only wrote the .db.)"""
import csv
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
w = csv.writer(sys.stdout)
w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
for name, calls, total_us, avg_us, pct in db.execute(
        "select name, total_calls, total_duration, average, percentage from top_kernels"):
    # top_kernels reports microseconds
    w.writerow([name, calls, round(total_us * 1e3), round(avg_us * 1e3), round(pct, 3)])
