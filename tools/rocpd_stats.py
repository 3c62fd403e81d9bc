"""Per-kernel summary (calls, total, average) of a rocprofv3 results database
(rocpd sqlite, the default output format of this image's rocprofv3).
usage: python tools/rocpd_stats.py run_results.db [top_n] [--csv out.csv]"""
import csv
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    q = ("select s.kernel_name, count(*), sum(d.end - d.start), avg(d.end - d.start), min(d.end - d.start), "
         "max(d.end - d.start) from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id "
         "group by s.kernel_name order by 3 desc")
    return [dict(zip(("Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs"), r)) for r in c.execute(q)]


if __name__ == "__main__":
    rows = stats(sys.argv[1])
    top = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 30
    if "--csv" in sys.argv:
        out = sys.argv[sys.argv.index("--csv") + 1]
        tot = sum(r["TotalDurationNs"] for r in rows)
        with open(out, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs",
                                              "MaxNs"])
            w.writeheader()
            for r in rows:
                w.writerow(dict(r, Percentage=100.0 * r["TotalDurationNs"] / tot))
    for r in rows[:top]:
        print(f'{r["TotalDurationNs"] / 1e6:9.3f} ms  n={r["Calls"]:>6} avg={r["AverageNs"] / 1e3:9.1f}us  {r["Name"][:100]}')
