"""Print the top kernels of a rocprofv3 run_results.db (rocpd SQLite output) and
optionally write a kernel_stats.csv in the --stats layout."""
import csv
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                 "from kernels group by name order by sum(duration) desc").fetchall()
tot = sum(r[2] for r in rows)
for name, k, s, a, lo, hi in rows[:n]:
    print(f"{s/1e6:9.1f} ms {100*s/tot:5.1f}% calls {k:7d} avg {a/1e3:8.1f} us  {name[:100]}")
print(f"total {tot/1e6:.1f} ms")
if len(sys.argv) > 3:
    with open(sys.argv[3], "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, k, s, a, lo, hi in rows:
            w.writerow([name, k, s, a, 100 * s / tot, lo, hi])
