"""Print the top kernels of a rocprofv3 --stats kernel_stats.csv."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.1f} ms {float(r["Percentage"]):5.1f}% calls {r["Calls"]:>7} '
          f'avg {float(r["AverageNs"])/1e3:8.1f} us  {r["Name"][:100]}')
print(f"total {tot/1e6:.1f} ms")
