"""Print the top kernels of a rocprofv3 --stats kernel_stats.csv."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 14
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print(f"{float(r['TotalDurationNs']) / 1e6:9.2f} ms {100 * float(r['TotalDurationNs']) / tot:5.1f}% "
          f"calls {r['Calls']:>5} avg {float(r['AverageNs']) / 1e3:8.1f} us  {r['Name'][:100]}")
