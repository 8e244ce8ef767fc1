"""Per-kernel share of a rocprofv3 kernel_stats.csv: python tools/kshare.py <csv> [n] [steps]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"total {tot / 1e6:.3f} ms")
for r in rows[:n]:
    print(f"{float(r['TotalDurationNs']) / tot * 100:5.1f}% {int(r['Calls']):6d} {float(r['AverageNs']) / 1000:8.1f}us "
          f"{float(r['TotalDurationNs']) / 1e6:8.3f}ms {r['Name'][:100]}")
