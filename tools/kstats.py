"""Print the per-kernel time split of a rocprofv3 --stats kernel_stats.csv (share, calls, avg, name)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 14]:
    print(f"{float(r['TotalDurationNs']) / tot * 100:5.1f}% {int(r['Calls']):5d} "
          f"{float(r['AverageNs']) / 1e3:9.1f}us {r['Name'][:80]}")
print(f"{tot / 1e6:.1f} ms total")
