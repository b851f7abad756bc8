"""Per-kernel mean of every counter in rocprofv3 --pmc CSV directories (one per pass).

usage: python tools/sq_summary.py FILTER DIR [DIR ...]"""
import csv
import glob
import sys
from collections import defaultdict

flt = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for d in sys.argv[2:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if flt in r["Kernel_Name"]:
                acc[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:32s} {sum(v) / len(v):16.0f}")
