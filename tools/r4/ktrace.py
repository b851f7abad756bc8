"""Per-dispatch view of a rocprofv3 --kernel-trace CSV: the last bench step (from the last k_conv_first dispatch
on), each dispatch's workgroup count and duration (with -v), and per kernel the time in dispatches that launch
fewer workgroups than one round of the chip (512 = two per CU).
usage: python tools/r4/ktrace.py run_kernel_trace.csv [-v]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
first = max(i for i, r in enumerate(rows) if "k_conv_first" in r["Kernel_Name"])
step = rows[first:]
t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step)
print(f"last step: {len(step)} dispatches, span {(t1 - t0) / 1e6:.3f} ms, kernel time {busy / 1e6:.3f} ms")
small = defaultdict(lambda: [0, 0.0])
allk = defaultdict(lambda: [0, 0.0])
for r in step:
    wg = 1
    for d in "XYZ":
        wg *= int(r[f"Grid_Size_{d}"]) // max(1, int(r[f"Workgroup_Size_{d}"]))
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    name = r["Kernel_Name"].split("(stif")[0].split("(float")[0].replace("void ", "").replace("(anonymous namespace)::", "")[:48]
    allk[name][0] += 1
    allk[name][1] += d
    if wg < 512:
        small[name][0] += 1
        small[name][1] += d
    if "-v" in sys.argv:
        print(f"  {d:8.1f} us  {wg:7d} WG  {name}")
tot = sum(v[1] for v in small.values())
print(f"dispatches with < 512 workgroups: {sum(v[0] for v in small.values())}, {tot / 1e3:.3f} ms")
for k, (n, d) in sorted(small.items(), key=lambda kv: -kv[1][1]):
    print(f"  {n:4d} x {d / n:7.1f} us = {d / 1e3:6.3f} ms  {k}   (all: {allk[k][0]} x, {allk[k][1] / 1e3:.3f} ms)")
