"""Per-dispatch view of a rocprofv3 --kernel-trace CSV: the dispatches of the last N_STEP_KERNELS (default: the
dispatches after the last gap >= 2 ms, i.e. the last bench step), each with its workgroup count and duration,
and the time in launches that fill less than one round of the chip (< 512 four-wave workgroups).
usage: python tools/r4/ktrace.py run_kernel_trace.csv"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last step: walk back from the end until a gap of >= 2 ms (the bench's barrier / sync between steps)
i = len(rows) - 1
while i > 0 and int(rows[i]["Start_Timestamp"]) - int(rows[i - 1]["End_Timestamp"]) < 2_000_000:
    i -= 1
step = rows[i:]
t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step)
print(f"last step: {len(step)} dispatches, span {(t1 - t0) / 1e6:.3f} ms, kernel time {busy / 1e6:.3f} ms")
small = defaultdict(lambda: [0, 0.0])
for r in step:
    wg = int(r["Grid_Size"]) // max(1, int(r["Workgroup_Size"]))
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("(anonymous namespace)::", "")[:60]
    if wg < 512:
        small[name][0] += 1
        small[name][1] += d
    if len(sys.argv) > 2:
        print(f"  {d:8.1f} us  {wg:7d} WG  {name}")
tot = sum(v[1] for v in small.values())
print(f"dispatches with < 512 workgroups: {sum(v[0] for v in small.values())}, {tot / 1e3:.3f} ms")
for k, (n, d) in sorted(small.items(), key=lambda kv: -kv[1][1]):
    print(f"  {n:4d} x {d / n:7.1f} us = {d / 1e3:6.3f} ms  {k}")
