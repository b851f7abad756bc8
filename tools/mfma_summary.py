"""Per-kernel MFMA-busy summary of a rocprofv3 SQ pass over the C0 bench (tools/prof_c0.sh, *_mfma).

usage: python tools/mfma_summary.py COUNTER_CSV > profiles/r02_mfma_c0.txt

MFMA-busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs): the share of the
kernel's SIMD cycles the MFMA pipe is busy (MI355X_MICROARCH.md: GRBM_GUI_ACTIVE sums the 8 XCDs,
SQ_VALU_MFMA_BUSY_CYCLES counts cycles).  VALU insts/wave-cycle = SQ_INSTS_VALU / SQ_WAVE_CYCLES
(quad-cycle units).  Kernels in first-dispatch order; per-dispatch means."""
import csv
import sys
from collections import OrderedDict, defaultdict

acc = OrderedDict()
for r in csv.DictReader(open(sys.argv[1])):
    acc.setdefault(r["Kernel_Name"], defaultdict(list))[r["Counter_Name"]].append(float(r["Counter_Value"]))
print("# SQ pass over one C0 bench step (rocprofv3 --pmc, tools/prof_c0.sh): per kernel, mean per dispatch.")
print("# MFMA-busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs): the share of SIMD "
      "cycles the MFMA pipe is busy")
mean = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}
for k, m in mean.items():
    simd = m.get("GRBM_GUI_ACTIVE", 0) / 8 * 1024
    busy = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / simd if simd else 0.0
    vpw = m.get("SQ_INSTS_VALU", 0) / m["SQ_WAVE_CYCLES"] if m.get("SQ_WAVE_CYCLES") else 0.0
    print(f"{k[:70]:70s} MFMA-busy {busy:6.3f}  VALU insts/wave-cycle {vpw:.3f}  GRBM {m.get('GRBM_GUI_ACTIVE', 0):.0f}")
print()
for k, m in mean.items():
    print(k[:70])
    for c, v in sorted(m.items()):
        print(f"   {c:32s} {v:16.0f}")
