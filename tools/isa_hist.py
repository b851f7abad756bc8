"""Static instruction histogram of one kernel in a device assembly file (hipcc --cuda-device-only -S).

usage: python tools/isa_hist.py FILE.s SYMBOL_SUBSTRING [TOP]"""
import collections
import sys

s = open(sys.argv[1]).read()
sym = next(l.split(":")[0] for l in s.splitlines() if l.startswith("_Z") and ":" in l and sys.argv[2] in l.split(":")[0])
i = s.index(sym + ":")
body = s[i:s.index(".Lfunc_end", i)].splitlines()
c = collections.Counter()
for l in body:
    l = l.strip()
    if not l or l.startswith((".", ";")) or l.endswith(":"):
        continue
    c[l.split()[0]] += 1
print(sym, "total", sum(c.values()))
cls = collections.Counter()
for k, v in c.items():
    cls["mfma" if "mfma" in k else k.split("_")[0]] += v
print("  by class:", dict(cls.most_common()))
for k, v in c.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 60):
    print(f"  {k:34s}{v}")
