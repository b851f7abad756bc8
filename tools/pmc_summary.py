"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into profiles/pmc_rNN.json.

usage: python tools/pmc_summary.py ROUND FETCH_CSV WRITE_CSV OUT_JSON

The bench's dominant kernel (residual 3x3 conv) is summarised per launch; every other kernel gets
its averages.  Corrections (MI355X_MICROARCH.md, HBM/rocprofv3 section): both counters are in KiB;
FETCH_SIZE undercounts 16-B-per-lane reads by 2x on gfx950.  Algorithmic bytes of the dominant
kernel: in0 + residual read + output write = 3 x 256 B per pixel (64 fp32 channels).
"""
import csv
import json
import sys
from collections import defaultdict

DOMINANT = "k_conv<3, 1, 2, 2, 4, 0, 3>"


def load(path):
    per = defaultdict(list)
    grid = defaultdict(list)
    for r in csv.DictReader(open(path)):
        per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
        grid[r["Kernel_Name"]].append(int(r["Grid_Size"]))
    return per, grid


def main():
    rnd, fcsv, wcsv, out = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4]
    fetch, grid = load(fcsv)
    write, _ = load(wcsv)
    dom = [k for k in fetch if DOMINANT in k]
    assert len(dom) == 1, dom
    k = dom[0]
    fb = 2 * 1024 * sum(fetch[k]) / len(fetch[k])
    wb = 1024 * sum(write[k]) / len(write[k])
    # a 256-thread workgroup covers 8 rows x 32 columns = 256 output pixels of its item (one slice:
    # cout 64), so output pixels = grid size when H % 8 == 0 and W % 32 == 0 (the C1 sizes)
    px = grid[k]
    alg = 3 * 256 * sum(px) / len(px)
    res = {
        "round": int(rnd),
        "command": "rocprofv3 --pmc FETCH_SIZE (pass 1) / --pmc WRITE_SIZE (pass 2) --output-format csv "
                   "-- python bench.py --steps 1 --warmup 1 --no-cpu-baseline",
        "kernel": k,
        "correction": "FETCH_SIZE and WRITE_SIZE are KiB; FETCH_SIZE x2 for 16-B/lane reads on gfx950 "
                      "(MI355X_MICROARCH.md HBM section)",
        "fetch_bytes_per_launch": fb,
        "write_bytes_per_launch": wb,
        "hbm_bytes_per_launch": fb + wb,
        "algorithmic_bytes_per_launch": alg,
        "dispatches": len(fetch[k]),
        "per_kernel": {n: {"FETCH_SIZE_KB_avg": sum(v) / len(v), "dispatches": len(v),
                           "WRITE_SIZE_KB_avg": sum(write.get(n, [0])) / max(1, len(write.get(n, [0])))}
                       for n, v in fetch.items()},
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({x: res[x] for x in ("kernel", "hbm_bytes_per_launch", "algorithmic_bytes_per_launch")}))


if __name__ == "__main__":
    main()
