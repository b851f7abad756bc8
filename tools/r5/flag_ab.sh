#!/bin/bash
# Same-tree A/B of bench.py flag sets: FLAGS_A / FLAGS_B (/ FLAGS_C), alternating, REPS reps, C0 --steps 20.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5
mkdir -p $O
cd $R
for rep in $(seq ${REPS:-3}); do
  for v in A B C D; do
    eval "f=\$FLAGS_$v"
    [ -z "$f" ] && continue
    timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 20 $f > $O/fab.json 2> $O/fab.err \
      || { tail -30 $O/fab.err; exit 1; }
    python - "$f" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/r5/fab.json").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:28s}", d["value"], "Mpix/s", d["ms_per_step"], "ms")
PY
  done
done
