#!/bin/bash
# kernel reports of the C0 bench in both operand modes (one untimed step each, HIP events per launch kind)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4
mkdir -p $O
for mf in f16x3 f32; do
  timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 10 --mfma $mf --kernel-report \
    > $O/kreport_$mf.json 2> $O/kreport_$mf.err || { tail -20 $O/kreport_$mf.err; exit 1; }
  echo "== $mf $(python -c "import json;d=json.loads(open('$O/kreport_$mf.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")"
  grep "launches" $O/kreport_$mf.err | head -24
done
