#!/bin/bash
# C0 kernel report (bench.py --kernel-report, one untimed step, HIP events per launch kind) of the in-tree
# library and of each LIBS variant, alternating, REPS reps; GREP selects the kernel-kind lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
for rep in $(seq ${REPS:-2}); do
  for v in in-tree $LIBS; do
    if [ "$v" = in-tree ]; then unset STIF_HIP_LIB; else export STIF_HIP_LIB=$PWD/$v; fi
    timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 10 --kernel-report $FLAGS \
      > $O/kr.json 2> $O/kr.err || { tail -20 $O/kr.err; exit 1; }
    echo "== $v $(python -c "import json;d=json.loads(open('$O/kr.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")"
    grep "launches" $O/kr.err | grep "${GREP:-.}"
  done
done
unset STIF_HIP_LIB
