#!/bin/bash
# Review r5 item 5(b): the strict-fp32 C0 line (bench --mfma f32) over 10 timed steps, same box, alternating the round-4
# tree (tools/r04_tree: its own host code and library) with the current tree, 3 reps.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6
mkdir -p $O
for rep in 1 2 3; do
  for tree in tools/r04_tree .; do
    cd $R/$tree
    timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --mfma f32 --steps 10 --warmup 2 > $O/f32.json 2> $O/f32.err \
      || { tail -20 $O/f32.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/f32.json').read().strip().splitlines()[-1]);print('$tree', d['value'],'Mpix/s',d['ms_per_step'],'ms')"
  done
done
