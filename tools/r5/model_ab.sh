#!/bin/bash
# Model-level change check: C0 window outputs of the in-tree build vs tools/exp_base.so bit for bit, the model /
# config / parallel GPU tests, then the C0 bench (kernel report) alternating in-tree / base, REPS reps.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5
mkdir -p $O
cd $R
timeout -k 10 200 python -u tools/r5/dump_root.py 2>&1 | sed '/amdgpu.ids/d' || exit 1
ROOT=$R/tools/base_tree TAG=base CMP=in-tree timeout -k 10 200 python -u tools/r5/dump_root.py 2>&1 | sed '/amdgpu.ids/d' || exit 1
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_model.py tests/test_gpu_configs.py tests/test_gpu_parallel.py} -x -q \
  --timeout 300 --timeout-method thread > $O/model_tests.log 2>&1 || { tail -40 $O/model_tests.log; exit 1; }
tail -1 $O/model_tests.log
for rep in $(seq ${REPS:-2}); do
  for v in in-tree tools/base_tree; do
    if [ "$v" != in-tree ]; then B=$R/$v; else B=$R; fi
    (cd $B && timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 20) > $O/ab.json 2> $O/ab.err \
      || { tail -30 $O/ab.err; exit 1; }
    python - $v <<'PY'
import json, sys
d = json.loads(open("gpurun_out/r5/ab.json").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:24s}", d["value"], "Mpix/s", d["ms_per_step"], "ms")
PY
  done
done
