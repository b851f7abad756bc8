#!/bin/bash
# Round-4 A/B driver: parity tests of the in-tree build ($TESTS), then the trunk-conv microbenchmark and the
# C0 bench kernel report, in-tree vs every tools/exp_*.so, alternating, $REPS reps.  Every GPU step under its
# own timeout; the first failure ends the call.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4
mkdir -p $O
cd $R
TESTS=${TESTS:-"tests/test_gpu_wino.py"}
REPS=${REPS:-2}
if [ "$TESTS" != none ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > $O/ab_tests.log 2>&1 \
    || { tail -40 $O/ab_tests.log; exit 1; }
  tail -2 $O/ab_tests.log
fi
for rep in $(seq $REPS); do
  for v in in-tree tools/exp_*.so; do
    if [ "$v" != in-tree ]; then export STIF_HIP_LIB=$R/$v; else unset STIF_HIP_LIB; fi
    echo "$v: $(N=18 HW=128 ONLY=wino16 timeout -k 10 120 python3 tools/bench_conv.py 2>&1 | grep -v amdgpu.ids | tr '\n' ' ')" || exit 1
  done
done
unset STIF_HIP_LIB
for rep in $(seq $REPS); do
  for v in in-tree tools/exp_*.so; do
    if [ "$v" != in-tree ]; then export STIF_HIP_LIB=$R/$v; else unset STIF_HIP_LIB; fi
    timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 20 --kernel-report > $O/ab.json 2> $O/ab.err \
      || { tail -30 $O/ab.err; exit 1; }
    python - $v <<'PY'
import json, sys
d = json.loads(open("gpurun_out/r4/ab.json").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:36s}", d["value"], "Mpix/s", d["ms_per_step"], "ms")
PY
    grep "'wino'\|'dcnsep'\|'dec" $O/ab.err | head -12
  done
done
