#!/bin/bash
# Round 4: validate the software-pipelined fused DCN_sep (k_dcn_sep_pipe) and A/B it.
# 1. the DCN_sep op tests of the in-tree build (the pipelined kernel forced by flag);
# 2. the C0/C1 model tests with every STIF DCN_sep launch on the pipelined kernel (tools/exp_DCNSEP_PIPE_1.so);
# 3. the DCN_sep microbenchmark and the C0 bench kernel report, in-tree vs every tools/exp_*.so, $REPS reps.
# Every GPU step under its own timeout; the first failure ends the call.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4
mkdir -p $O
cd $R
REPS=${REPS:-2}
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -k dcn_sep -x -q --timeout 120 --timeout-method thread \
  > $O/pipe_ops.log 2>&1 || { tail -40 $O/pipe_ops.log; exit 1; }
tail -2 $O/pipe_ops.log
STIF_HIP_LIB=$R/tools/exp_DCNSEP_PIPE_1.so timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py \
  -k "c0 or c1 or zero_state or range" -x -q --timeout 200 --timeout-method thread > $O/pipe_cfg.log 2>&1 \
  || { tail -40 $O/pipe_cfg.log; exit 1; }
tail -2 $O/pipe_cfg.log
for rep in $(seq $REPS); do
  for v in in-tree tools/exp_*.so; do
    if [ "$v" != in-tree ]; then export STIF_HIP_LIB=$R/$v; else unset STIF_HIP_LIB; fi
    echo "$v: $(N=48 HW=128 timeout -k 10 120 python3 tools/bench_dcnsep.py 2>&1 | grep -v amdgpu.ids | tr '\n' ' ')" || exit 1
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
    grep "'dcnsep'\|'dec" $O/ab.err | head -6
  done
done
