#!/bin/bash
# Round-6 decoder A/B, second step: k_dec1 in 8-wave workgroups (DEC1_NW 8, in-tree) vs 4 (exp_DEC1_NW_4) vs the
# round-5 decoder (exp_base); decoder tests on the in-tree build first.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_fullsize.py tests/test_gpu_configs.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > $O/dec_tests2.log 2>&1 || { tail -40 $O/dec_tests2.log; exit 1; }
tail -1 $O/dec_tests2.log
run() {  # label, lib, config, steps
  if [ -n "$2" ]; then export STIF_HIP_LIB=$R/$2; else unset STIF_HIP_LIB; fi
  timeout -k 10 400 python -u bench.py --no-extras --no-cpu-baseline --config $3 --steps $4 --warmup 1 --kernel-report > $O/da.json 2> $O/da.err \
    || { tail -30 $O/da.err; exit 1; }
  echo "== $1 $3: $(python -c "import json;d=json.loads(open('$O/da.json').read().strip().splitlines()[-1]);print(d['value'],'Mpix/s',d['ms_per_step'],'ms')")"
  grep -E "\('dec" $O/da.err | head -4
}
for rep in 1 2; do
  run base tools/exp_base.so c0 10
  run dec1-nw4 tools/exp_DEC1_NW_4.so c0 10
  run in-tree "" c0 10
done
run base tools/exp_base.so c2 2
run dec1-nw4 tools/exp_DEC1_NW_4.so c2 2
run in-tree "" c2 2
