# fused DCN_sep launch-size tile-height selection: the DCN op / config / model tests on the in-tree build,
# then C0 bench kernel reports (and C1) alternating with the previous commit's library (tools/exp_base.so)
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_configs.py tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread -k "dcn_sep or c0 or c1 or model or reference or deterministic" > gpurun_out/r3/nw_tests.log 2>&1 || { tail -40 gpurun_out/r3/nw_tests.log; exit 1; }
tail -1 gpurun_out/r3/nw_tests.log
for rep in 1 2; do
for v in in-tree tools/exp_base.so; do
  if [ "$v" != in-tree ]; then export STIF_HIP_LIB=$R/$v; else unset STIF_HIP_LIB; fi
  for c in c0 c1; do
    timeout -k 10 300 python -u bench.py --config $c --no-extras --no-cpu-baseline --steps 10 --kernel-report > gpurun_out/r3/ab.json 2> gpurun_out/r3/ab.err || { tail -30 gpurun_out/r3/ab.err; exit 1; }
    python - $v $c <<'PY'
import json, sys
d = json.loads(open("gpurun_out/r3/ab.json").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:22s} {sys.argv[2]}", d["value"], "Mpix/s", d["ms_per_step"], "ms", {k: v["avg_us"] for k, v in d["hot_path_kernels"].items() if "dcn" in k})
PY
  done
done
done
