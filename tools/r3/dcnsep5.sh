# fused DCN_sep (deterministic tap loop, biases in the accumulator init): determinism, op + model parity,
# microbenchmark and C0 bench in-tree (NW 4) vs tools/exp_DCNSEP_NW_8.so
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3
cd $R
for lib in in-tree tools/exp_DCNSEP_NW_8.so; do
  if [ "$lib" != in-tree ]; then export STIF_HIP_LIB=$R/$lib; else unset STIF_HIP_LIB; fi
  timeout -k 10 300 python -u tools/r3/det_model.py 2>&1 | grep -v amdgpu.ids
  timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q --timeout 120 --timeout-method thread -k "dcn_sep" > gpurun_out/r3/dcnsep_ops.log 2>&1 || { tail -30 gpurun_out/r3/dcnsep_ops.log; exit 1; }
  tail -1 gpurun_out/r3/dcnsep_ops.log
done
unset STIF_HIP_LIB
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3/dcnsep_model.log 2>&1 || { tail -40 gpurun_out/r3/dcnsep_model.log; exit 1; }
tail -1 gpurun_out/r3/dcnsep_model.log
for rep in 1 2; do
  echo "in-tree: $(timeout -k 10 120 python3 tools/bench_dcnsep.py 2>&1 | grep -v amdgpu.ids)"
  echo "NW8: $(STIF_HIP_LIB=$R/tools/exp_DCNSEP_NW_8.so timeout -k 10 120 python3 tools/bench_dcnsep.py 2>&1 | grep -v amdgpu.ids)"
done
for v in in-tree tools/exp_DCNSEP_NW_8.so in-tree tools/exp_DCNSEP_NW_8.so; do
  if [ "$v" != in-tree ]; then export STIF_HIP_LIB=$R/$v; else unset STIF_HIP_LIB; fi
  timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 20 --kernel-report > gpurun_out/r3/ab.json 2> gpurun_out/r3/ab.err || { tail -30 gpurun_out/r3/ab.err; exit 1; }
  python - $v <<'PY'
import json, sys
d = json.loads(open("gpurun_out/r3/ab.json").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:28s}", d["value"], "Mpix/s", d["ms_per_step"], "ms", {k: v["avg_us"] for k, v in d["hot_path_kernels"].items()})
PY
done
