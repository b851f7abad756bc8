# Winograd A/B: parity of the in-tree build (Winograd op tests + model / config tests), then the trunk-conv
# microbenchmark and the C0 bench kernel report, in-tree vs every tools/exp_*.so
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_wino.py tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3/wino_tests.log 2>&1 || { tail -40 gpurun_out/r3/wino_tests.log; exit 1; }
tail -1 gpurun_out/r3/wino_tests.log
for rep in 1 2; do
  echo "in-tree: $(N=18 HW=128 ONLY=wino16 timeout -k 10 120 python3 tools/bench_conv.py 2>&1 | grep -v amdgpu.ids | tr '\n' ' ')"
  for lib in tools/exp_*.so; do
    echo "$lib: $(STIF_HIP_LIB=$R/$lib N=18 HW=128 ONLY=wino16 timeout -k 10 120 python3 tools/bench_conv.py 2>&1 | grep -v amdgpu.ids | tr '\n' ' ')"
  done
done
for rep in 1 2; do
for v in in-tree tools/exp_*.so; do
  if [ "$v" != in-tree ]; then export STIF_HIP_LIB=$R/$v; else unset STIF_HIP_LIB; fi
  timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 20 --kernel-report > gpurun_out/r3/ab.json 2> gpurun_out/r3/ab.err || { tail -30 gpurun_out/r3/ab.err; exit 1; }
  python - $v <<'PY'
import json, sys
d = json.loads(open("gpurun_out/r3/ab.json").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:36s}", d["value"], "Mpix/s", d["ms_per_step"], "ms")
PY
  grep "'wino'" gpurun_out/r3/ab.err | head -8
done
done
