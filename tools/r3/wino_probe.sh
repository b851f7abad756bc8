# k_wino f16x3 trunk conv (C0 shape 16 x 128^2 x 64, RES / RELU epilogues): in-tree vs timing probes
# tools/exp_WINO_EXP_{1,2,3}.so (no staging DMA / no B refills / no output exchange)
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3
cd $R
for rep in 1 2; do
  echo "in-tree: $(N=16 HW=128 ONLY=wino16 timeout -k 10 120 python3 tools/bench_conv.py 2>&1 | grep -v amdgpu.ids | head -2 | tr '\n' ' ')"
  for lib in tools/exp_WINO_EXP_*.so; do
    echo "$lib: $(STIF_HIP_LIB=$R/$lib N=16 HW=128 ONLY=wino16 timeout -k 10 120 python3 tools/bench_conv.py 2>&1 | grep -v amdgpu.ids | head -2 | tr '\n' ' ')"
  done
done
# fused DCN_sep probes: no fallback loads (EXP 4), no phase 1 (EXP 1)
for rep in 1 2; do
  echo "in-tree: $(timeout -k 10 120 python3 tools/bench_dcnsep.py 2>&1 | grep -v amdgpu.ids)"
  for lib in tools/exp_DCNSEP_EXP_*.so; do
    echo "$lib: $(STIF_HIP_LIB=$R/$lib timeout -k 10 120 python3 tools/bench_dcnsep.py 2>&1 | grep -v amdgpu.ids)"
  done
done
for v in in-tree tools/exp_DCNSEP_EXP_4.so; do
  if [ "$v" != in-tree ]; then export STIF_HIP_LIB=$R/$v; else unset STIF_HIP_LIB; fi
  timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 20 --kernel-report > gpurun_out/r3/ab.json 2> gpurun_out/r3/ab.err || { tail -30 gpurun_out/r3/ab.err; exit 1; }
  python - $v <<'PY'
import json, sys
d = json.loads(open("gpurun_out/r3/ab.json").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:28s}", d["value"], "Mpix/s", d["ms_per_step"], "ms", {k: v["avg_us"] for k, v in d["hot_path_kernels"].items() if "dcn" in k})
PY
done
