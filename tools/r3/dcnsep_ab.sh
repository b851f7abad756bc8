# fused DCN_sep A/B: in-tree vs every tools/exp_*.so (one-object variants, tools/build_obj_variants.sh):
# microbenchmark at the C0 L1 shape (2 reps), then the C0 bench kernel report
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3
cd $R
for rep in 1 2; do
  echo "in-tree: $(timeout -k 10 120 python3 tools/bench_dcnsep.py 2>&1 | grep -v amdgpu.ids)"
  for lib in tools/exp_*.so; do
    echo "$lib: $(STIF_HIP_LIB=$R/$lib timeout -k 10 120 python3 tools/bench_dcnsep.py 2>&1 | grep -v amdgpu.ids)"
  done
done
for v in in-tree tools/exp_*.so; do
  if [ "$v" != in-tree ]; then export STIF_HIP_LIB=$R/$v; else unset STIF_HIP_LIB; fi
  timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 10 --kernel-report > gpurun_out/r3/ab.json 2> gpurun_out/r3/ab.err || { tail -30 gpurun_out/r3/ab.err; exit 1; }
  python - $v <<'PY'
import json, sys
d = json.loads(open("gpurun_out/r3/ab.json").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:36s}", d["value"], "Mpix/s", d["ms_per_step"], "ms", {k: v["avg_us"] for k, v in d["hot_path_kernels"].items() if "dcn" in k})
PY
done
