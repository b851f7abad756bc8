# k_wino start-stagger probe: trunk-conv microbenchmark and C0 kernel report, in-tree vs tools/exp_*.so
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3
cd $R
for rep in 1 2; do
  for lib in tools/exp_*.so; do
    echo "$lib: $(STIF_HIP_LIB=$R/$lib N=18 HW=128 ONLY=wino16 timeout -k 10 120 python3 tools/bench_conv.py 2>&1 | grep -v amdgpu.ids | tr '\n' ' ')"
  done
done
for v in tools/exp_*.so; do
  export STIF_HIP_LIB=$R/$v
  timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 20 --kernel-report > gpurun_out/r3/ab.json 2> gpurun_out/r3/ab.err || { tail -30 gpurun_out/r3/ab.err; exit 1; }
  python - $v <<'PY'
import json, sys
d = json.loads(open("gpurun_out/r3/ab.json").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:36s}", d["value"], "Mpix/s", d["ms_per_step"], "ms")
PY
  grep "'wino'" gpurun_out/r3/ab.err | head -3
done
