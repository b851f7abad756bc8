# fused DCN_sep tap pipeline: op parity (in-tree NW 4 and the NW 8 build), microbenchmark and C0 bench
# in-tree vs tools/exp_pipe8.so (NW 8 pipelined) vs tools/exp_head8.so (NW 8, previous commit)
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "dcn_sep" > gpurun_out/r3/dcnsep_ops.log 2>&1 || { tail -40 gpurun_out/r3/dcnsep_ops.log; exit 1; }
tail -1 gpurun_out/r3/dcnsep_ops.log
STIF_HIP_LIB=$R/tools/exp_pipe8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "dcn_sep" > gpurun_out/r3/dcnsep_ops8.log 2>&1 || { tail -40 gpurun_out/r3/dcnsep_ops8.log; exit 1; }
tail -1 gpurun_out/r3/dcnsep_ops8.log
for rep in 1 2; do
echo "in-tree: $(timeout -k 10 120 python3 tools/bench_dcnsep.py 2>&1 | grep -v amdgpu.ids)"
for lib in tools/exp_*.so; do
  echo "$lib: $(STIF_HIP_LIB=$R/$lib timeout -k 10 120 python3 tools/bench_dcnsep.py 2>&1 | grep -v amdgpu.ids)"
done
done
for v in in-tree tools/exp_pipe8.so tools/exp_head8.so in-tree tools/exp_pipe8.so tools/exp_head8.so; do
  if [ "$v" != in-tree ]; then export STIF_HIP_LIB=$R/$v; else unset STIF_HIP_LIB; fi
  timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 20 --kernel-report > gpurun_out/r3/ab.json 2> gpurun_out/r3/ab.err || { tail -30 gpurun_out/r3/ab.err; exit 1; }
  python - $v <<'PY'
import json, sys
d = json.loads(open("gpurun_out/r3/ab.json").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:28s}", d["value"], "Mpix/s", d["ms_per_step"], "ms", {k: v["avg_us"] for k, v in d["hot_path_kernels"].items() if "dcn" in k})
PY
done
