# Fused DCN_sep: op parity, model parity, then the C0 bench: fused (unrolled / rolled phase 2, tools/exp_*.so)
# vs the two-kernel path, with the per-kind launch report (same box, alternating).
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "dcn_sep" > gpurun_out/r3/dcnsep_ops.log 2>&1 || { tail -40 gpurun_out/r3/dcnsep_ops.log; exit 1; }
tail -1 gpurun_out/r3/dcnsep_ops.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_configs.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3/dcnsep_model.log 2>&1 || { tail -40 gpurun_out/r3/dcnsep_model.log; exit 1; }
tail -1 gpurun_out/r3/dcnsep_model.log
for rep in 1 2; do
for v in "in-tree:1" "in-tree:0" "tools/exp_DCNSEP_ROLL_1.so:1"; do
  lib=${v%%:*}; f=${v##*:}
  if [ "$lib" != in-tree ]; then export STIF_HIP_LIB=$R/$lib; else unset STIF_HIP_LIB; fi
  tag=$(basename $lib .so)_$f
  timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 20 --fused-dcn $f --kernel-report > gpurun_out/r3/ab_$tag.json 2> gpurun_out/r3/ab_$tag.err || { tail -30 gpurun_out/r3/ab_$tag.err; exit 1; }
  python - $tag <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/r3/ab_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:28s}", d["value"], "Mpix/s", d["ms_per_step"], "ms", {k: v["avg_us"] for k, v in d["hot_path_kernels"].items()})
PY
done
done
unset STIF_HIP_LIB
grep -E "dcn|4, 0, 216" gpurun_out/r3/ab_in-tree_1.err gpurun_out/r3/ab_in-tree_0.err | head -20
