# Full C0 bench (no CPU baseline / extras) for the in-tree library and every tools/exp_*.so variant,
# alternating, REPS rounds (same box): value, ms per step and the DCN / decoder kernel averages.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
  for lib in "" tools/exp_*.so; do
    if [ -n "$lib" ]; then export STIF_HIP_LIB=$R/$lib; else unset STIF_HIP_LIB; fi
    timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps ${STEPS:-20} ${BENCH_ARGS} > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
    python - "${lib:-in-tree}" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab.json").read().strip().splitlines()[-1])
hot = {k: v["avg_us"] for k, v in d.get("hot_path_kernels", {}).items()}
print(f"{sys.argv[1]:28s} {d['value']:8.3f} Mpix/s  {d['ms_per_step']:8.3f} ms  dom {d['roofline']['avg_launch_us']} us  {hot}")
PY
  done
done
