# k_wino static-priority probe: C0 bench kernel report, in-tree vs tools/exp_*.so, 3 alternating reps
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3
cd $R
for rep in 1 2 3; do
for v in in-tree tools/exp_*.so; do
  if [ "$v" != in-tree ]; then export STIF_HIP_LIB=$R/$v; else unset STIF_HIP_LIB; fi
  timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 20 --kernel-report > gpurun_out/r3/ab.json 2> gpurun_out/r3/ab.err || { tail -30 gpurun_out/r3/ab.err; exit 1; }
  python - $v <<'PY'
import json, sys
d = json.loads(open("gpurun_out/r3/ab.json").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:36s}", d["value"], "Mpix/s", d["ms_per_step"], "ms")
PY
  grep "'wino'" gpurun_out/r3/ab.err | head -2
done
done
