# A/B of the in-tree build against variant libraries (LIBS) on the larger bench configs (CFGS), alternating
# reps, every GPU step under its own timeout; prints each run's value and its kernel-report lines (GREP)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4
mkdir -p $O
cd $R
for rep in $(seq ${REPS:-2}); do
  for cfg in ${CFGS:-c1 c2}; do
    for v in in-tree $LIBS; do
      if [ "$v" != in-tree ]; then export STIF_HIP_LIB=$R/$v; else unset STIF_HIP_LIB; fi
      timeout -k 10 300 python -u bench.py --config $cfg --no-extras --no-cpu-baseline --steps ${STEPS:-3} --warmup 1 \
        --kernel-report > $O/abc.json 2> $O/abc.err || { tail -30 $O/abc.err; exit 1; }
      python - $v $cfg <<'PY'
import json, sys
d = json.loads(open("gpurun_out/r4/abc.json").read().strip().splitlines()[-1])
print(f"{sys.argv[2]} {sys.argv[1]:34s}", d["value"], "Mpix/s", d["ms_per_step"], "ms")
PY
      grep "${GREP:-dcnsep}" $O/abc.err
    done
  done
done
