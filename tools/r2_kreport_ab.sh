# Per-launch-kind time (bench.py --kernel-report: one untimed step, HIP events per launch) of the
# in-tree library and every tools/exp_*.so variant on the C0 bench, alternating, REPS times; KINDS
# is a grep pattern of the kinds to print.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
  for lib in "" tools/exp_*.so; do
    export STIF_HIP_LIB=${lib:+$R/$lib}; [ -z "$lib" ] && unset STIF_HIP_LIB
    timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 10 --kernel-report > gpurun_out/kr.json 2> gpurun_out/kr.err || { tail -20 gpurun_out/kr.err; exit 1; }
    echo "== ${lib:-in-tree} $(python -c "import json; d=json.loads(open('gpurun_out/kr.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
    grep -E "${KINDS:-.}" gpurun_out/kr.err || true
  done
done
