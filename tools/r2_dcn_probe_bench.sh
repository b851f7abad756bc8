R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for rep in 1 2; do
  for v in "" DCN_EXP_NOFB DCN_EXP_NOFB+DCN_EXP_OMCOAL; do
    export STIF_HIP_LIB=${v:+$R/tools/exp_$v.so}; [ -z "$v" ] && unset STIF_HIP_LIB
    timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 20 > gpurun_out/pr.json 2> gpurun_out/pr.err || { tail -20 gpurun_out/pr.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/pr.json').read().strip().splitlines()[-1])
print('${v:-in-tree}', d['value'], d['ms_per_step'], {k: v['avg_us'] for k, v in d['hot_path_kernels'].items()})"
  done
done
