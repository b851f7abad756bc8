# fused DCN_sep timing probes (tools/exp_DCNSEP_EXP_{1,3,4}.so: no phase 1 / no phase 2 / no fallback
# loads; wrong results) at the C0 L1 microbenchmark shape and in the C0 bench kernel report
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3
cd $R
for rep in 1 2; do
  echo "in-tree: $(timeout -k 10 120 python3 tools/bench_dcnsep.py 2>&1 | grep -v amdgpu.ids)"
  for lib in tools/exp_DCNSEP_EXP_*.so; do
    echo "$lib: $(STIF_HIP_LIB=$R/$lib timeout -k 10 120 python3 tools/bench_dcnsep.py 2>&1 | grep -v amdgpu.ids)"
  done
done
for v in in-tree tools/exp_DCNSEP_EXP_1.so tools/exp_DCNSEP_EXP_3.so; do
  if [ "$v" != in-tree ]; then export STIF_HIP_LIB=$R/$v; else unset STIF_HIP_LIB; fi
  timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 10 --kernel-report > gpurun_out/r3/ab.json 2> gpurun_out/r3/ab.err || { tail -30 gpurun_out/r3/ab.err; exit 1; }
  echo "$v"; grep dcnsep gpurun_out/r3/ab.err
done
