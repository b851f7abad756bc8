# k_dcn_sep microbenchmark at the C0 L1 shape: in-tree, two-kernel path, tools/exp_*.so probes; then the
# fused-DCN op parity tests.
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "dcn_sep" > gpurun_out/r3/dcnsep_ops.log 2>&1 || { tail -40 gpurun_out/r3/dcnsep_ops.log; exit 1; }
tail -1 gpurun_out/r3/dcnsep_ops.log
for rep in 1 2; do
  FUSED=0 timeout -k 10 120 python3 tools/bench_dcnsep.py 2>&1 | grep -v amdgpu.ids
  timeout -k 10 120 python3 tools/bench_dcnsep.py 2>&1 | grep -v amdgpu.ids
  for lib in tools/exp_*.so; do
    [ -e "$lib" ] || continue
    echo "$lib: $(STIF_HIP_LIB=$R/$lib timeout -k 10 120 python3 tools/bench_dcnsep.py 2>&1 | grep -v amdgpu.ids)"
  done
done
