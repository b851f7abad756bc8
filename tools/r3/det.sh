# determinism of every fused dcn_sep launch of a C0 window + the many-workgroup op test, per build
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3
cd $R
for lib in in-tree tools/exp_*.so; do
  if [ "$lib" != in-tree ]; then export STIF_HIP_LIB=$R/$lib; else unset STIF_HIP_LIB; fi
  timeout -k 10 300 python -u tools/r3/det_model.py 2>&1 | grep -v amdgpu.ids
  timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q --timeout 120 --timeout-method thread -k "many_workgroups or batch_independent" 2>&1 | tail -1
done
