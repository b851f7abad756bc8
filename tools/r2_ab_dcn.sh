# A/B of the DCN core (in-tree vs tools/exp_*.so): DCN GPU tests, then the C1 L1 and C0 L1 shapes
R=$GRAFT_REPO_ROOT
cd $R
for lib in "" tools/exp_*.so; do
  echo "== ${lib:-in-tree}"
  if [ -n "$lib" ]; then export STIF_HIP_LIB=$R/$lib; else unset STIF_HIP_LIB; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k dcn > gpurun_out/abd_tests.log 2>&1 || { tail -20 gpurun_out/abd_tests.log; exit 1; }
  tail -1 gpurun_out/abd_tests.log
  timeout -k 10 120 python -u tools/bench_dcn16.py 2>&1 | grep -v amdgpu.ids
  N=24 HW=128 timeout -k 10 120 python -u tools/bench_dcn16.py 2>&1 | grep -v amdgpu.ids
done
