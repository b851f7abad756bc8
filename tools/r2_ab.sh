# A/B of the in-tree library against tools/exp_*.so on the conv microbenchmarks (same box)
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_wino.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
for lib in "" tools/exp_*.so; do
  echo "== ${lib:-in-tree}"
  export STIF_HIP_LIB=${lib:+$R/$lib}
  [ -z "$lib" ] && unset STIF_HIP_LIB
  ONLY=wino16 timeout -k 10 120 python -u tools/bench_conv.py 2>&1 | grep -v amdgpu.ids | grep -v "max |"
  HW=128 ONLY=wino16 timeout -k 10 120 python -u tools/bench_conv.py 2>&1 | grep -v amdgpu.ids | grep -v "max |"
  timeout -k 10 120 python -u tools/bench_om.py 2>&1 | grep "G=8 N=6 256\|G=2 N=6 128"
done
