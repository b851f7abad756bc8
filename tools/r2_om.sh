# k_wino_om check: Winograd GPU tests, then the offset/mask conv timing for the in-tree build and
# every tools/exp_*.so variant.
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_wino.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/om_tests.log 2>&1 || { tail -30 gpurun_out/om_tests.log; exit 1; }
tail -2 gpurun_out/om_tests.log
echo "== in-tree" > gpurun_out/om_bench.log
timeout -k 10 120 python -u tools/bench_om.py >> gpurun_out/om_bench.log 2>&1 || exit 1
for f in tools/exp_*.so; do
  echo "== $(basename $f .so)" >> gpurun_out/om_bench.log
  STIF_HIP_LIB=$R/$f timeout -k 10 120 python -u tools/bench_om.py >> gpurun_out/om_bench.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/om_bench.log
