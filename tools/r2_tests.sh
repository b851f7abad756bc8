# GPU suite only (verbose, per-test timeout).
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r2_gpu_tests.log 2>&1
echo "pytest rc=$?"
tail -3 gpurun_out/r2_gpu_tests.log
