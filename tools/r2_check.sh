# Round-2 check on one MI355X: GPU suite (verbose, per-test timeout), then the default bench line.
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r2_gpu_tests.log 2>&1
echo "pytest rc=$?"
timeout -k 10 600 python -u bench.py > gpurun_out/r2_bench.log 2>&1
echo "bench rc=$?"
