# Round-2 evidence on one MI355X: GPU suite, smoke, default bench (C0, with CPU baseline + extras),
# kernel-trace stats and FETCH/WRITE/MFMA PMC passes of the C0 bench.  TAG names the outputs.
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r2}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.log 2>&1
echo "pytest rc=$?"; tail -2 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 600 python -u bench.py --kernel-report > gpurun_out/${TAG}_bench.log 2>&1 || { echo bench failed; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-300
TAG=$TAG bash tools/r2_prof.sh
