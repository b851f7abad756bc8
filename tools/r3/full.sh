# Round-3 evidence: the whole GPU suite, the default bench (all extra lines, CPU baseline, parity), then
# the C0 profile passes (tools/prof_c0.sh: kernel-trace stats, FETCH/WRITE, SQ MFMA-busy)
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r3/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r3/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r3/gpu_tests.log
timeout -k 10 900 python -u bench.py > gpurun_out/r3/bench.json 2> gpurun_out/r3/bench.err || { tail -30 gpurun_out/r3/bench.err; exit 1; }
tail -c 1500 gpurun_out/r3/bench.json
TAG=r03 bash tools/prof_c0.sh
