# Default bench (all extra lines, CPU baseline, parity) after the config tests touched by the last change.
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 400 --timeout-method thread -k "chunked" > gpurun_out/r3/gpu_tests2.log 2>&1 || { tail -40 gpurun_out/r3/gpu_tests2.log; exit 1; }
tail -1 gpurun_out/r3/gpu_tests2.log
timeout -k 10 900 python -u bench.py > gpurun_out/r3/bench.json 2> gpurun_out/r3/bench.err || { tail -30 gpurun_out/r3/bench.err; exit 1; }
tail -c 4000 gpurun_out/r3/bench.json
