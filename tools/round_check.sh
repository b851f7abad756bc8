# Round check on one MI355X: GPU test suite, smoke(), C1 bench line (with CPU baseline), C2 bench line.
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/bench_c1.log 2>&1
timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/bench_c2.log 2>&1
echo done
