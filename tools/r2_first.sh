set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2a_gpu_tests.log 2>&1
timeout -k 10 300 python -u bench.py --config c0 --no-cpu-baseline --steps 10 --warmup 2 --kernel-report > gpurun_out/r2a_bench_c0.log 2>&1
timeout -k 10 300 python -u bench.py --config c1 --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/r2a_bench_c1.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r2a_prof_c0 -o run -- python3 $R/bench.py --config c0 --no-cpu-baseline --steps 5 --warmup 1 > $R/gpurun_out/r2a_prof_c0.log 2>&1
echo done
