# fused DCN_sep change: its op / model / config parity tests on the in-tree build, then the A/B
# (tools/r3/dcnsep_ab.sh: microbenchmark + C0 kernel report, in-tree vs tools/exp_*.so)
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_configs.py tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread -k "dcn_sep or c0 or c1 or model or reference or deterministic" > gpurun_out/r3/dcnsep_tests.log 2>&1 || { tail -40 gpurun_out/r3/dcnsep_tests.log; exit 1; }
tail -1 gpurun_out/r3/dcnsep_tests.log
bash tools/r3/dcnsep_ab.sh
