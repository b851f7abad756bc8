set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread -k "c1_full_pair or dcn_sep_launches" > gpurun_out/r3/new_tests.log 2>&1 || { tail -40 gpurun_out/r3/new_tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/r3/new_tests.log | tail -6
bash tools/r3/dcnsep_sq.sh
