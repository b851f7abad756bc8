# A/B of the working tree against tools/base_tree (a whole exported revision, tools/build_base.sh)
# and any tools/exp_*.so library variants on the full C0 bench (same box, alternating), after the
# model-level GPU parity tests on the in-tree build.  TESTS= overrides the test files.
R=$GRAFT_REPO_ROOT
cd $R
T=${TESTS:-tests/test_gpu_model.py tests/test_gpu_configs.py}
timeout -k 10 600 python -u -m pytest $T -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/abf_tests.log 2>&1 || { tail -30 gpurun_out/abf_tests.log; exit 1; }
tail -1 gpurun_out/abf_tests.log
for rep in 1 2; do
  for lib in "" base tools/exp_*.so; do
    [ "$lib" = tools/exp_base.so ] && continue   # the base tree runs with its own library
    B=bench.py
    [ "$lib" = base ] && B=tools/base_tree/bench.py
    export STIF_HIP_LIB=${lib:+$R/$lib}
    { [ -z "$lib" ] || [ "$lib" = base ]; } && unset STIF_HIP_LIB
    timeout -k 10 300 python -u $B --no-extras --no-cpu-baseline --steps ${STEPS:-20} ${BENCH_ARGS} > gpurun_out/abf.json 2> gpurun_out/abf.err || { tail -20 gpurun_out/abf.err; exit 1; }
    python - "${lib:-in-tree}" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/abf.json").read().strip().splitlines()[-1])
hot = {k: v["avg_us"] for k, v in d.get("hot_path_kernels", {}).items()}
print(f"{sys.argv[1]:24s} {d['value']:8.3f} Mpix/s  {d['ms_per_step']:8.3f} ms  dom {d['roofline']['avg_launch_us']} us  {hot}")
PY
  done
done
