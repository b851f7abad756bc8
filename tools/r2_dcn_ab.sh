# DCN-core experiment libraries (tools/build_obj_variants.sh dcn ...) on one box: DCN GPU tests for the
# variants named in VALID, the k_dcn microbenchmark at the C0 L1 / L2 shapes for every library, then the
# full C0 bench for the in-tree library and the VALID variants, alternating, twice.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
for v in $VALID; do
  STIF_HIP_LIB=$R/tools/exp_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "dcn" -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/dcnab_t_$v.log 2>&1 || { echo "$v tests FAILED"; tail -20 gpurun_out/dcnab_t_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/dcnab_t_$v.log)"
done
for rep in 1 2; do
  for lib in "" tools/exp_*.so; do
    export STIF_HIP_LIB=${lib:+$R/$lib}; [ -z "$lib" ] && unset STIF_HIP_LIB
    for shp in "48 128" "24 128" "48 64"; do
      set -- $shp
      r=$(N=$1 HW=$2 timeout -k 10 120 python -u tools/bench_dcn16.py 2>&1 | grep "dcn f16x3") || { echo "micro failed $lib"; exit 1; }
      echo "${lib:-in-tree} N=$1 HW=$2 $r"
    done
  done
done
for rep in 1 2; do
  for v in "" $VALID; do
    export STIF_HIP_LIB=${v:+$R/tools/exp_$v.so}; [ -z "$v" ] && unset STIF_HIP_LIB
    timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 20 > gpurun_out/dcnab.json 2> gpurun_out/dcnab.err || { tail -20 gpurun_out/dcnab.err; exit 1; }
    python - "${v:-in-tree}" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/dcnab.json").read().strip().splitlines()[-1])
hot = {k: v["avg_us"] for k, v in d.get("hot_path_kernels", {}).items()}
print(f"{sys.argv[1]:24s} {d['value']:8.3f} Mpix/s  {d['ms_per_step']:8.3f} ms  {hot}")
PY
  done
done
