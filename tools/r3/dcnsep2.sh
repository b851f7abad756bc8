# fused DCN_sep v2: op + model parity, microbenchmark (with phase probes), C0 bench fused vs two-kernel
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "dcn_sep" > gpurun_out/r3/dcnsep_ops.log 2>&1 || { tail -40 gpurun_out/r3/dcnsep_ops.log; exit 1; }
tail -1 gpurun_out/r3/dcnsep_ops.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3/dcnsep_model.log 2>&1 || { tail -40 gpurun_out/r3/dcnsep_model.log; exit 1; }
tail -1 gpurun_out/r3/dcnsep_model.log
FUSED=0 timeout -k 10 120 python3 tools/bench_dcnsep.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 120 python3 tools/bench_dcnsep.py 2>&1 | grep -v amdgpu.ids
for lib in tools/exp_*.so; do
  echo "$lib: $(STIF_HIP_LIB=$R/$lib timeout -k 10 120 python3 tools/bench_dcnsep.py 2>&1 | grep -v amdgpu.ids)"
done
for f in 1 0 1 0; do
  timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 20 --fused-dcn $f --kernel-report > gpurun_out/r3/ab_$f.json 2> gpurun_out/r3/ab_$f.err || { tail -30 gpurun_out/r3/ab_$f.err; exit 1; }
  python - $f <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/r3/ab_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print("fused" if sys.argv[1] == "1" else "two-kernel", d["value"], "Mpix/s", d["ms_per_step"], "ms", {k: v["avg_us"] for k, v in d["hot_path_kernels"].items()})
PY
done
grep -E "dcn|4, 0, 216" gpurun_out/r3/ab_1.err gpurun_out/r3/ab_0.err | head -20
cd /tmp && export TMPDIR=/tmp
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES"
C2="SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_MFMA_MOPS_F16"
C3="SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_IFETCH SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
i=0
for C in "$C1" "$C2" "$C3"; do
  i=$((i+1))
  REPS=3 timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/r3/dcnsep2_sq$i -o run -- python3 $R/tools/bench_dcnsep.py > $R/gpurun_out/r3/dcnsep2_sq$i.log 2>&1
  for e in 1 3; do
    STIF_HIP_LIB=$R/tools/exp_DCNSEP_EXP_$e.so REPS=3 timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/r3/dcnsep2_e${e}_sq$i -o run -- python3 $R/tools/bench_dcnsep.py > $R/gpurun_out/r3/dcnsep2_e${e}_sq$i.log 2>&1
  done
done
echo "== full"; python3 $R/tools/sq_summary.py k_dcn_sep $R/gpurun_out/r3/dcnsep2_sq1 $R/gpurun_out/r3/dcnsep2_sq2 $R/gpurun_out/r3/dcnsep2_sq3
echo "== no phase 1"; python3 $R/tools/sq_summary.py k_dcn_sep $R/gpurun_out/r3/dcnsep2_e1_sq1 $R/gpurun_out/r3/dcnsep2_e1_sq2 $R/gpurun_out/r3/dcnsep2_e1_sq3
echo "== no phase 2"; python3 $R/tools/sq_summary.py k_dcn_sep $R/gpurun_out/r3/dcnsep2_e3_sq1 $R/gpurun_out/r3/dcnsep2_e3_sq2 $R/gpurun_out/r3/dcnsep2_e3_sq3
