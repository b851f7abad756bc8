# SQ counter passes over the DCN-core microbenchmark (tools/bench_dcn16.py at the C0 L1 shape, 48 x 128^2,
# two-row kernel): issue / wait / LDS / MFMA breakdown of k_dcn (one rocprofv3 pass per counter set).
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
N=48 HW=128 timeout -k 10 120 python3 $R/tools/bench_dcn16.py 2>&1 | grep -v amdgpu.ids
cd /tmp && export TMPDIR=/tmp
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES"
C2="SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_MFMA_MOPS_F16"
C3="SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
i=0
for C in "$C1" "$C2" "$C3"; do
  i=$((i+1))
  N=48 HW=128 timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/dcn_sq$i -o run -- python3 $R/tools/bench_dcn16.py > $R/gpurun_out/dcn_sq$i.log 2>&1
done
echo done
