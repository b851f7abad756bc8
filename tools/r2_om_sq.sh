# SQ counter pass over tools/bench_om.py (k_wino_om, in-tree build).
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES"
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/om_sq -o run -- python3 $R/tools/bench_om.py > $R/gpurun_out/om_sq.log 2>&1
C2="SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"
timeout -s KILL 120 rocprofv3 --pmc $C2 --output-format csv -d $R/gpurun_out/om_sq2 -o run -- python3 $R/tools/bench_om.py > $R/gpurun_out/om_sq2.log 2>&1
echo done
