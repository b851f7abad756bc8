# Profile of the default (C0) bench: kernel-trace stats, FETCH/WRITE passes and one SQ
# MFMA-busy pass (separate rocprofv3 runs, MI355X_MICROARCH.md PMC rules).  TAG names the outputs.
set -e
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r03}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extras --steps 10 --warmup 2 --kernel-report > gpurun_out/${TAG}_bench_c0.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_stats -o run -- python3 $R/bench.py --no-cpu-baseline --no-extras --steps 5 --warmup 1 > $R/gpurun_out/${TAG}_stats.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/${TAG}_fetch -o run -- python3 $R/bench.py --no-cpu-baseline --no-extras --steps 1 --warmup 1 > $R/gpurun_out/${TAG}_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/${TAG}_write -o run -- python3 $R/bench.py --no-cpu-baseline --no-extras --steps 1 --warmup 1 > $R/gpurun_out/${TAG}_write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/${TAG}_mfma -o run -- python3 $R/bench.py --no-cpu-baseline --no-extras --steps 1 --warmup 1 > $R/gpurun_out/${TAG}_mfma.log 2>&1
echo done
