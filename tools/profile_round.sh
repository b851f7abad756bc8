# Round profile of the C1 bench: rocprofv3 kernel-trace stats + two PMC passes (FETCH_SIZE,
# WRITE_SIZE; separate runs as MI355X_MICROARCH.md prescribes).  Outputs under gpurun_out/prof_*;
# the summaries worth keeping are copied into profiles/ by hand (tools/pmc_summary.py).
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_stats -o run -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/prof_stats.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof_fetch -o run -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 1 > $R/gpurun_out/prof_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof_write -o run -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 1 > $R/gpurun_out/prof_write.log 2>&1
echo done
