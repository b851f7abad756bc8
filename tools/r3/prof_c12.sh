# kernel-trace stats of the C1 and C2 configs (bench.py --config c1 / c2, 2 timed steps)
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for c in c1 c2; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03_stats_$c -o run -- python3 $R/bench.py --config $c --no-cpu-baseline --no-extras --steps 2 --warmup 1 > $R/gpurun_out/r03_stats_$c.log 2>&1
  tail -c 400 $R/gpurun_out/r03_stats_$c.log
done
