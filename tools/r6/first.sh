#!/bin/bash
# Round-6 first call: GPU suite on the inherited build, then the default C0 bench (no extras) for a same-box
# reference point.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 20 > $O/bench_c0.json 2> $O/bench_c0.err \
  || { tail -30 $O/bench_c0.err; exit 1; }
tail -1 $O/bench_c0.json | cut -c1-300
done
