#!/bin/bash
# Round-6 evidence of the current build: the full default bench line (extras + CPU baseline), then the C0 profile passes
# of tools/prof_c0.sh (kernel-trace stats, FETCH_SIZE, WRITE_SIZE, SQ/MFMA), TAG=r06.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6
cd $R
timeout -k 10 900 python -u bench.py > gpurun_out/r6/bench_full.json 2> gpurun_out/r6/bench_full.err || { tail -30 gpurun_out/r6/bench_full.err; exit 1; }
tail -1 gpurun_out/r6/bench_full.json | cut -c1-400
TAG=r06 timeout -k 10 900 bash tools/prof_c0.sh || exit 1
