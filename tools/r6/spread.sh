#!/bin/bash
# box-to-box / run-to-run spread of the default bench line on the final build (3 runs of the C0 line, no extras)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline > gpurun_out/r6/spread.json 2> gpurun_out/r6/spread.err || { tail -20 gpurun_out/r6/spread.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r6/spread.json').read().strip().splitlines()[-1]);print(d['value'],'Mpix/s',d['ms_per_step'],'ms, k_dcn_sep<0>',d['roofline']['avg_launch_us'],'us, frac',d['roofline']['frac'])"
done
