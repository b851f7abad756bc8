#!/bin/bash
# Round-5 first GPU call: the torchrun/nccl world-1 bench (RCCL init + all_reduce path, kept as evidence),
# then the plain C0 bench with the kernel report.  Every GPU step under its own timeout; the first failure ends.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5
mkdir -p $O
cd $R
export NCCL_DEBUG=VERSION
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --gpus 1 --steps 20 --warmup 2 --backend nccl --no-cpu-baseline \
  > $O/bench_nccl_world1.json 2> $O/bench_nccl_world1.err || { tail -30 $O/bench_nccl_world1.err; exit 1; }
tail -1 $O/bench_nccl_world1.json | cut -c1-300
grep -i "rccl\|nccl version" $O/bench_nccl_world1.err | head -3
unset NCCL_DEBUG
timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 20 --kernel-report \
  > $O/bench_c0.json 2> $O/bench_c0.err || { tail -30 $O/bench_c0.err; exit 1; }
tail -1 $O/bench_c0.json | cut -c1-300
grep "'" $O/bench_c0.err | head -40
