#!/bin/bash
# round 4: sine accuracy tool + torchrun nccl world-1 bench (the RCCL init / all_reduce / teardown path)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4
mkdir -p $O
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -o $O/sin_acc tools/experiments/sin_acc.hip 2>/dev/null \
  && timeout -k 10 60 $O/sin_acc > $O/sin_acc.log 2>&1 && cat $O/sin_acc.log || exit 1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 1 --steps 10 --warmup 2 > $O/torchrun_nccl_w1.json 2> $O/torchrun_nccl_w1.err || { tail -20 $O/torchrun_nccl_w1.err; exit 1; }
head -c 400 $O/torchrun_nccl_w1.json; echo
