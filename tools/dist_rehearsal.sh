#!/bin/bash
# GPU box: bench.py's multi-rank path with 2 ranks sharing the one GPU over gloo (the driver's
# N>1 runs use RCCL, one GPU per rank); small workload.
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --dist-backend gloo --envs 1024 --sims 25 --steps 1 --warmup 1 --coach-games 512
