#!/bin/bash
# round-4: parity of the net prior (selfplay, net, config 5) and the A/B after the head's 3-product GEMM
cd "$(dirname "$0")/.." || exit 2
exec bash tools/gpu_steps.sh \
  "gtests:600:python -u -m pytest tests/test_gpu_selfplay.py tests/test_gpu_net.py tests/test_gpu_config5.py tests/test_gpu_arena.py -x -q -s --timeout 300 --timeout-method thread" \
  "ab:420:bash tools/ab_bench.sh 2 fastexp=x"
