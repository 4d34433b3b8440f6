#!/bin/bash
# round-4: full GPU suite, divergence statistic (256 games), A/B of the softmax exp variants
cd "$(dirname "$0")/.." || exit 2
D="python -u -m pytest tests/test_gpu_divergence.py -x -q -s --timeout 300 --timeout-method thread"
exec bash tools/gpu_steps.sh \
  "gtests:700:python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread" \
  "div_head:330:YK_DIVERGENCE_STRIDE=16 YK_DIVERGENCE_TAG=head2 $D" \
  "ab:420:bash tools/ab_bench.sh 2 fastexp=x libexp=x 'noroot=--root-scan 0'"
