#!/bin/bash
# round-4 step runner: GPU self-play parity, the interleaved A/B and the select phase timings
cd "$(dirname "$0")/.." || exit 2
exec bash tools/gpu_steps.sh \
  "gtests:420:python -u -m pytest tests/test_gpu_selfplay.py -x -q -s --timeout 240 --timeout-method thread" \
  "ab:420:bash tools/ab_bench.sh 2 'noroot=--root-scan 0' fastexp=x" \
  "sel:200:YK_LIB_PATH=tools/_variants/sel/libyacht_hip.so timeout -k 5 180 python -u tools/diag_select.py"
