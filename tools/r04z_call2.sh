#!/bin/bash
# round-4 evidence, part 2: the default bench line, the interleaved A/B, the divergence statistic,
# the descent / expansion phase stamps and the AMP train step time
cd "$(dirname "$0")/.." || exit 2
D="python -u -m pytest tests/test_gpu_divergence.py -x -q -s --timeout 300 --timeout-method thread"
exec bash tools/gpu_steps.sh \
  "bench:600:python -u bench.py > gpurun_out/bench_r04z.json" \
  "ab:500:bash tools/ab_bench.sh 2 'noroot=--root-scan 0' fastexp=x" \
  "div_head:330:YK_DIVERGENCE_STRIDE=16 YK_DIVERGENCE_TAG=head $D" \
  "div_fast:330:YK_DIVERGENCE_STRIDE=16 YK_DIVERGENCE_TAG=fastexp YK_LIB_PATH=tools/_variants/fastexp/libyacht_hip.so $D" \
  "sel:200:YK_LIB_PATH=tools/_variants/sel/libyacht_hip.so timeout -k 5 180 python -u tools/diag_select.py" \
  "t_amp:120:YK_AMP=1 python -u tools/train_time.py 512"
