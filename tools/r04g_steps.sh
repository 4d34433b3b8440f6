#!/bin/bash
# round-4: AMP train parity + step time + per-kernel stats after the dW item order
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
exec bash tools/gpu_steps.sh \
  "gtrain:400:python -u -m pytest tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread" \
  "t_head:120:YK_AMP=1 python -u tools/train_time.py 512" \
  "p_head:200:YK_AMP=1 rocprofv3 --kernel-trace --stats -d gpurun_out/trp_head -o tr --output-format csv -- python3 tools/prof_train.py"
