#!/bin/bash
# round-4: AMP train parity after the native SiLU, its step time, block-2 phase stamps
cd "$(dirname "$0")/.." || exit 2
exec bash tools/gpu_steps.sh \
  "gtrain:400:python -u -m pytest tests/test_gpu_train.py tests/test_gpu_config5.py -x -q -s --timeout 300 --timeout-method thread" \
  "t_head:120:YK_AMP=1 python -u tools/train_time.py 512" \
  "amp_ts:120:YK_LIB_PATH=tools/_variants/amp/libyacht_hip.so python -u tools/diag_amp.py"
