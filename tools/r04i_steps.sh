#!/bin/bash
# round-4: the AMP train step (8-row trunk workgroups): parity, time twice (determinism), kernel stats, block stamps
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
exec bash tools/gpu_steps.sh \
  "gtrain:400:python -u -m pytest tests/test_gpu_train.py tests/test_gpu_config5.py -x -q --timeout 300 --timeout-method thread" \
  "td1:120:YK_AMP=1 python -u tools/train_time.py 512" \
  "td2:120:YK_AMP=1 python -u tools/train_time.py 512" \
  "p_trv:200:YK_AMP=1 rocprofv3 --kernel-trace --stats -d gpurun_out/trp_trv8 -o tr --output-format csv -- python3 tools/prof_train.py" \
  "amp_ts:120:YK_LIB_PATH=tools/_variants/amp/libyacht_hip.so python -u tools/diag_amp.py"
