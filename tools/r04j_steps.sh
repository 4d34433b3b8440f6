#!/bin/bash
# round-4: AMP step with the heads' dW inside k_amp_bwd (in-tree), and head partitions HQ 16 / BQ 12 (variants)
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
exec bash tools/gpu_steps.sh \
  "gtrain:400:python -u -m pytest tests/test_gpu_train.py tests/test_gpu_config5.py -x -q --timeout 300 --timeout-method thread" \
  "t_head:120:YK_AMP=1 python -u tools/train_time.py 512" \
  "t_hq16:120:YK_AMP=1 YK_LIB_PATH=tools/_variants/hq16/libyacht_hip.so python -u tools/train_time.py 512" \
  "t_hq16bq12:120:YK_AMP=1 YK_LIB_PATH=tools/_variants/hq16bq12/libyacht_hip.so python -u tools/train_time.py 512" \
  "t_head2:120:YK_AMP=1 python -u tools/train_time.py 512" \
  "p_trv:200:YK_AMP=1 rocprofv3 --kernel-trace --stats -d gpurun_out/trp_trv8 -o tr --output-format csv -- python3 tools/prof_train.py" \
  "p_hq:200:YK_AMP=1 YK_LIB_PATH=tools/_variants/hq16bq12/libyacht_hip.so rocprofv3 --kernel-trace --stats -d gpurun_out/trp_hq -o tr --output-format csv -- python3 tools/prof_train.py"
