#!/bin/bash
# round-4: k tiles per trunk dW item (YK_DW_KG): 2 (in-tree) vs 4 (round-4 default) vs 1, interleaved
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
T="python -u tools/train_time.py 512"
exec bash tools/gpu_steps.sh \
  "gtrain:300:python -u -m pytest tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread" \
  "kg2a:120:YK_AMP=1 $T" \
  "kg4a:120:YK_AMP=1 YK_LIB_PATH=tools/_variants/kg4/libyacht_hip.so $T" \
  "kg1a:120:YK_AMP=1 YK_LIB_PATH=tools/_variants/kg1/libyacht_hip.so $T" \
  "kg2b:120:YK_AMP=1 $T" \
  "kg4b:120:YK_AMP=1 YK_LIB_PATH=tools/_variants/kg4/libyacht_hip.so $T" \
  "kg1b:120:YK_AMP=1 YK_LIB_PATH=tools/_variants/kg1/libyacht_hip.so $T" \
  "p_kg2:200:YK_AMP=1 rocprofv3 --kernel-trace --stats -d gpurun_out/trp_kg2 -o tr --output-format csv -- python3 tools/prof_train.py"
