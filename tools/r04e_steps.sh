#!/bin/bash
# round-4: what the AMP train step's time is made of: dropout (Philox) and the accurate SiLU
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
P="python3 tools/prof_train.py"
exec bash tools/gpu_steps.sh \
  "t_base:120:YK_AMP=1 python -u tools/train_time.py 512" \
  "t_nodrop:120:YK_AMP=1 YK_DROPOUT=0 python -u tools/train_time.py 512" \
  "t_fsilu:120:YK_AMP=1 YK_LIB_PATH=tools/_variants/fsilu/libyacht_hip.so python -u tools/train_time.py 512" \
  "p_base:200:YK_AMP=1 rocprofv3 --kernel-trace --stats -d gpurun_out/trp_base -o tr --output-format csv -- $P" \
  "p_nodrop:200:YK_AMP=1 YK_DROPOUT=0 rocprofv3 --kernel-trace --stats -d gpurun_out/trp_nodrop -o tr --output-format csv -- $P" \
  "p_fsilu:200:YK_AMP=1 YK_LIB_PATH=tools/_variants/fsilu/libyacht_hip.so rocprofv3 --kernel-trace --stats -d gpurun_out/trp_fsilu -o tr --output-format csv -- $P"
