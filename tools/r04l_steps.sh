#!/bin/bash
# round-4: the fused gradient norm (yk_trainer_step skips k_amp_sq)
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
exec bash tools/gpu_steps.sh \
  "gtrain:400:python -u -m pytest tests/test_gpu_train.py tests/test_gpu_config5.py tests/test_gpu_coach.py -x -q --timeout 300 --timeout-method thread" \
  "td1:120:YK_AMP=1 python -u tools/train_time.py 512" \
  "td2:120:YK_AMP=1 python -u tools/train_time.py 512" \
  "p_trv:200:YK_AMP=1 rocprofv3 --kernel-trace --stats -d gpurun_out/trp_fnorm3 -o tr --output-format csv -- python3 tools/prof_train.py"
