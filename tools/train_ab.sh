#!/bin/bash
# diagnostic (GPU box): interleaved A/B of the train step (tools/train_time.py, event-timed) between
# the in-tree library ("head") and the baseline ("base": tools/_variants/base if prebuilt, else the
# sources staged under ab_base/csrc).  usage: tools/train_ab.sh [ROUNDS] [amp|f32]
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
base=tools/_variants/base/libyacht_hip.so
if [ ! -f $base ]; then bash tools/variant_lib.sh base > /dev/null || exit 3; base=/tmp/yk_base/libyacht_hip.so; fi
amp=1; [ "${2:-amp}" = f32 ] && amp=0
for r in $(seq 1 "${1:-3}"); do
  for b in 512 64; do
    echo "head r$r $(YK_AMP=$amp timeout -k 10 120 python -u tools/train_time.py $b 2>/dev/null | grep batch)"
    echo "base r$r $(YK_AMP=$amp YK_LIB_PATH=$base timeout -k 10 120 python -u tools/train_time.py $b 2>/dev/null | grep batch)"
  done
done
