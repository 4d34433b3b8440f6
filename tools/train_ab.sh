#!/bin/bash
# diagnostic (GPU box): interleaved A/B of the train step (tools/train_time.py, event-timed) between
# the in-tree library ("head"), the baseline ("base": tools/_variants/base if prebuilt, else the
# sources staged under ab_base/csrc) and prebuilt variants (tools/_variants/NAME/libyacht_hip.so).
# usage: tools/train_ab.sh [ROUNDS] [amp|f32] [NAME ...]
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
base=tools/_variants/base/libyacht_hip.so
if [ ! -f $base ]; then bash tools/variant_lib.sh base > /dev/null || exit 3; base=/tmp/yk_base/libyacht_hip.so; fi
R=${1:-3}; amp=1; [ "${2:-amp}" = f32 ] && amp=0
shift 2 2>/dev/null
names=(head base "$@")
for r in $(seq 1 "$R"); do
  for b in 512 64; do
    for n in "${names[@]}"; do
      lib=""; [ "$n" = base ] && lib=$base
      [ "$n" != head ] && [ "$n" != base ] && lib=tools/_variants/$n/libyacht_hip.so
      echo "$n r$r $(YK_AMP=$amp YK_LIB_PATH=$lib timeout -k 10 120 python -u tools/train_time.py $b 2>/dev/null | grep batch)"
    done
  done
done
