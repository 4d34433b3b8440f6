#!/bin/bash
# diagnostic (GPU box): interleaved A/B of the train step (tools/train_time.py) between the in-tree
# library ("head") and the staged baseline sources (ab_base/csrc, "base").  usage: tools/train_ab.sh [ROUNDS]
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
bash tools/variant_lib.sh base > /dev/null || exit 3
for r in $(seq 1 "${1:-3}"); do
  for b in 512 64; do
    echo "head r$r $(timeout -k 10 120 python -u tools/train_time.py $b 2>/dev/null | grep batch)"
    echo "base r$r $(YK_LIB_PATH=/tmp/yk_base/libyacht_hip.so timeout -k 10 120 python -u tools/train_time.py $b 2>/dev/null | grep batch)"
  done
done
