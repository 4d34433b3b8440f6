#!/bin/bash
# diagnostic (GPU box): descent/expand phase accounting (-DYK_SEL_TIMING, tools/diag_select.py)
# of the in-tree sources and of the staged baseline (ab_base/csrc).  usage: tools/diag_ab.sh [FLAGS]
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
set -e
bash tools/variant_lib.sh headt -DYK_SEL_TIMING "$@" > /dev/null
bash tools/variant_lib.sh baset -DYK_SEL_TIMING > /dev/null
for n in headt baset; do
  echo "== $n"
  YK_LIB_PATH=/tmp/yk_$n/libyacht_hip.so timeout -k 5 200 python tools/diag_select.py 2>&1 | grep -v amdgpu.ids
done
