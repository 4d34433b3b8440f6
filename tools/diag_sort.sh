#!/bin/bash
# diagnostic (GPU box): policy-head tile demand in game order vs leaves grouped by class (tools/diag_sort.py)
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
set -e
bash tools/variant_lib.sh tiles -DYK_TILESTAT > /dev/null
YK_LIB_PATH=/tmp/yk_tiles/libyacht_hip.so timeout -k 5 300 python tools/diag_sort.py "$@" 2>&1 | grep -v amdgpu.ids
