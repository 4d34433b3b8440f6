#!/bin/bash
# diagnostic (GPU box): policy-head tile demand under valid-only columns (tools/diag_tiles.py)
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
set -e
bash tools/variant_lib.sh tiles -DYK_TILESTAT > /dev/null
YK_LIB_PATH=/tmp/yk_tiles/libyacht_hip.so timeout -k 5 200 python tools/diag_tiles.py "$@" 2>&1 | grep -v amdgpu.ids
