#!/bin/bash
# diagnostic (GPU box): k_expand_backup launch span vs per-game times (tools/diag_xspan.py)
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
set -e
bash tools/variant_lib.sh xspan -DYK_XSPAN > /dev/null
YK_LIB_PATH=/tmp/yk_xspan/libyacht_hip.so timeout -k 5 200 python tools/diag_xspan.py "$@" 2>&1 | grep -v amdgpu.ids
