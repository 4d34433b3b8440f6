#!/bin/bash
# GPU box: the production self-play path of the in-tree library against the staged baseline
# (ab_base/csrc): the records must be identical (a layout change must not move a bit).
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
set -e
bash tools/variant_lib.sh base > /dev/null
YK_LIB_PATH=/tmp/yk_base/libyacht_hip.so timeout -k 5 120 python tools/engine_records_dump.py /tmp/rec_base.npz
timeout -k 5 120 python tools/engine_records_dump.py gpurun_out/rec_head.npz
cp /tmp/rec_base.npz gpurun_out/rec_base.npz
python - <<'PY'
import numpy as np
a, b = np.load("gpurun_out/rec_base.npz"), np.load("gpurun_out/rec_head.npz")
bad = [k for k in a.files if not np.array_equal(a[k], b[k])]
print("records identical" if not bad else f"records DIFFER: {bad}")
PY
