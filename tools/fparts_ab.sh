#!/bin/bash
# diagnostic (GPU box): the forward head split (2 / 4 workgroups per 16-row tile when the tiles do
# not fill the CUs) against one workgroup per tile (-DYK_FPARTS_MAX=1), interleaved over R rounds,
# at config 3's per-GPU shape (2048 x 200), 1024 x 100 and the bench shape (4096 x 100, no split).
# usage: tools/fparts_ab.sh R
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/variant_lib.sh p1 -DYK_FPARTS_MAX=1 > /dev/null && bash tools/variant_lib.sh p4 -DYK_FPARTS_MAX=4 > /dev/null || exit 3
B="python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-arena --no-train --no-coach --no-shape"
for r in $(seq 1 "${1:-2}"); do
  for shape in "2048 200" "1024 100" "4096 100"; do
    set -- $shape
    for v in p4 p1; do
      lib=/tmp/yk_$v/libyacht_hip.so
      YK_LIB_PATH=$lib timeout -k 10 150 $B --envs $1 --sims $2 > gpurun_out/fp_${v}_$1_$r.json 2> gpurun_out/fp_${v}_$1_$r.err || exit $?
      python3 -c "
import json; d=json.load(open('gpurun_out/fp_${v}_$1_$r.json'))
print('$v', '$1x$2', 'r$r', round(d['value']/1e6,3), 'M exp/s parts', d.get('forward_parts'), {k: v['avg_ms'] for k, v in d.get('kernel_ms', {}).items() if k in ('forward', 'expand_backup_select')})"
    done
  done
done
