#!/bin/bash
# diagnostic (GPU box): config 5's per-GPU shape (8192 games x 100 sims) with one game group,
# two groups (head, the streams run free) and two groups with forward-to-forward stagger events
# (-DYK_STAGGER: head now runs without them), interleaved over R rounds.  usage: tools/stagger_ab.sh R
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/variant_lib.sh stag -DYK_STAGGER > /dev/null || exit 3
B="python -u bench.py --envs 8192 --steps 2 --warmup 1 --no-cpu-baseline --no-arena --no-train --no-coach --no-shape"
for r in $(seq 1 "${1:-2}"); do
  for v in g1 g2 stag; do
    lib=""; extra="--groups 2"
    case $v in g1) extra="--groups 1" ;; stag) lib=/tmp/yk_stag/libyacht_hip.so ;; esac
    YK_LIB_PATH=$lib timeout -k 10 150 $B $extra > gpurun_out/stag_${v}_$r.json 2> gpurun_out/stag_${v}_$r.err || exit $?
    python3 -c "
import json,sys; d=json.load(open('gpurun_out/stag_${v}_$r.json'))
print('$v', 'r$r', round(d['value']/1e6,3), 'M exp/s', {k: v['avg_ms'] for k, v in d.get('kernel_ms', {}).items()})"
  done
done
