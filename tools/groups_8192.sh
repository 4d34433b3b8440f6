#!/bin/bash
# diagnostic (GPU box): config 5's per-GPU shape (8192 games x 100 sims) with 1, 2 and 4 game
# groups (with 4, each group's 128 row tiles take the forward head split), R rounds interleaved.
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python -u bench.py --envs 8192 --steps 1 --warmup 1 --no-cpu-baseline --no-arena --no-train --no-coach --no-shape"
for r in $(seq 1 "${1:-2}"); do
  for g in 1 2 4; do
    timeout -k 10 150 $B --groups $g > gpurun_out/g8k_${g}_$r.json 2> gpurun_out/g8k_${g}_$r.err || exit $?
    python3 -c "
import json; d=json.load(open('gpurun_out/g8k_${g}_$r.json'))
print('groups $g r$r', round(d['value']/1e6,3), 'M exp/s parts', d.get('forward_parts'), {k: v['avg_ms'] for k, v in d.get('kernel_ms', {}).items() if k in ('forward', 'expand_backup_select')})"
  done
done
