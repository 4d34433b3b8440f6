#!/bin/bash
# diagnostic (GPU box): bench at 1..4 game groups, interleaved, R rounds.  usage: tools/groups_ab.sh R [ARGS]
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${1:-2}; shift
for r in $(seq 1 "$R"); do
  for g in 1 2 3 4; do
    timeout -k 10 120 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-arena --no-train --groups $g "$@" \
      > gpurun_out/grp_${g}_$r.json 2> gpurun_out/grp_${g}_$r.err || exit $?
    python3 -c "
import json; d = json.load(open('gpurun_out/grp_${g}_$r.json')); k = d['kernel_ms']
print('groups $g r$r', round(d['value'] / 1e6, 3), 'M exp/s', {a: b['avg_ms'] for a, b in k.items()}, flush=True)"
  done
done
