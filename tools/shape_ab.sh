#!/bin/bash
# diagnostic (GPU box): bench at other per-GPU shapes and group counts.  usage: tools/shape_ab.sh "ENVS:SIMS:GROUPS" ...
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "$@"; do
  IFS=: read -r e s g <<< "$spec"
  timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-arena --no-train --envs "$e" --sims "$s" \
    --groups "$g" > "gpurun_out/shape_${e}_${s}_${g}.json" 2> "gpurun_out/shape_${e}_${s}_${g}.err" || exit $?
  python3 -c "
import json; d = json.load(open('gpurun_out/shape_${e}_${s}_${g}.json')); k = d['kernel_ms']
print('envs $e sims $s groups $g:', round(d['value'] / 1e6, 3), 'M exp/s', round(d['ms_per_step'], 1), 'ms/step',
      {a: b['avg_ms'] for a, b in k.items()}, d['capacity_use'], flush=True)"
done
