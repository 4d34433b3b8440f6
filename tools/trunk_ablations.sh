#!/bin/bash
# diagnostic: per-phase stamps of k_forward (tools/trunk_ablate.cpp, full launches of 3480 rows)
# for the baseline and ablations: YK_ABL_W (no weight stream: every slice from 2 KB),
# YK_ABL_LN (the trunk's LayerNorms skipped), both.  GPU box.
cd "$(dirname "$0")/.." || exit 2
set -e
bash tools/stage_hooks.sh
i=0
for v in "" "-DYK_ABL_W" "-DYK_ABL_LN" "-DYK_ABL_W -DYK_ABL_LN"; do
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -DYK_TIMING $v -Iinclude \
     -I/tmp/yk_hooks/csrc tools/trunk_ablate.cpp /tmp/yk_hooks/csrc/yk_env.hip -o /tmp/tabl_$i -w &
  i=$((i+1))
done
wait
i=0
for v in "base" "no-stream" "no-LN" "no-stream+no-LN"; do
  echo "=== $v"; timeout -k 5 60 /tmp/tabl_$i 3480; i=$((i+1))
done
