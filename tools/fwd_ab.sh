#!/bin/bash
# diagnostic (GPU box): the timing harness (tools/trunk_ablate.cpp, per-phase stamps) for variant
# defines of yk_net.hip.  usage: tools/fwd_ab.sh ROWS "" "-DFOO" ...
cd "$(dirname "$0")/.." || exit 2
set -e
bash tools/stage_hooks.sh
rows=$1; shift
i=0
for v in "$@"; do
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -DYK_TIMING $v -Iinclude \
     -I/tmp/yk_hooks/csrc tools/trunk_ablate.cpp /tmp/yk_hooks/csrc/yk_env.hip -o /tmp/fab_$i -w &
  i=$((i+1))
done
wait
i=0
for v in "$@"; do echo "=== [$v]"; timeout -k 5 60 /tmp/fab_$i $rows; i=$((i+1)); done
