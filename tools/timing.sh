#!/bin/bash
# diagnostic: per-phase s_memtime profile of k_forward (GPU box)
cd "$(dirname "$0")/.." || exit 2
set -e
bash tools/stage_hooks.sh
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -DYK_TIMING -Iinclude -I/tmp/yk_hooks/csrc \
   tools/trunk_ablate.cpp /tmp/yk_hooks/csrc/yk_env.hip -o /tmp/abl_t -w
for v in ${@:-3480}; do timeout -k 5 60 /tmp/abl_t $v; done
