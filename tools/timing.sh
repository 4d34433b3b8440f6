#!/bin/bash
# diagnostic: per-phase s_memtime profile of k_forward (GPU box)
cd "$(dirname "$0")/.." || exit 2
set -e
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -DYK_TIMING -Iinclude -Inypc-yacht-auction_amd/csrc \
   tools/trunk_ablate.cpp nypc-yacht-auction_amd/csrc/yk_env.hip -o /tmp/abl_t -w
for v in ${@:-3480}; do timeout -k 5 60 /tmp/abl_t $v; done
