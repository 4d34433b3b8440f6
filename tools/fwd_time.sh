#!/bin/bash
# diagnostic: k_forward time on synthetic rows (GPU box)
cd "$(dirname "$0")/.." || exit 2
set -e
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off $YK_EXTRA -Iinclude -Inypc-yacht-auction_amd/csrc \
   tools/trunk_ablate.cpp nypc-yacht-auction_amd/csrc/yk_env.hip -o /tmp/abl_f -w
for v in ${@:-3480 4096}; do timeout -k 5 60 /tmp/abl_f $v; done
