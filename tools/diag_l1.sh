#!/bin/bash
# diagnostic: forward timing with the policy-head weight loads confined to an L1-resident footprint
cd "$(dirname "$0")/.." || exit 2
set -e
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -DYK_TIMING -DYK_DIAG_L1 -Iinclude -Inypc-yacht-auction_amd/csrc \
   tools/trunk_ablate.cpp nypc-yacht-auction_amd/csrc/yk_env.hip -o /tmp/abl_l1 -w
timeout -k 5 60 /tmp/abl_l1 ${1:-3480}
