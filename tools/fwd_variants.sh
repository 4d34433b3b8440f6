#!/bin/bash
# diagnostic: k_forward time for ring-depth variants (GPU box)
cd "$(dirname "$0")/.." || exit 2
set -e
for v in "-DYK_PW=2" "-DYK_PW=4"; do
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off $v -Iinclude -Inypc-yacht-auction_amd/csrc \
     tools/trunk_ablate.cpp nypc-yacht-auction_amd/csrc/yk_env.hip -o /tmp/abl_v -w
  echo "[$v]"; timeout -k 5 60 /tmp/abl_v 3480
done
