#!/bin/bash
# diagnostic: build and time the trunk ablation variants (GPU box)
cd "$(dirname "$0")/.." || exit 2
set -e
for v in 0 1 2 3; do
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -DYK_ABL=$v -Iinclude -Inypc-yacht-auction_amd/csrc \
     tools/trunk_ablate.cpp nypc-yacht-auction_amd/csrc/yk_env.hip -o /tmp/abl_$v
done
for v in 0 1 2 3; do timeout -k 5 60 /tmp/abl_$v ${1:-3480}; done
