#!/bin/bash
# diagnostic: k_forward with and without the trunk tile rotation (GPU box)
cd "$(dirname "$0")/.." || exit 2
set -e
for v in "" "-DYK_NO_TRUNK_ROT"; do
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off $v -Iinclude -Inypc-yacht-auction_amd/csrc \
     tools/trunk_ablate.cpp nypc-yacht-auction_amd/csrc/yk_env.hip -o /tmp/abl_r$v -w
done
for n in 3480 4096; do
  for v in "" "-DYK_NO_TRUNK_ROT"; do echo "variant [$v]"; timeout -k 5 60 /tmp/abl_r$v $n; done
done
