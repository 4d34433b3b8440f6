#!/bin/bash
# diagnostic: k_forward time (tools/trunk_ablate.cpp harness, explicit features = full launches)
# for variant defines (GPU box).  usage: tools/fwd_variants.sh "" "-DFOO" ...
cd "$(dirname "$0")/.." || exit 2
set -e
i=0
for v in "$@"; do
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off $v -Iinclude -Inypc-yacht-auction_amd/csrc \
     tools/trunk_ablate.cpp nypc-yacht-auction_amd/csrc/yk_env.hip -o /tmp/abl_v$i -w &
  i=$((i+1))
done
wait
for r in 1 2; do
  i=0
  for v in "$@"; do echo "[$v] $(timeout -k 5 60 /tmp/abl_v$i 3480)"; i=$((i+1)); done
done
