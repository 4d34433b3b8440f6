#!/bin/bash
# diagnostic: forward timing with the policy-head weight loads confined to an L1-resident footprint
cd "$(dirname "$0")/.." || exit 2
set -e
bash tools/stage_hooks.sh
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -DYK_TIMING -DYK_DIAG_L1 -Iinclude -I/tmp/yk_hooks/csrc \
   tools/trunk_ablate.cpp /tmp/yk_hooks/csrc/yk_env.hip -o /tmp/abl_l1 -w
timeout -k 5 60 /tmp/abl_l1 ${1:-3480}
