#!/bin/bash
# diagnostic: per-phase cycle accounting of k_select (GPU box).  Builds a separate library with
# -DYK_SEL_TIMING into /tmp and runs tools/diag_select.py against it.
cd "$(dirname "$0")/.." || exit 2
set -e
bash tools/stage_hooks.sh
mkdir -p /tmp/yk_diag
for f in yk_env yk_net yk_engine yk_train yk_train_amp yk_replay; do
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -ffp-contract=off -DYK_SEL_TIMING $YK_EXTRA \
     -Iinclude -I/tmp/yk_hooks/csrc -c /tmp/yk_hooks/csrc/$f.hip -o /tmp/yk_diag/$f.o
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o /tmp/yk_diag/libyacht_hip.so /tmp/yk_diag/*.o -L/opt/rocm/lib -lrocblas -Wl,-rpath,/opt/rocm/lib
YK_LIB_PATH=/tmp/yk_diag/libyacht_hip.so timeout -k 5 200 python tools/diag_select.py "$@"
