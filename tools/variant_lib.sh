#!/bin/bash
# diagnostic: builds a variant of libyacht_hip.so with extra defines into /tmp/yk_NAME/
# (GPU box or here).  usage: tools/variant_lib.sh NAME "-DFOO=1 ..."; then
# YK_LIB_PATH=/tmp/yk_NAME/libyacht_hip.so python bench.py ...
# A NAME starting with "base" builds the sources staged under ab_base/csrc (an A/B baseline).
cd "$(dirname "$0")/.." || exit 2
set -e
name=$1; shift
src=nypc-yacht-auction_amd/csrc
case $name in base*) src=ab_base/csrc ;; esac
out=/tmp/yk_$name
mkdir -p $out
# the diagnostic hooks (stamps, ablation switches, yk_diag_* readers) live in tools/diag_hooks.patch,
# not in the production sources: stage a copy with the hooks applied (a no-op without their defines)
rm -rf $out/stage && mkdir -p $out/stage && cp -r $src $out/stage/csrc
patch -s -d $out/stage -p2 < tools/diag_hooks.patch
src=$out/stage/csrc
for f in yk_env yk_net yk_engine yk_train yk_train_amp yk_replay; do
  [ -f $src/$f.hip ] || continue
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -ffp-contract=off -w "$@" \
     -Iinclude -I$src -c $src/$f.hip -o $out/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $out/libyacht_hip.so $out/yk_*.o -L/opt/rocm/lib -lrocblas -Wl,-rpath,/opt/rocm/lib
echo "built $out/libyacht_hip.so"
