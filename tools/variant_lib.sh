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
# the diagnostic hooks (stamps, yk_diag_* readers) are not in the production sources: with a
# -DYK_* switch, build from a copy with them inserted (tools/diag_sources.py)
case " $* " in
  *" -DYK_"*)
    [ "$src" = nypc-yacht-auction_amd/csrc ] || { echo "hooks need the in-tree sources" >&2; exit 2; }
    python3 tools/diag_sources.py $out/stage > /dev/null
    src=$out/stage/csrc ;;
esac
rm -f $out/*.o $out/libyacht_hip.so  # (a failed compile must not link a stale object)
pids=()
for f in yk_env yk_net yk_engine yk_train yk_train_amp yk_replay; do
  [ -f $src/$f.hip ] || continue
  fc=off; [ $f = yk_train_amp ] && fc=fast  # (as the Makefile)
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -ffp-contract=$fc -w "$@" \
     -Iinclude -I$src -c $src/$f.hip -o $out/$f.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p || { echo "variant $name: compile failed" >&2; exit 1; }; done
libs=""  # (baselines staged from before round 5 still call rocBLAS in the f32 trainer)
grep -q rocblas $src/yk_train.hip && libs="-L/opt/rocm/lib -lrocblas -Wl,-rpath,/opt/rocm/lib"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $out/libyacht_hip.so $out/yk_*.o $libs
echo "built $out/libyacht_hip.so"
