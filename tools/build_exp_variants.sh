#!/bin/bash
# (container) prebuilt A/B variants of the policy softmax's exp: fastexp (__expf) and libexp (the
# library expf) in place of exp_acc -> tools/_variants/{fastexp,libexp}/libyacht_hip.so
cd "$(dirname "$0")/.." || exit 2
set -e
for v in fastexp:__expf libexp:expf; do
  name=${v%%:*}; fn=${v#*:}
  rm -rf /tmp/yk_src_$name /tmp/yk_$name; mkdir -p /tmp/yk_src_$name /tmp/yk_$name tools/_variants/$name
  cp -r nypc-yacht-auction_amd/csrc /tmp/yk_src_$name/
  sed -i "s/exp_acc(\([a-z]\)/$fn(\1/g" /tmp/yk_src_$name/csrc/yk_fwd.h /tmp/yk_src_$name/csrc/yk_engine.hip /tmp/yk_src_$name/csrc/yk_net.hip
  for f in yk_env yk_net yk_engine yk_train yk_train_amp yk_replay; do
    /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -ffp-contract=off -w -Iinclude -I/tmp/yk_src_$name/csrc \
      -c /tmp/yk_src_$name/csrc/$f.hip -o /tmp/yk_$name/$f.o &
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o tools/_variants/$name/libyacht_hip.so /tmp/yk_$name/yk_*.o -L/opt/rocm/lib -lrocblas -Wl,-rpath,/opt/rocm/lib
  echo "built $name: $(grep -c "$fn(" /tmp/yk_src_$name/csrc/yk_fwd.h) uses in yk_fwd.h"
done
