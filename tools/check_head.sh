#!/bin/bash
# GPU box: the GPU test suite, a short bench of the in-tree library, and the same bench for
# each variant build given as NAME='-DFLAG=..' arguments (tools/variant_lib.sh).
# usage: tools/check_head.sh [NAME=FLAGS ...]
cd "$(dirname "$0")/.." || exit 2
B="python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-arena --no-train"
steps=('gputests:420:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread'
       "bench:300:$B > gpurun_out/bench_head.json")
for v in "$@"; do
  name="${v%%=*}"; flags="${v#*=}"
  steps+=("$name:300:bash tools/variant_lib.sh $name $flags && YK_LIB_PATH=/tmp/yk_$name/libyacht_hip.so $B > gpurun_out/bench_$name.json")
done
exec bash tools/gpu_steps.sh "${steps[@]}"
