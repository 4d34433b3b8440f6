#!/bin/bash
# diagnostic (GPU box): interleaved A/B bench of the in-tree library ("head"), the staged
# baseline sources ("base", ab_base/csrc) and variants, R rounds each, so box-to-box drift
# cancels.  A variant is NAME=-DFLAGS (a build, tools/variant_lib.sh) or NAME=--bench-args
# (the head library, or the base one when NAME starts with "base", with extra bench.py args).
# usage: tools/ab_bench.sh ROUNDS [NAME=FLAGS ...]
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${1:-2}; shift
names=(head); declare -A LIB ARGS
LIB[head]=""; ARGS[head]=""
# a variant prebuilt in the container (tools/_variants/NAME/libyacht_hip.so, git-ignored) is used as is
pre() { [ -f tools/_variants/$1/libyacht_hip.so ] && echo tools/_variants/$1/libyacht_hip.so; }
if [ -d ab_base/csrc ] || [ -n "$(pre base)" ]; then
  if [ -n "$(pre base)" ]; then LIB[base]=$(pre base); else bash tools/variant_lib.sh base > /dev/null || exit 3; LIB[base]=/tmp/yk_base/libyacht_hip.so; fi
  names+=(base); ARGS[base]=""
fi
for v in "$@"; do
  n="${v%%=*}"; f="${v#*=}"
  names+=("$n")
  case "$f" in
    --*) ARGS[$n]="$f"; LIB[$n]=""; case $n in base*) LIB[$n]=${LIB[base]} ;; esac ;;
    *) if [ -n "$(pre $n)" ]; then LIB[$n]=$(pre $n); else bash tools/variant_lib.sh "$n" $f > /dev/null || exit 3; LIB[$n]=/tmp/yk_$n/libyacht_hip.so; fi
       ARGS[$n]="" ;;
  esac
done
B="python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-arena --no-train --no-coach --no-shape"
for r in $(seq 1 "$R"); do
  for n in "${names[@]}"; do
    YK_LIB_PATH=${LIB[$n]} timeout -k 10 120 $B ${ARGS[$n]} > gpurun_out/ab_${n}_$r.json 2> gpurun_out/ab_${n}_$r.err || exit $?
    python3 - "$n" "$r" <<'EOF'
import json, sys
n, r = sys.argv[1], sys.argv[2]
d = json.load(open(f"gpurun_out/ab_{n}_{r}.json"))
k = {a: round(b["avg_ms"] * 1000, 2) for a, b in d.get("kernel_ms", {}).items()}
c = d.get("capacity_use", {})
print(f"{n:8s} r{r} {d['value'] / 1e6:7.3f}M exp/s  fwd {k.get('forward')}  exp {k.get('expand_backup_select')}  "
      f"sel {k.get('select')}  rs {k.get('root_sort_select')}  mb {k.get('move_begin')}  me {k.get('move_end')}  arena {c.get('max_arena')}/"
      f"{c.get('arena_cap')}" + (f"  f16 {d['predict_f16']['expansions_per_s'] / 1e6:.3f}M fwd16 "
      f"{round(d['predict_f16'].get('kernel_avg_ms', {}).get('forward', 0) * 1000, 2)}" if 'predict_f16' in d else ""), flush=True)
EOF
  done
done
