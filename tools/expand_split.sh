#!/bin/bash
# GPU box: k_expand_backup's time and HBM traffic split into its two halves - the expansion +
# backup, and the next simulation's descent - by running the bench configuration with
# YK_SPLIT_DESCENT=1 (the descent as its own k_select launch; identical trees): a kernel trace, then
# FETCH_SIZE and WRITE_SIZE passes over k_expand_backup and k_select.
# usage: tools/expand_split.sh TAG  -> gpurun_out/split_TAG/{trace,FETCH_SIZE,WRITE_SIZE}/, summary.json
cd "$(dirname "$0")/.." || exit 2
set -e
export TMPDIR=/tmp YK_SPLIT_DESCENT=1
tag=${1:-r05}
out=gpurun_out/split_$tag
mkdir -p $out
args="--steps 1 --warmup 1 --no-cpu-baseline --no-arena --no-coach --no-shape --no-f16 --no-train"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o split --output-format csv -- python3 bench.py $args > $out/bench_trace.json
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --kernel-include-regex 'k_expand_backup|k_select' --pmc $c -d $out/$c -o $c --output-format csv -- python3 bench.py $args --no-profile > $out/bench_$c.json
done
python3 tools/summarize_prof.py $out > $out/summary.json
cat $out/summary.json
