#!/bin/bash
# wave-state and instruction-cache counters of the engine's kernels (GPU box), one --pmc pass each
# (separate passes: a pass over the block's slot count hangs).  -> gpurun_out/pmc_TAG/
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
tag=${1:-x}
out=gpurun_out/pmc_$tag
mkdir -p $out
args="--steps 1 --warmup 1 --no-cpu-baseline --no-arena --no-coach --no-shape --no-f16 --no-train --no-steady --no-profile"
rocprofv3 -L > $out/avail.txt 2>&1 || true
grep -oE "SQC?_[A-Z0-9_]+" $out/avail.txt | sort -u > $out/names.txt || true
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES" \
           "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH"; do
  ok=1
  for c in $set; do grep -qx "$c" $out/names.txt || { echo "no counter $c"; ok=0; }; done
  [ $ok = 1 ] || continue
  i=$((i + 1))
  timeout -s KILL 240 rocprofv3 --kernel-include-regex 'k_expand_backup|k_select|k_forward' --pmc $set \
    -d $out/p$i -o p$i --output-format csv -- python3 bench.py $args > $out/bench_p$i.json || exit $?
done
python3 tools/pmc_kernels.py $out/p* | tee $out/summary.txt
# keep the summaries only (gpurun copies back at most 64 MiB)
rm -rf $out/p*/ 2>/dev/null || true
