#!/bin/bash
# diagnostic: HBM bytes and cache behaviour of k_expand_backup in the bench configuration
# (GPU box), one rocprofv3 --pmc pass per counter group.  -> gpurun_out/pmc_expand/
cd "$(dirname "$0")/.." || exit 2
set -e
export TMPDIR=/tmp
out=gpurun_out/pmc_expand
mkdir -p $out
args="--steps 1 --warmup 1 --no-cpu-baseline --no-arena --no-train --no-profile"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -k 10 400 rocprofv3 --kernel-include-regex "k_expand_backup|k_forward" --pmc $grp -d $out/g$i -o g$i \
     --output-format csv -- python3 bench.py $args > $out/bench_g$i.json
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/pmc_expand/g*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        acc[(r["Kernel_Name"][:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(acc.items()):
        print(f"{k:40s} {c:24s} mean {sum(v)/len(v):14.1f}  n={len(v)}")
PY
