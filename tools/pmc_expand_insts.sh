#!/bin/bash
# diagnostic (GPU box): instruction mix of k_expand_backup and k_forward per wave (SQ counters)
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
set -e
out=gpurun_out/pmc_insts
mkdir -p $out
timeout -s KILL 120 rocprofv3 --kernel-include-regex 'k_expand_backup|k_forward' \
  --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  -d $out -o insts --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-arena --no-train --no-profile > $out/bench.json
python3 - <<'PY'
import csv, glob
from collections import defaultdict
f = glob.glob("gpurun_out/pmc_insts/**/*counter_collection.csv", recursive=True)[0]
acc = defaultdict(lambda: defaultdict(float)); n = defaultdict(int)
for r in csv.DictReader(open(f)):
    k = "forward" if "k_forward" in r["Kernel_Name"] else "expand"
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in acc.items():
    w = c["SQ_WAVES"]
    print(k, {name: round(v / w, 1) for name, v in c.items() if name != "SQ_WAVES"}, "waves", int(w))
PY
