"""Per-kernel averages of rocprofv3 --pmc passes: python3 tools/pmc_kernels.py DIR [DIR ...]
(each DIR one pass's -d directory).  Prints kernel, dispatches and the mean of every counter."""
import collections
import csv
import glob
import os
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:48]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(acc.items()):
    n = max(len(v) for v in cs.values())
    print(f"{k}  ({n} dispatches)")
    for c, v in sorted(cs.items()):
        print(f"    {c:32s} {sum(v) / len(v):16.1f}")
