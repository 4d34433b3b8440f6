"""Per-kernel average durations of rocprofv3 --stats runs side by side:
python3 tools/kstats.py DIR [DIR ...] (each DIR a -d directory holding *kernel_stats.csv)."""
import csv
import glob
import os
import sys

cols = []
for d in sys.argv[1:]:
    f = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    rows = {}
    for r in csv.DictReader(open(f[0])) if f else []:
        n = r["Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:34]
        rows[n] = (int(r["Calls"]), float(r["AverageNs"]) / 1000)
    cols.append(rows)
names = sorted({n for c in cols for n in c}, key=lambda n: -max(c.get(n, (0, 0))[1] * c.get(n, (0, 0))[0] for c in cols))
print(f"{'kernel':36s}" + "".join(f"{os.path.basename(d.rstrip('/'))[:14]:>16s}" for d in sys.argv[1:]))
for n in names:
    print(f"{n:36s}" + "".join(f"{c[n][1]:10.2f} x{c[n][0]:<4d}" if n in c else f"{'-':>16s}" for c in cols))
