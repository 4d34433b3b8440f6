"""Summarise a tools/profile_bench.sh directory: per-kernel average duration (kernel trace) and
the k_forward / k_expand_backup HBM bytes per launch from the PMC passes (FETCH_SIZE doubled on gfx950 and
WRITE_SIZE as read; both counters in KiB, MI355X_MICROARCH.md 'HBM')."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

d = sys.argv[1]
out = {}
_sha = os.path.join(d, "kernel_src_sha16.txt")
if os.path.exists(_sha):
    out["kernel_src_sha16"] = open(_sha).read().strip()
st = glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True)
if st:
    rows = list(csv.DictReader(open(st[0])))
    out["kernel_stats"] = {r["Name"]: {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                                       "total_ms": float(r["TotalDurationNs"]) / 1e6} for r in rows}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(os.path.join(d, c, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        continue
    vals = defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        if r["Counter_Name"] == c:
            vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    for k, v in vals.items():
        out.setdefault("pmc", {}).setdefault(k, {})[c + "_KiB_mean"] = sum(v) / len(v)
        out["pmc"][k]["launches"] = len(v)
f = glob.glob(os.path.join(d, "MFMA", "**", "*counter_collection.csv"), recursive=True)
if f:
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(f[0])):
        acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        e = out.setdefault("pmc", {}).setdefault(k, {})
        e.update({c + "_mean": x for c, x in m.items()})
        if m.get("GRBM_GUI_ACTIVE"):
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS); 256 CUs x 4 SIMDs
            e["mfma_busy_frac"] = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (m["GRBM_GUI_ACTIVE"] / 8 * 1024)
for k, v in out.get("pmc", {}).items():
    if "FETCH_SIZE_KiB_mean" in v and "WRITE_SIZE_KiB_mean" in v:
        v["hbm_bytes_per_launch"] = 1024 * (2 * v["FETCH_SIZE_KiB_mean"] + v["WRITE_SIZE_KiB_mean"])
print(json.dumps(out, indent=1))
