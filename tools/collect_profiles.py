"""Copy a GPU run's evidence from gpurun_out/ into profiles/ (tracked) under one tag.
usage: python tools/collect_profiles.py TAG [ENVS SIMS]
  gpurun_out/bench_TAG.json            -> profiles/TAG_bench.json (the bench line)
  gpurun_out/prof_TAG/trace/*stats.csv -> profiles/TAG_kernel_stats.csv (rocprofv3 --kernel-trace --stats)
  gpurun_out/prof_TAG/summary.json     -> profiles/TAG_prof_summary.json and, per kernel,
      profiles/TAG_forward_traffic.json / TAG_expand_traffic.json (HBM bytes per launch) and
      profiles/TAG_forward_mfma.json (MFMA busy fraction), which bench.py reads for its line
  gpurun_out/dist2_TAG.json            -> profiles/TAG_dist2_gloo_rehearsal.json
"""
import glob
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
envs, sims = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (4096, 100)
src, dst = os.path.join(REPO, "gpurun_out"), os.path.join(REPO, "profiles")
cfg = {"envs": envs, "sims": sims, "hidden": 256, "nblocks": 6}
cmd = (f"tools/profile_bench.sh {tag}: rocprofv3 --kernel-include-regex 'k_forward|k_expand_backup' --pmc "
       "FETCH_SIZE|WRITE_SIZE (separate passes) -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline "
       "--no-arena --no-coach --no-shape --no-f16 --no-train --no-profile")


def copy(a, b):
    if os.path.exists(a):
        shutil.copy(a, b)
        print("wrote", os.path.relpath(b, REPO))


copy(os.path.join(src, f"bench_{tag}.json"), os.path.join(dst, f"{tag}_bench.json"))
copy(os.path.join(src, f"dist2_{tag}.json"), os.path.join(dst, f"{tag}_dist2_gloo_rehearsal.json"))
st = glob.glob(os.path.join(src, f"prof_{tag}", "trace", "**", "*kernel_stats.csv"), recursive=True)
if st:
    copy(st[0], os.path.join(dst, f"{tag}_kernel_stats.csv"))
summ = os.path.join(src, f"prof_{tag}", "summary.json")
if os.path.exists(summ):
    copy(summ, os.path.join(dst, f"{tag}_prof_summary.json"))
    s = json.load(open(summ))
    stats = s.get("kernel_stats", {})
    for kname, v in s.get("pmc", {}).items():
        kind = "forward" if "k_forward" in kname else "expand" if "k_expand_backup" in kname else None
        if kind is None:
            continue
        avg = next((x["avg_us"] for n, x in stats.items() if n == kname), None)
        short = "k_forward<256, 2>" if kind == "forward" else "k_expand_backup"
        if "hbm_bytes_per_launch" in v:
            out = {"kernel": short, "config": cfg, "kernel_src_sha16": s.get("kernel_src_sha16"), "command": cmd,
                   "launches": v["launches"],
                   "FETCH_SIZE_KiB_mean": v["FETCH_SIZE_KiB_mean"], "WRITE_SIZE_KiB_mean": v["WRITE_SIZE_KiB_mean"],
                   "correction": "FETCH_SIZE x2 on gfx950 (MI355X_MICROARCH.md, HBM); WRITE_SIZE as read",
                   "hbm_bytes_per_launch": v["hbm_bytes_per_launch"], "kernel_trace_avg_us": avg}
            p = os.path.join(dst, f"{tag}_{kind}_traffic.json")
            json.dump(out, open(p, "w"), indent=1)
            print("wrote", os.path.relpath(p, REPO))
        if kind == "forward" and "mfma_busy_frac" in v:
            out = {"kernel": short, "config": cfg, "kernel_src_sha16": s.get("kernel_src_sha16"),
                   "command": f"tools/profile_bench.sh {tag}: rocprofv3 --kernel-include-regex k_forward --pmc "
                              "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -- python3 "
                              "bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-arena --no-coach --no-shape "
                              "--no-f16 --no-train --no-profile",
                   "counters_mean_per_launch": {c: v[c + "_mean"] for c in ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES",
                                                                          "SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE")},
                   "busy_frac": v["mfma_busy_frac"],
                   "formula": "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 256 CUs x 4 SIMDs): the share of "
                              "SIMD cycles the matrix pipes were busy while the kernel ran (GRBM_GUI_ACTIVE reads a few % "
                              "high on ~80 us dispatches, MI355X_MICROARCH.md 'DVFS', so this is a slight underestimate)",
                   "kernel_trace_avg_us": avg}
            p = os.path.join(dst, f"{tag}_forward_mfma.json")
            json.dump(out, open(p, "w"), indent=1)
            print("wrote", os.path.relpath(p, REPO))
