"""Diagnostic: where k_select's time goes (needs the -DYK_SEL_TIMING library, `tools/variant_lib.sh sel -DYK_SEL_TIMING`; tools/evidence.sh select)."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nypc-yacht-auction_amd"))
from yacht_amd._lib import lib  # noqa: E402
from yacht_amd.engine import SelfPlayEngine  # noqa: E402
from yacht_amd.nnet import YachtNNet, YkNet  # noqa: E402

E, sims = int(sys.argv[1]) if len(sys.argv) > 1 else 4096, 100
torch.manual_seed(0)
net = YkNet(YachtNNet(hidden=256, nblocks=6).state_dict(), 256, 6)
eng = SelfPlayEngine(E, sims, 1.5, 15, net=net, max_moves=64)
L = lib()
L.yk_diag_select.argtypes = [C.c_void_p, C.c_int]
out = np.zeros((E, 16), dtype=np.uint64)
eng.run(0, 0)
L.yk_diag_select(out.ctypes.data, E)  # discard the warm-up
eng.profile(True)
eng.run(1, 0)
L.yk_diag_select(out.ctypes.data, E)
kt = eng.kernel_times()
st = eng.stats()
lv = out[:, 4].sum()
tot = out[:, 3].astype(np.float64)
print(f"select kernel: {kt['select'][0] / kt['select'][1] * 1e3:.1f} us avg over {kt['select'][1]} launches")
print(f"levels per game-sim: {lv / (E * st['sims']):.2f}; valid entries scanned per level: {out[:, 5].sum() / lv:.0f}")
names = ["lookup (ended+hash+probe)", "UCB scan + argmax (full scans)", "step + canonical", "whole descent"]
per = tot.sum()
for k, nm in enumerate(names):
    c = out[:, k].astype(np.float64).sum()
    print(f"  {nm:28s} {c / (E * st['sims']):9.0f} cycles per game-sim  ({100 * c / per:5.1f}% of descent)")
print(f"  max descent per game-sim    {tot.max() / st['sims']:9.0f}")
rs = out[:, 13].astype(np.float64).sum()
print(f"  root incremental scan (root_scan) {rs / (E * st['sims']):9.0f} cycles per game-sim  "
      f"({100 * rs / per:5.1f}% of descent); entries read {out[:, 14].astype(np.float64).sum() / (E * st['sims']):.0f} "
      f"per game-sim vs {out[:, 5].astype(np.float64).sum() / (E * st['sims']):.0f} in full scans")
ex = out[:, 6].astype(np.float64).sum()
print(f"  expand + backup (fused kernel) {ex / (E * st['sims']):9.0f} cycles per game-sim")
for k, nm in ((8, "expand: logits load, max, sum-exp"), (9, "expand: mask + pairwise sum"),
              (10, "expand: P / slot write"), (12, "backup")):
    print(f"    {nm:34s} {out[:, k].astype(np.float64).sum() / (E * st['sims']):9.0f} cycles per game-sim")
print(f"expand_backup kernel: {kt['expand_backup_select'][0] / kt['expand_backup_select'][1] * 1e3:.1f} us avg")
print(f"forward kernel: {kt['forward'][0] / kt['forward'][1] * 1e3:.1f} us avg")
