"""Diagnostic: how a k_expand_backup launch's time relates to its games' own times (needs the
-DYK_XSPAN library, tools/diag_xspan.sh): 16 sampled launches of a 4096 x 100 batch, per game the
start / end-of-expand / end stamps, the expanded node's valid count, descent depth and the wave's
CU / XCD."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nypc-yacht-auction_amd"))
from yacht_amd._lib import lib  # noqa: E402
from yacht_amd.engine import SelfPlayEngine  # noqa: E402
from yacht_amd.nnet import YachtNNet, YkNet  # noqa: E402

E, sims = 4096, 100
torch.manual_seed(0)
net = YkNet(YachtNNet(hidden=256, nblocks=6).state_dict(), 256, 6)
eng = SelfPlayEngine(E, sims, 1.5, 15, net=net, max_moves=64)
L = lib()
L.yk_diag_xspan.argtypes = [C.c_void_p]
eng.run(0, 0)
out = np.zeros((16, E, 8), dtype=np.uint64)
L.yk_diag_xspan(out.ctypes.data)
rows = []
for k in range(16):
    o = out[k].astype(np.int64)
    ok = o[:, 2] > 0
    if not ok.any():
        continue
    o = o[ok]
    t0, t1, t2 = o[:, 0], o[:, 1], o[:, 2]
    dur = t2 - t0
    v = o[:, 3].astype(np.int64)
    exp = v != 0xFFFFFFFF
    hw = o[:, 5]
    xcc = hw >> 32
    # spans from s_memrealtime (100 MHz, device-wide), in shader ticks at the games' own clock rate
    r0, r2 = o[:, 6], o[:, 7]
    rate = dur.sum() / max((r2 - r0).sum(), 1)  # shader ticks per realtime tick
    spans = np.array([(r2[xcc == x].max() - r0[xcc == x].min()) * rate for x in np.unique(xcc)])
    starts = np.array([(r0[xcc == x].max() - r0[xcc == x].min()) * rate for x in np.unique(xcc)])
    spans = np.append(spans, (r2.max() - r0.min()) * rate)  # last: the whole launch
    slow = np.argsort(dur)[-40:]
    span = spans[-1]
    print(f"launch {k}: span {spans[-1]:.0f}, per XCD mean {spans[:-1].mean():.0f} ticks (start spread {starts.mean():.0f}); "
          f"game time mean {dur.mean():.0f} p50 {np.percentile(dur, 50):.0f} p90 {np.percentile(dur, 90):.0f} "
          f"p99 {np.percentile(dur, 99):.0f} max {dur.max()}")
    ve = v[exp] if exp.any() else np.zeros(1)
    print(f"   expansions {exp.sum()}, V of expanded: mean {ve.mean():.0f}; slowest 40 games: expanded "
          f"{exp[slow].sum()}, depth mean {o[slow, 4].mean():.2f} (all {o[:, 4].mean():.2f}); their expand part "
          f"{np.mean(t1[slow] - t0[slow]):.0f} descent part {np.mean(t2[slow] - t1[slow]):.0f} "
          f"(all {np.mean(t1 - t0):.0f} / {np.mean(t2 - t1):.0f})")
    cu_busy = spans[:-1]
    rows.append((span, dur.mean(), np.percentile(dur, 99), dur.max(), cu_busy.mean()))
r = np.array(rows, dtype=np.float64)
print(f"over {len(r)} launches: span {r[:, 0].mean():.0f} mean {r[:, 4].mean():.0f}; game time mean "
      f"{r[:, 1].mean():.0f}, p99 {r[:, 2].mean():.0f}, max {r[:, 3].mean():.0f} ticks")
