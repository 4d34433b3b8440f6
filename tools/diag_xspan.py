"""Diagnostic: how a k_expand_backup launch's time relates to its games' own times (needs the
-DYK_XSPAN library, `tools/variant_lib.sh xspan -DYK_XSPAN`; tools/evidence.sh xspan): 16 sampled
launches of a 4096 x 100 batch, per game the start / end-of-expand / end stamps, the expanded
node's valid count, descent depth and the wave's CU / XCD.

Co-residency (round 6): every game is one wave and all 4096 are resident at once (16 per CU).  Per
launch, a game's own work is predicted from its expand (valid count V of the expanded node, 0 when
none) and descent depth by least squares on the game times; each CU's load is the sum of its games'
predicted work.  Printed: the correlation of a game's time with its CU's load beyond its own work
(the interference), and of each CU's finish (realtime, device-wide) with its load - high values
would mean the launch tail is co-residency load that dealing games to CUs by predicted work could
even out."""
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
rows, corr = [], []
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
    # ---- co-residency: the CU of each game (XCC, SE / SH / CU fields of HW_ID bits 8-15)
    cu = (xcc << 8) | ((hw >> 8) & 0xFF)
    X = np.stack([np.ones(len(o)), np.where(exp, v, 0).astype(np.float64), exp.astype(np.float64),
                  o[:, 4].astype(np.float64)], 1)
    coef, *_ = np.linalg.lstsq(X, dur.astype(np.float64), rcond=None)
    own = X @ coef
    ucu, inv = np.unique(cu, return_inverse=True)
    load = np.bincount(inv, weights=own)
    ngames = np.bincount(inv)
    others = load[inv] - own  # the co-resident games' predicted work
    resid = dur - own
    r_int = np.corrcoef(resid, others)[0, 1]
    r_own = np.corrcoef(dur, own)[0, 1]
    fin = np.zeros(len(ucu))
    np.maximum.at(fin, inv, (r2 - r0.min()).astype(np.float64))
    r_fin = np.corrcoef(fin, load)[0, 1]
    lo, hi = np.percentile(load, [10, 90])
    print(f"   co-residency: {len(ucu)} CUs, {ngames.mean():.1f} games each (min {ngames.min()}, max {ngames.max()}); "
          f"own-work fit r {r_own:.2f} (ticks = {coef[0]:.0f} + {coef[1]:.1f} V + {coef[2]:.0f} expanded + "
          f"{coef[3]:.0f} depth); corr(time - own, co-resident work) {r_int:.2f}; corr(CU finish, CU load) "
          f"{r_fin:.2f}; CU load p10 {lo:.0f} p90 {hi:.0f} max {load.max():.0f}; CU finish p10 "
          f"{np.percentile(fin, 10) * rate:.0f} p90 {np.percentile(fin, 90) * rate:.0f} max {fin.max() * rate:.0f} ticks")
    corr.append((r_own, r_int, r_fin, load.max() / load.mean(), fin.max() / fin.mean()))
r = np.array(rows, dtype=np.float64)
c = np.array(corr)
print(f"co-residency over {len(c)} launches: corr(time, own work) {c[:, 0].mean():.2f}, corr(time - own, "
      f"co-resident work) {c[:, 1].mean():.2f}, corr(CU finish, CU load) {c[:, 2].mean():.2f}; max / mean CU load "
      f"{c[:, 3].mean():.2f}, max / mean CU finish {c[:, 4].mean():.2f}")
print(f"over {len(r)} launches: span {r[:, 0].mean():.0f} mean {r[:, 4].mean():.0f}; game time mean "
      f"{r[:, 1].mean():.0f}, p99 {r[:, 2].mean():.0f}, max {r[:, 3].mean():.0f} ticks")
