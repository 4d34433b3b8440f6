"""Diagnostic: policy-head tile demand per forward workgroup with the rows in game order (the
engine's layout) and with the leaves regrouped by their valid-column class, from the row
descriptors a -DYK_TILESTAT library dumps (tools/diag_sort.sh)."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nypc-yacht-auction_amd"))
from yacht_amd._lib import lib  # noqa: E402
from yacht_amd.engine import SelfPlayEngine  # noqa: E402
from yacht_amd.nnet import YachtNNet, YkNet  # noqa: E402

NBID, NCOMB, NCAT, ASIZE = 202, 252, 12, 3226
E, sims = int(sys.argv[1]) if len(sys.argv) > 1 else 4096, 100
torch.manual_seed(0)
net = YkNet(YachtNNet(hidden=256, nblocks=6).state_dict(), 256, 6)
eng = SelfPlayEngine(E, sims, 1.5, 15, net=net, max_moves=64)
L = lib()
L.yk_diag_tiles.argtypes = [C.c_void_p]
L.yk_diag_vdump.argtypes = [C.c_void_p]
out = np.zeros(16, dtype=np.uint64)
L.yk_diag_tiles(out.ctypes.data)
eng.run(0, 0)
vd = np.zeros((64, 8192), dtype=np.uint32)
L.yk_diag_vdump(vd.ctypes.data)


def tile_set(v):
    m = v & 0xF
    if m == 0:
        return set()
    if m == 4:
        return set(range((ASIZE - 1) // 16 + 1))
    if m == 1:
        return set(range((NBID - 1) // 16 + 1))
    t = set()
    for c in range(NCAT):
        if not (v >> (4 + c)) & 1:
            a0 = NBID + NCOMB * c
            t |= set(range(a0 // 16, (a0 + (NCOMB - 1 if m == 2 else 0)) // 16 + 1))
    return t


cache = {}


def tiles(v):
    if v not in cache:
        cache[v] = tile_set(int(v))
    return cache[v]


def wg_unions(rows):
    u = []
    for i in range(0, len(rows), 16):
        s = set()
        for v in rows[i:i + 16]:
            s |= tiles(v)
        if any(v & 0xF for v in rows[i:i + 16]):
            u.append(len(s))
    return u


def sort_key(v):
    m = int(v) & 0xF
    # bids first, then score5, score10 by used mask, then the full rows
    order = {1: 0, 3: 1, 2: 2, 4: 3}[m]
    return (order, int(v) >> 4)


res = {"game": [], "sorted": []}
for k in range(64):
    rows = vd[k, :E]
    if not rows.any():
        continue
    u0 = wg_unions(list(rows))
    leaves = sorted([v for v in rows if v & 0xF], key=sort_key)
    u1 = wg_unions(leaves)
    res["game"].append((np.mean(u0), max(u0), len(u0)))
    res["sorted"].append((np.mean(u1), max(u1), len(u1)))
    kinds = np.bincount(rows & 0xF, minlength=5)
    print(f"sample {k:2d}: leaves {int((rows & 0xF != 0).sum())} (bid {kinds[1]}, s10 {kinds[2]}, s5 {kinds[3]}, all {kinds[4]})"
          f"  game order: wg {len(u0)} mean {np.mean(u0):.1f} max {max(u0)}  sorted: wg {len(u1)} mean {np.mean(u1):.1f} max {max(u1)}")
for k, v in res.items():
    a = np.array(v)
    print(f"{k:7s}: workgroups {a[:, 2].mean():.1f}, tiles per workgroup mean {a[:, 0].mean():.1f}, launch max {a[:, 1].mean():.1f} (of 202)")
