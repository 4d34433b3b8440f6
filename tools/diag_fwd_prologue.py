"""Diagnostic: k_forward's phases inside the engine (the -DYK_TIMING library: tools/evidence.sh fwdts).

Runs self-play batches at the bench shape; each workgroup of every forward launch adds its wave-0
stamps (tools/diag_sources.py: slots 1-15 the phases, 32-40 the prologue, the tile list and the v_head.2 chunk) relative to its start
into a device accumulator, read after the batch.  Ticks are s_memtime counts."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nypc-yacht-auction_amd"))
from yacht_amd._lib import lib  # noqa: E402
from yacht_amd.engine import SelfPlayEngine  # noqa: E402
from yacht_amd.nnet import YachtNNet, YkNet  # noqa: E402

E = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
sims = int(sys.argv[2]) if len(sys.argv) > 2 else 100
S = 48  # TS_STRIDE
nwg = (E + 15) // 16
torch.manual_seed(0)
net = YkNet(YachtNNet(hidden=256, nblocks=6).state_dict(), 256, 6)
eng = SelfPlayEngine(E, sims, 1.5, 15, net=net, max_moves=64)
L = lib()
L.yk_diag_fwd_ts.argtypes = [C.c_void_p, C.c_int]
L.yk_diag_fwd_tacc.argtypes = [C.c_void_p, C.c_int]
seq = [("vstat->LDS", 0, 32), ("weights issued (w0)", 32, 38), ("features", 38, 33), ("input barrier", 33, 34),
       ("tile masks", 34, 1), ("input GEMM", 1, 35), ("input T barrier", 35, 36),
       ("input row pass", 36, 2), ("blk0", 2, 3), ("blk1", 3, 4), ("blk2", 4, 5), ("blk3", 5, 6), ("blk4", 6, 7),
       ("blk5", 7, 8), ("heads LN", 8, 9), ("v_head.2 chunk", 9, 40), ("  full / list reads", 9, 43), ("  chunk 0 tiles", 43, 41),
       ("  chunk 0 ring issue", 41, 42), ("  v_head.2 MFMAs", 42, 40), ("policy chunks", 40, 14), ("end", 14, 15), ("  value head (waves 0-3)", 14, 46), ("  stat merges", 46, 44),
       ("  end barrier", 44, 45), ("  SS stores", 45, 23), ("  mlse", 23, 15),
       ("(blk0: wave 0's tile-list chunk)", 39, 37)]
eng.run(0, 0)  # warm-up
torch.cuda.synchronize()
rows = []
for rep in range(2):
    L.yk_diag_fwd_tacc(None, 1)
    eng.run(1 + rep, 0)
    torch.cuda.synchronize()
    a = np.zeros(S, dtype=np.uint64)
    if L.yk_diag_fwd_tacc(a.ctypes.data, 0):
        raise SystemExit("yk_diag_fwd_tacc failed")
    n = float(a[S - 1])
    m = a.astype(np.float64) / n  # mean ticks of slot i after the workgroup's start
    m[0] = 0.0
    rows.append((n, [m[b] - m[a_] for _, a_, b in seq], m[15], [m[24 + w] - m[9] for w in range(8)]))
print(f"k_forward phases, mean ticks over every workgroup of every launch of a batch ({E} games x {sims} sims)")
print("  " + " ".join(f"{'batch ' + str(i):>10s}" for i in range(len(rows))) + "   phase")
for j, (k, _, _) in enumerate(seq):
    print("  " + " ".join(f"{r[1][j]:10.0f}" for r in rows) + f"   {k}")
print("  " + " ".join(f"{r[2]:10.0f}" for r in rows) + "   total")
print("  " + " ".join(f"{r[0]:10.0f}" for r in rows) + "   workgroup-launches")
for w in range(8):
    print("  " + " ".join(f"{r[3][w]:10.0f}" for r in rows) + f"   wave {w}: end of its policy chunks after the heads' LayerNorm")
