"""Diagnostic: how many policy-head tiles a forward workgroup would need if it computed only the
union of its rows' valid columns (needs the -DYK_TILESTAT library, tools/diag_tiles.sh)."""
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
L.yk_diag_tiles.argtypes = [C.c_void_p]
out = np.zeros(16, dtype=np.uint64)
L.yk_diag_tiles(out.ctypes.data)
eng.run(0, 0)
L.yk_diag_tiles(out.ctypes.data)
wg, tiles, rows, bid, lmax, _, launches = (int(x) for x in out[:7])
print(f"forward workgroups with a leaf: {wg}; rows with stored logits per workgroup {rows / wg:.2f}")
print(f"policy tiles needed per workgroup: {tiles / wg:.1f} of 204 ({100 * tiles / wg / 204:.1f}%); "
      f"bid-only workgroups {100 * bid / wg:.1f}%")
print(f"per launch: max tiles over its workgroups, averaged over {launches} launches: {lmax / launches:.1f}")
print("histogram of tiles per workgroup (bins of 32):", [int(x) for x in out[8:15]])
