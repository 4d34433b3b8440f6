"""Diagnostic (GPU box): where a residual block of the AMP train step goes - per-wave s_memtime
stamps of block 2 in k_amp_fwd and k_amp_bwd (the -DYK_AMP_TIMING library:
tools/variant_lib.sh amp -DYK_AMP_TIMING=1, then YK_LIB_PATH=/tmp/yk_amp/libyacht_hip.so).
Prints each phase's ticks (mean over the 32 tiles of a 512-row minibatch, per wave)."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nypc-yacht-auction_amd"))
from yacht_amd import kernels as K  # noqa: E402
from yacht_amd._lib import lib  # noqa: E402
from yacht_amd.nnet import YachtNNet  # noqa: E402
from yacht_amd.train import Trainer  # noqa: E402

B = 512
torch.manual_seed(0)
sd = YachtNNet(hidden=256, nblocks=6).state_dict()
rng = np.random.RandomState(0)
n = 8192
out, _ = K.init_board(0, np.arange(n), 0)
tg = torch.tensor(rng.randint(0, 202, n), dtype=torch.int32, device="cuda")
vv = torch.tensor(rng.rand(n) * 2 - 1, dtype=torch.float32, device="cuda")
tr = Trainer(sd, 256, 6, max_batch=B, dropout=float(os.environ.get("YK_DROPOUT", "0.3")), amp=True)
for i in range(12):
    tr.step(out, tg, vv, idx=torch.arange(i * B, (i + 1) * B, dtype=torch.int32, device="cuda"))
torch.cuda.synchronize()
L = lib()
L.yk_diag_amp_ts.argtypes = [C.c_void_p]
ts = np.zeros((2, 64, 8, 16), dtype=np.uint64)
assert L.yk_diag_amp_ts(ts.ctypes.data) == 0
T = B // 8  # the trunk workgroups (TRV = 8 rows each)
names = {0: ["GEMM + acc store", "T-layout store (waves 0-3)", "barrier 1", "row pass", "barrier 2"],
         1: ["row pass", "barrier", "column partials", "T-layout store", "row prefetch", "GEMM + acc store", "barrier"]}
for kk, kname in ((0, "k_amp_fwd"), (1, "k_amp_bwd")):
    print(f"{kname}, residual block 2 (ticks, mean over {T} tiles):")
    for half in ((0, 1) if kk == 0 else (1, 0)):
        s = ts[kk, :T, :, half * 8:half * 8 + 8].astype(np.int64)
        nph = len(names[kk])
        d = np.diff(s[:, :, :nph + 1], axis=2).mean(0)  # [wave][phase]
        tot = (s[:, :, nph] - s[:, :, 0]).mean(0)
        print(f"  half {half}: " + " | ".join(f"{nm} {d[:, k].mean():6.0f}" for k, nm in enumerate(names[kk])) +
              f" | total {tot.mean():6.0f}")
        for w in range(8):
            print(f"     wave {w}: " + " ".join(f"{d[w, k]:6.0f}" for k in range(nph)) + f"  = {tot[w]:6.0f}")
