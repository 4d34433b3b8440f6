"""Diagnostic (GPU box): time of the native train step (NNetWrapper.train's minibatch, 512 x YachtNNet
256 x 6, dropout 0.3) with HIP events over 100 steps after 10 warm-up steps."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nypc-yacht-auction_amd"))
from yacht_amd import kernels as K  # noqa: E402
from yacht_amd.nnet import YachtNNet  # noqa: E402
from yacht_amd.train import Trainer  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
torch.manual_seed(0)
sd = YachtNNet(hidden=256, nblocks=6).state_dict()
rng = np.random.RandomState(0)
n = 16384
out, _ = K.init_board(0, np.arange(n), 0)
tg = torch.tensor(rng.randint(0, 202, n), dtype=torch.int32, device="cuda")
vv = torch.tensor(rng.rand(n) * 2 - 1, dtype=torch.float32, device="cuda")
tr = Trainer(sd, 256, 6, max_batch=B, dropout=float(os.environ.get("YK_DROPOUT", "0.3")), amp=os.environ.get("YK_AMP", "0") == "1")
idx = [torch.arange(j, j + B, dtype=torch.int32, device="cuda") for j in range(0, n - B, B)]
for i in range(10):
    tr.step(out, tg, vv, idx=idx[i % len(idx)])
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
e0.record()
for i in range(100):
    tr.step(out, tg, vv, idx=idx[i % len(idx)])
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 100
print(f"batch {B}: {ms * 1000:.1f} us per train step, {B / ms * 1000:.0f} examples/s, losses {tr.losses()}")
