"""Diagnostic: 30 native train steps (batch 512, hidden 256 x 6) for rocprofv3 --kernel-trace --stats."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nypc-yacht-auction_amd"))
from yacht_amd import kernels as K  # noqa: E402
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
tr = Trainer(sd, 256, 6, max_batch=B, dropout=float(os.environ.get("YK_DROPOUT", "0.3")), amp=os.environ.get("YK_AMP", "0") == "1")
for i in range(30):
    idx = torch.arange((i * B) % (n - B), (i * B) % (n - B) + B, dtype=torch.int32, device="cuda")
    tr.step(out, tg, vv, idx=idx)
torch.cuda.synchronize()
print("done", tr.losses())
