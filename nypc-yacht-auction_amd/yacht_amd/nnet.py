"""YachtNNet weights (torch) + NNetWrapper.predict / train on the MI355X.

``YachtNNet`` repeats the reference architecture (yacht/pytorch/YachtNNet.py:8-70) so its
``state_dict`` names and initialisation match; torch only holds the weights.  Inference
(``NNetWrapper.predict``, NNet.py:177-195) runs through ``yk_net_predict`` - featurize,
13 dense layers, both heads and exp(log_softmax) on the GPU; ``NNetWrapper.train``
(NNet.py:118-174) through the native trainer (train.py, yk_trainer_*).
"""
from __future__ import annotations

import ctypes as C
import os
from collections import OrderedDict

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import kernels as K
from ._lib import call, lib, ptr, stream_ptr
from .state import ACTION_SIZE, pack
from .utils import dotdict

DEFAULT_ARGS = dotdict(dict(lr=2e-3, weight_decay=1e-4, epochs=15, batch_size=512, vloss_weight=1.5,
                            cuda=True, hidden=256, nblocks=6, dropout=0.3))  # main.py:31-42


class ResidualBlock(nn.Module):  # YachtNNet.py:8-21
    def __init__(self, dim, dropout=0.2):
        super().__init__()
        self.fc1 = nn.Linear(dim, dim)
        self.ln1 = nn.LayerNorm(dim)
        self.fc2 = nn.Linear(dim, dim)
        self.ln2 = nn.LayerNorm(dim)
        self.dropout = nn.Dropout(dropout)

    def forward(self, x):
        h = self.ln1(F.silu(self.fc1(x)))
        h = self.dropout(h)
        h = self.ln2(F.silu(self.fc2(h)))
        return x + h


class YachtNNet(nn.Module):  # YachtNNet.py:24-70
    def __init__(self, input_len=59, action_size=ACTION_SIZE, hidden=256, nblocks=6, dropout=0.3,
                 kaiming_init=True):
        """kaiming_init=False keeps torch's default Linear init, as the submission bot's copy of
        the class does (agent.py:30-67)."""
        super().__init__()
        self.input_len, self.action_size = input_len, action_size
        self.inp = nn.Sequential(nn.Linear(input_len, hidden), nn.LayerNorm(hidden), nn.SiLU(), nn.Dropout(dropout))
        self.blocks = nn.ModuleList([ResidualBlock(hidden, dropout) for _ in range(nblocks)])
        self.pi_head = nn.Sequential(nn.LayerNorm(hidden), nn.SiLU(), nn.Linear(hidden, action_size))
        self.v_head = nn.Sequential(nn.LayerNorm(hidden), nn.SiLU(), nn.Linear(hidden, 128), nn.SiLU(),
                                    nn.Linear(128, 1))
        for m in self.modules() if kaiming_init else ():
            if isinstance(m, nn.Linear):
                nn.init.kaiming_uniform_(m.weight, nonlinearity="relu")
                nn.init.zeros_(m.bias)

    def forward(self, x):
        if x.ndim == 3:
            x = x.squeeze(1)
        h = self.inp(x)
        for blk in self.blocks:
            h = blk(h)
        return self.pi_head(h), torch.tanh(self.v_head(h))


PRECISIONS = {"f32": 0, "f16": 1}  # YK_PREDICT_F32 / YK_PREDICT_F16 (include/yacht_hip.h)


class YkNet:
    """Owns a device copy of the weights in the kernels' layout (yk_net_create).

    precision "f32" (default): f32-equivalent products, within 1e-5 of the reference's float32
    predict.  "f16": fp16 weights / GEMM inputs with f32 accumulation and f32 Linear outputs - the
    operand precision of the reference's own GPU predict under autocast('cuda') (NNet.py:186-189;
    autocast also rounds the outputs to fp16, this mode does not), an opt-in perf mode."""

    def __init__(self, state_dict, hidden: int, nblocks: int, precision: str = "f32"):
        arrs = [np.ascontiguousarray(t.detach().to("cpu", torch.float32).numpy() if torch.is_tensor(t)
                                     else np.asarray(t, dtype=np.float32)) for t in state_dict.values()]
        if len(arrs) != 14 + 8 * nblocks:
            raise ValueError(f"state_dict has {len(arrs)} tensors, expected {14 + 8 * nblocks}")
        ptrs = (C.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
        h = C.c_void_p()
        call("yk_net_create", C.byref(h), hidden, nblocks, ptrs, len(arrs))
        self.handle = h.value
        self.hidden, self.nblocks = hidden, nblocks
        if precision not in PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(PRECISIONS)}")
        self.precision = precision
        call("yk_net_set_precision", self.handle, PRECISIONS[precision])

    def predict_states(self, states: torch.Tensor):
        """states int64[n, 8] (device) -> pi f32[n, 3226], v f32[n]."""
        n = states.shape[0]
        pi = torch.empty((n, ACTION_SIZE), dtype=torch.float32, device="cuda")
        v = torch.empty(n, dtype=torch.float32, device="cuda")
        call("yk_net_predict", self.handle, ptr(states.contiguous()), ptr(pi), ptr(v), n, stream_ptr())
        return pi, v

    def leaf_prior(self, states: torch.Tensor):
        """The self-play engine's leaf prior before renormalisation (yk_net_leaf_prior): pi at the
        valid actions of each canonical state (softmax over them), 0 elsewhere, and v."""
        n = states.shape[0]
        pi = torch.empty((n, ACTION_SIZE), dtype=torch.float32, device="cuda")
        v = torch.empty(n, dtype=torch.float32, device="cuda")
        call("yk_net_leaf_prior", self.handle, ptr(states.contiguous()), ptr(pi), ptr(v), n, stream_ptr())
        return pi, v

    def predict_features(self, x: torch.Tensor):
        x = x.to("cuda", torch.float32).contiguous()
        n = x.shape[0]
        pi = torch.empty((n, ACTION_SIZE), dtype=torch.float32, device="cuda")
        v = torch.empty(n, dtype=torch.float32, device="cuda")
        call("yk_net_predict_features", self.handle, ptr(x), ptr(pi), ptr(v), n, stream_ptr())
        return pi, v

    def policy_action(self, states: torch.Tensor):
        """states int64[n, 8] canonical (device) -> (actions i32[n], probs f32[n]): the most probable
        valid action per row, as the submission bot picks it (agent.py:248-280); -1 if none."""
        n = states.shape[0]
        actions = torch.empty(n, dtype=torch.int32, device="cuda")
        probs = torch.empty(n, dtype=torch.float32, device="cuda")
        call("yk_net_policy_action", self.handle, ptr(states.contiguous()), ptr(actions), ptr(probs), n,
             stream_ptr())
        return actions, probs

    def errors(self) -> int:
        """The device check flags of this net's forwards since the last call (yk_net_errors; synchronises
        the device): 0, or YK_NET_ERR_SYNC when a value-head wave timed out on its v_head.2 hand-off."""
        f = C.c_uint32()
        call("yk_net_errors", self.handle, C.byref(f))
        return int(f.value)

    def __del__(self):
        try:
            if getattr(self, "handle", None):
                lib().yk_net_destroy(self.handle)
                self.handle = None
        except Exception:
            pass


class NNetWrapper:
    """NeuralNet plugin (NeuralNet.py:14-50, NNet.py:91-213) with GPU inference."""

    def __init__(self, game, args=None):
        self.game = game
        self.args = args or DEFAULT_ARGS
        self.input_len = 59
        self.action_size = game.getActionSize()
        self.nnet = YachtNNet(self.input_len, self.action_size, self.args.hidden, self.args.nblocks,
                              self.args.dropout)
        self._yk = None
        self._yk_version = None

    def _weights_version(self):
        return tuple(p._version for p in self.nnet.parameters())

    def yk_net(self) -> YkNet:
        """Device weights for the kernels; rebuilt when the torch parameters change."""
        v = self._weights_version()
        if self._yk is None or v != self._yk_version:
            self._yk = YkNet(self.nnet.state_dict(), self.args.hidden, self.args.nblocks)
            self._yk_version = v
        return self._yk

    def predict(self, board):  # NNet.py:177-195
        pi, v = self.yk_net().predict_states(K.states_to_device(pack(board)))
        return pi[0].cpu().numpy(), np.float32(v[0].item())

    def predict_batch(self, states: torch.Tensor):
        return self.yk_net().predict_states(states)

    # ---- training (NNet.py:118-174) on the native trainer (yacht_amd/train.py)
    def uses_amp(self) -> bool:
        """The reference trains under autocast('cuda') + GradScaler whenever args.cuda
        (NNet.py:113-116, 141-155) and in float32 otherwise (:157-165): args.amp, when given,
        overrides that (amp=False: the float32 step on the GPU)."""
        a = self.args
        return bool(a.get("amp", a.get("cuda", True)))

    def _trainer(self):
        from .train import Trainer
        if getattr(self, "_tr", None) is None:
            a = self.args
            self._tr = Trainer(self.nnet.state_dict(), a.hidden, a.nblocks, lr=a.lr, weight_decay=a.weight_decay,
                               max_batch=a.batch_size, vloss_weight=a.get("vloss_weight", 1.0),
                               dropout=a.dropout, seed=a.get("seed", 0), amp=self.uses_amp())
        return self._tr

    def train(self, examples, verbose=True):
        """The reference loop: `epochs` passes over shuffled minibatches of `batch_size`
        (drop_last False), one CE(argmax pi) + vloss_weight * MSE step each, clip 5.0, AdamW -
        as the reference's GPU path when args.cuda (autocast('cuda') + GradScaler,
        NNet.py:113-116, 141-155) on fp16 MFMA kernels, or in float32 (the reference's CPU path)
        with args.cuda False or args.amp False (uses_amp).
        Shuffles come from a torch generator seeded per call (the reference uses the global
        torch RNG); dropout masks from the trainer's Philox stream.

        `examples`: the reference's list of (board, pi, v), an ExampleShard (device replay
        buffer), or a list of either (trainExamplesHistory).  Under torch.distributed every
        rank holds the same pooled examples and draws the same permutation, and
        args.ddp_batch picks how the ranks share a minibatch:
          "replicated" (default): every rank takes the whole minibatch's step itself - no
            collective, parameters bit-identical to one process training alone.  The step is
            latency-bound (a 16-row tile per workgroup, 32 of them at batch 512), so
            a rank's share of a split batch would not run faster, and the split adds an
            all-reduce per step;
          "split": the minibatch split across the ranks, the share-weighted gradients
            all-reduced (DDP): the single-process step up to f32 summation order;
          "per_rank": every rank its own batch_size rows (a world x batch_size global batch)."""
        from . import dist as D
        from .replay import as_device_examples
        tr = self._trainer()
        states, targets, values = as_device_examples(examples)
        rank, world = D.rank_world()
        n = states.shape[0]
        bs = self.args.batch_size
        mode = self.args.get("ddp_batch", "replicated") if world > 1 else "replicated"
        if mode not in ("replicated", "split", "per_rank"):
            raise ValueError(f"ddp_batch must be replicated, split or per_rank, not {mode!r}")
        rows = bs * world if mode == "per_rank" else bs
        vw = self.args.get("vloss_weight", 1.0)
        g = torch.Generator(device="cuda")
        g.manual_seed(int(self.args.get("seed", 0)) + 1000003 * tr.step_count)
        for epoch in range(self.args.epochs):
            perm = torch.randperm(n, generator=g, device="cuda").to(torch.int32)
            report = verbose and (epoch % 5 == 0 or epoch == self.args.epochs - 1)
            if report:
                tr.epoch_loss_begin(vw)  # summed on the device, read once after the epoch
            for i in range(0, n, rows):
                idx = perm[i:i + rows]
                if mode == "replicated":
                    tr.step(states, targets, values, idx=idx)
                    b = idx.numel()
                else:
                    parts = torch.tensor_split(idx, world)
                    loc = parts[rank]
                    b = loc.numel()
                    row0 = sum(int(x.numel()) for x in parts[:rank])  # this rank's rows in the minibatch
                    if b:
                        tr.backward(states, targets, values, idx=loc, row0=row0)
                    else:
                        tr.grads().zero_()
                    D.allreduce_grads(tr, weight=b / idx.numel())
                    tr.apply()
            if report:
                total, count = tr.epoch_loss_end()
                if rank == 0:
                    print(f"Epoch {epoch + 1}/{self.args.epochs}, Avg Loss: {total / max(count, 1):.4f}")
        with torch.no_grad():
            self.nnet.load_state_dict(tr.state_dict())  # the torch copy feeds checkpoints and predict
        self._yk = None

    # ---- checkpoints (NNet.py:198-213): the reference's dict, loaded without unpickling code
    def save_checkpoint(self, folder="checkpoint", filename="checkpoint.pth.tar"):
        from .train import optimizer_state_dict
        os.makedirs(folder, exist_ok=True)
        if getattr(self, "_tr", None) is not None:
            opt = optimizer_state_dict(self._tr, self.nnet, self.args.lr, self.args.weight_decay)
        else:
            opt = torch.optim.AdamW(self.nnet.parameters(), lr=self.args.lr,
                                    weight_decay=self.args.weight_decay).state_dict()
        torch.save({"state_dict": self.nnet.state_dict(), "optimizer": opt, "args": dict(self.args)},
                   os.path.join(folder, filename))

    def load_checkpoint(self, folder="checkpoint", filename="checkpoint.pth.tar", load_optimizer=False):
        from .train import load_optimizer_state_dict
        ck = torch.load(os.path.join(folder, filename), map_location="cpu", weights_only=True)
        sd = ck["state_dict"] if "state_dict" in ck else ck
        self.nnet.load_state_dict(OrderedDict(sd))
        self._yk = None
        if getattr(self, "_tr", None) is not None:
            self._tr.load_params(self.nnet.state_dict())
        if load_optimizer and "optimizer" in ck:
            load_optimizer_state_dict(self._trainer(), self.nnet, ck["optimizer"])


class HashPriorNet:
    """Deterministic stand-in for NNetWrapper (oracle/spec.py hash_prior, computed on the
    GPU by the engine itself).  It exists so whole self-play episodes can be compared
    bit-for-bit with the reference's own Coach/MCTS code; it is not a model."""

    yk_prior = "hash"

    def __init__(self, game=None, args=None):
        self.game = game

    def predict(self, board):
        pi, v = K.hash_prior(K.states_to_device(pack(board)))
        return pi[0].cpu().numpy(), np.float32(v[0].item())
