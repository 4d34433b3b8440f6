"""Training on the MI355X: NNetWrapper.train (NNet.py:118-174) over the native
trainer of include/yacht_hip.h (yk_trainer_*).

A ``Trainer`` owns flat device buffers (parameters, gradients, AdamW moments) in
``YachtNNet.state_dict()`` order.  One ``step`` = gather + forward + backward + clip + AdamW for
a minibatch of replay entries; ``backward`` / ``apply`` split it so a DDP all-reduce of the
gradient buffer (``grads()``, zero-copy torch view) can run in between, as torch DDP does.
The replay buffer lives on the device as packed boards (64 B), hard targets (argmax of the
policy, NNet.py:145-146) and values.
"""
from __future__ import annotations

import ctypes as C
from collections import OrderedDict

import numpy as np
import torch

from ._lib import YkError, call, lib, ptr, stream_ptr


class _DevView:
    """__cuda_array_interface__ wrapper: a torch tensor view of a device buffer we own."""

    def __init__(self, p: int, n: int):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<f4", "data": (p, False), "version": 3}


class YkTrainConfig(C.Structure):
    _fields_ = [("max_batch", C.c_int), ("lr", C.c_float), ("weight_decay", C.c_float), ("beta1", C.c_float),
                ("beta2", C.c_float), ("eps", C.c_float), ("max_grad_norm", C.c_float),
                ("vloss_weight", C.c_float), ("dropout", C.c_float), ("seed", C.c_uint64), ("amp", C.c_int),
                ("init_scale", C.c_float), ("growth_interval", C.c_int)]


class Trainer:
    """amp=False: the float32 step (the reference's CPU path, NNet.py:157-165).  amp=True: the
    reference's GPU path (NNet.py:113-116, 141-155) - autocast('cuda') arithmetic on fp16 MFMA
    kernels, GradScaler('cuda') loss scaling (init_scale, growth_interval; a step whose gradients
    overflow is skipped and the scale halved)."""

    def __init__(self, state_dict, hidden: int, nblocks: int, lr=2e-3, weight_decay=1e-4, max_batch=512,
                 vloss_weight=1.5, dropout=0.3, seed=0, betas=(0.9, 0.999), eps=1e-8, max_grad_norm=5.0,
                 amp=False, init_scale=65536.0, growth_interval=2000):
        self.names = list(state_dict.keys())
        self.shapes = [tuple(t.shape) for t in state_dict.values()]
        arrs = [np.ascontiguousarray(t.detach().to("cpu", torch.float32).numpy()) for t in state_dict.values()]
        ptrs = (C.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
        self.cfg = YkTrainConfig(max_batch, lr, weight_decay, betas[0], betas[1], eps, max_grad_norm, vloss_weight,
                                 dropout, seed & (2**64 - 1), 1 if amp else 0, init_scale, growth_interval)
        self.amp = bool(amp)
        h = C.c_void_p()
        call("yk_trainer_create", C.byref(h), hidden, nblocks, ptrs, len(arrs), C.byref(self.cfg))
        self.handle = h.value
        self.hidden, self.nblocks, self.max_batch = hidden, nblocks, max_batch
        pp, gp, n = C.c_void_p(), C.c_void_p(), C.c_int64()
        call("yk_trainer_buffers", self.handle, C.byref(pp), C.byref(gp), C.byref(n))
        self.nparams = int(n.value)
        self._pptr, self._gptr = pp.value, gp.value

    # ---- device views (no copies)
    def params(self) -> torch.Tensor:
        return torch.as_tensor(_DevView(self._pptr, self.nparams), device="cuda")

    def grads(self) -> torch.Tensor:
        return torch.as_tensor(_DevView(self._gptr, self.nparams), device="cuda")

    # ---- steps
    def backward(self, states, targets, values, idx=None, batch=None, stream=None, row0=0):
        """row0: the global row of this batch's first example in the minibatch (dropout masks)."""
        n = int(batch if batch is not None else (idx.numel() if idx is not None else states.shape[0]))
        call("yk_trainer_set_row_offset", self.handle, int(row0))
        call("yk_trainer_backward", self.handle, ptr(states), ptr(targets), ptr(values),
             ptr(idx) if idx is not None else None, n, stream_ptr(stream))

    def apply(self, stream=None):
        call("yk_trainer_apply", self.handle, stream_ptr(stream))

    def step(self, states, targets, values, idx=None, batch=None, stream=None):
        n = int(batch if batch is not None else (idx.numel() if idx is not None else states.shape[0]))
        call("yk_trainer_set_row_offset", self.handle, 0)
        call("yk_trainer_step", self.handle, ptr(states), ptr(targets), ptr(values),
             ptr(idx) if idx is not None else None, n, stream_ptr(stream))

    def losses(self):
        """(sum of CE, sum of squared value error, grad sq-norm) of the last batch."""
        out = np.zeros(3, dtype=np.float64)
        call("yk_trainer_losses", self.handle, out.ctypes.data)
        return out

    def epoch_loss_begin(self, vloss_weight: float):
        """Start a device-side running sum of every later backward's ce/b + vw*se/b."""
        call("yk_trainer_epoch_loss_begin", self.handle, float(vloss_weight))

    def epoch_loss_end(self):
        """(sum of the batch losses since epoch_loss_begin, number of batches); synchronises."""
        out = np.zeros(2, dtype=np.float64)
        call("yk_trainer_epoch_loss_end", self.handle, out.ctypes.data)
        return float(out[0]), int(out[1])

    @property
    def step_count(self) -> int:
        """Optimiser steps taken (amp: skipped steps are not counted, as torch's AdamW state)."""
        return int(lib().yk_trainer_step_count(self.handle))

    def amp_state(self) -> dict:
        """GradScaler state (amp mode): scale, growth tracker, steps taken, last step skipped."""
        out = np.zeros(4, dtype=np.float64)
        call("yk_trainer_amp_state", self.handle, out.ctypes.data)
        return {"scale": float(out[0]), "growth_tracker": int(out[1]), "steps": int(out[2]),
                "found_inf": bool(out[3])}

    # ---- host copies in state_dict order
    def _get(self, which):
        outs = [np.zeros(s, dtype=np.float32) for s in self.shapes]
        arr = (C.c_void_p * len(outs))(*[o.ctypes.data for o in outs])
        call("yk_trainer_get", self.handle, which, arr)
        return OrderedDict((k, torch.from_numpy(o)) for k, o in zip(self.names, outs))

    def state_dict(self):
        return self._get(0)

    def gradients(self):
        return self._get(1)

    def moments(self):
        return self._get(2), self._get(3)

    def set_moments(self, exp_avg, exp_avg_sq, step: int):
        for which, d in ((2, exp_avg), (3, exp_avg_sq)):
            arrs = [np.ascontiguousarray(d[k].detach().to("cpu", torch.float32).numpy()) for k in self.names]
            p = (C.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
            call("yk_trainer_set", self.handle, which, p, int(step))

    def load_params(self, state_dict):
        arrs = [np.ascontiguousarray(state_dict[k].detach().to("cpu", torch.float32).numpy()) for k in self.names]
        p = (C.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
        call("yk_trainer_set", self.handle, 0, p, -1)

    def close(self):
        if getattr(self, "handle", None):
            lib().yk_trainer_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def examples_to_device(examples):
    """[(YachtState, pi, v)] (Coach.py:72) -> device (states int64[n, 8], targets int32[n], values f32[n]).
    The target is argmax(pi) - the reference's hard cross-entropy label (NNet.py:145-146)."""
    from . import kernels as K
    from .state import pack_many
    states = K.states_to_device(pack_many([b for b, _, _ in examples]))
    targets = torch.tensor([int(np.argmax(np.asarray(p))) for _, p, _ in examples], dtype=torch.int32, device="cuda")
    values = torch.tensor([float(v) for _, _, v in examples], dtype=torch.float32, device="cuda")
    return states, targets, values


def optimizer_state_dict(trainer: Trainer, model: torch.nn.Module, lr, weight_decay, betas=(0.9, 0.999), eps=1e-8):
    """The trainer's AdamW state as torch.optim.AdamW(model.parameters()).state_dict() (the
    'optimizer' entry of the reference checkpoint, NNet.py:198-205)."""
    opt = torch.optim.AdamW(model.parameters(), lr=lr, weight_decay=weight_decay, betas=betas, eps=eps)
    m, v = trainer.moments()
    step = trainer.step_count
    names = [n for n, _ in model.named_parameters()]
    if step > 0:
        for name, p in zip(names, model.parameters()):
            opt.state[p] = {"step": torch.tensor(float(step)), "exp_avg": m[name].clone(), "exp_avg_sq": v[name].clone()}
    return opt.state_dict()


def load_optimizer_state_dict(trainer: Trainer, model: torch.nn.Module, sd):
    """Inverse of optimizer_state_dict (a reference checkpoint's 'optimizer' entry)."""
    names = [n for n, _ in model.named_parameters()]
    st = sd.get("state", {})
    if not st:
        return
    m = OrderedDict((n, st[i]["exp_avg"]) for i, n in enumerate(names))
    v = OrderedDict((n, st[i]["exp_avg_sq"]) for i, n in enumerate(names))
    step = int(float(st[0]["step"]))
    trainer.set_moments(m, v, step)


__all__ = ["Trainer", "examples_to_device", "optimizer_state_dict", "load_optimizer_state_dict", "YkError"]
