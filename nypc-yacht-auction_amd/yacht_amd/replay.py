"""The replay buffer (Coach.py:84-101): self-play examples kept on the device.

Coach.learn keeps ``trainExamplesHistory``, one deque of ``(canonicalBoard, pi, v)`` per
iteration.  At config 5's scale (65536 games x 48 moves per iteration) those Python lists do
not fit (a dense pi is 3226 floats), and NNetWrapper.train only uses ``argmax(pi)`` of them
(NNet.py:145-146).  So an iteration's examples are an ``ExampleShard``: device arrays of
packed boards (64 B), argmax targets and float32 values, built by ``yk_examples_from_records``
straight from the (all-gathered) trajectory record images, plus the full visit policies as a
device CSR (``yk_examples_policies``) for the examples file (Coach.py:144-151) and for code that
iterates the reference's tuples.  The record images are not kept.
"""
from __future__ import annotations

import ctypes as C
from collections import deque

import numpy as np
import torch

from ._lib import call, stream_ptr


def _vcap(max_moves: int, sims: int) -> int:
    return 2 * max_moves * max(sims, 32)


class ExampleShard:
    """One iteration's examples (``iterationTrainExamples``, Coach.py:86-90) on the device:
    ``states`` int64[n, 8] (packed canonical boards), ``targets`` int32[n] (argmax pi),
    ``values`` float32[n], and - when built from record images - ``policies``: the full visit
    policies as a device CSR (``pi_indptr`` int64[n+1], ``pi_cols`` int32, ``pi_vals`` float64,
    ``values64`` float64[n]; yk_examples_policies).  ``len`` and iteration behave like the
    reference's deque of ``(YachtState, pi list, v)`` tuples."""

    def __init__(self, states, targets, values, policies=None):
        self.states, self.targets, self.values = states, targets, values
        self.policies = policies
        self._host = None

    def __len__(self):
        return int(self.targets.numel())

    def host(self) -> dict:
        """Host arrays of the shard with the full policies (float64 as MCTS.getActionProb returns
        them): states u64[n, 8], pi_indptr i64[n+1], pi_cols i32, pi_vals f64, values f64[n],
        targets i32[n].  One device-to-host copy of the compact arrays, cached."""
        if self._host is None:
            if self.policies is None:
                raise ValueError("this shard was not built from record images: it has no policies")
            P = self.policies
            self._host = dict(states=self.states.cpu().numpy().view(np.uint64), values=P["values64"].cpu().numpy(),
                              targets=self.targets.cpu().numpy(), pi_indptr=P["pi_indptr"].cpu().numpy(),
                              pi_cols=P["pi_cols"].cpu().numpy(), pi_vals=P["pi_vals"].cpu().numpy())
        return self._host

    def __iter__(self):
        from .state import ACTION_SIZE, unpack
        h = self.host()
        for k in range(len(self)):
            pi = [0.0] * ACTION_SIZE
            a0, a1 = int(h["pi_indptr"][k]), int(h["pi_indptr"][k + 1])
            for c, v in zip(h["pi_cols"][a0:a1], h["pi_vals"][a0:a1]):
                pi[int(c)] = float(v)
            yield unpack(h["states"][k]), pi, float(h["values"][k])

    def __getitem__(self, k):
        from .state import ACTION_SIZE, unpack
        h = self.host()
        k = range(len(self))[k]
        pi = [0.0] * ACTION_SIZE
        a0, a1 = int(h["pi_indptr"][k]), int(h["pi_indptr"][k + 1])
        for c, v in zip(h["pi_cols"][a0:a1], h["pi_vals"][a0:a1]):
            pi[int(c)] = float(v)
        return unpack(h["states"][k]), pi, float(h["values"][k])


def examples_from_images(images: torch.Tensor, n_envs: int, max_moves: int, sims: int, n_games: int = -1,
                         maxlen: int = None, stream=None) -> ExampleShard:
    """Record images (device uint8 [R, nbytes]: every rank's yk_engine_pack_records after the
    all-gather) -> ExampleShard of the first n_games games, keeping the last `maxlen` examples
    (the maxlenOfQueue deque, Coach.py:86-90).  The shard holds only compact arrays (examples and
    the policies' CSR, about a third of the images' bytes); the images can be released."""
    imgs = images.reshape(images.shape[0] if images.dim() > 1 else 1, -1).contiguous()
    R = imgs.shape[0]
    cnt = C.c_int64()
    sp = stream_ptr(stream)
    call("yk_examples_from_records", imgs.data_ptr(), R, n_envs, max_moves, sims, n_games, 0, 0, None, None, None,
         C.byref(cnt), sp)
    total = int(cnt.value)
    skip = max(total - int(maxlen), 0) if maxlen is not None else 0
    n = total - skip
    states = torch.empty((max(n, 1), 8), dtype=torch.int64, device="cuda")
    targets = torch.empty(max(n, 1), dtype=torch.int32, device="cuda")
    values = torch.empty(max(n, 1), dtype=torch.float32, device="cuda")
    call("yk_examples_from_records", imgs.data_ptr(), R, n_envs, max_moves, sims, n_games, skip, n,
         states.data_ptr(), targets.data_ptr(), values.data_ptr(), C.byref(cnt), sp)
    if int(cnt.value) != n:
        raise RuntimeError(f"yk_examples_from_records wrote {cnt.value} examples, expected {n}")
    indptr = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    nnz = C.c_int64()
    call("yk_examples_policies", imgs.data_ptr(), R, n_envs, max_moves, sims, n_games, skip, n, indptr.data_ptr(),
         None, None, 0, None, C.byref(nnz), sp)
    k = int(nnz.value)
    cols = torch.empty(max(k, 1), dtype=torch.int32, device="cuda")
    vals = torch.empty(max(k, 1), dtype=torch.float64, device="cuda")
    v64 = torch.empty(max(n, 1), dtype=torch.float64, device="cuda")
    call("yk_examples_policies", imgs.data_ptr(), R, n_envs, max_moves, sims, n_games, skip, n, indptr.data_ptr(),
         cols.data_ptr(), vals.data_ptr(), k, v64.data_ptr(), C.byref(nnz), sp)
    pol = dict(pi_indptr=indptr, pi_cols=cols[:k], pi_vals=vals[:k], values64=v64[:n])
    return ExampleShard(states[:n], targets[:n], values[:n], policies=pol)


# ---------------------------------------------------------------- what NNetWrapper.train takes
def _is_example(x) -> bool:
    return isinstance(x, tuple) and len(x) == 3 and not isinstance(x[0], (ExampleShard, list, deque))


def as_device_examples(examples):
    """examples: an ExampleShard, a list of (board, pi, v) tuples (Coach.py:72), or a list of
    either (trainExamplesHistory) -> device (states int64[n, 8], targets int32[n], values f32[n])."""
    from .train import examples_to_device
    if isinstance(examples, ExampleShard):
        return examples.states, examples.targets, examples.values
    items = list(examples)
    if not items or _is_example(items[0]):
        if not items:
            return (torch.zeros((0, 8), dtype=torch.int64, device="cuda"),
                    torch.zeros(0, dtype=torch.int32, device="cuda"), torch.zeros(0, dtype=torch.float32, device="cuda"))
        return examples_to_device(items)
    parts = [as_device_examples(x) for x in items]
    parts = [p for p in parts if p[1].numel()]
    if not parts:
        return as_device_examples([])
    if len(parts) == 1:
        return parts[0]
    return tuple(torch.cat([p[i] for p in parts]) for i in range(3))


__all__ = ["ExampleShard", "examples_from_images", "as_device_examples"]
