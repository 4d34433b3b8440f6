"""Batched Game-plugin kernels on device tensors (thin layer over include/yacht_hip.h).

States are ``torch.int64[n, 8]`` CUDA tensors holding the packed uint64 words
(``state.pack``).  Every function enqueues on the current torch stream.  There is no CPU
path: CPU tensors are rejected.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from ._lib import call, ptr, stream_ptr

ACTION_SIZE = 3226
MASK_WORDS = 101
FEATURES = 59


def _dev(x, dtype):
    t = torch.as_tensor(x, dtype=dtype)
    if not t.is_cuda:
        t = t.to("cuda")
    return t.contiguous()


def states_to_device(words) -> torch.Tensor:
    """numpy uint64[n, 8] (or [8]) -> CUDA int64[n, 8]."""
    a = np.ascontiguousarray(np.asarray(words, dtype=np.uint64).reshape(-1, 8))
    return torch.from_numpy(a.view(np.int64)).to("cuda")


def states_to_host(t: torch.Tensor) -> np.ndarray:
    return t.detach().to("cpu").contiguous().numpy().view(np.uint64).reshape(-1, 8)


def _bcast(x, n, dtype):
    t = _dev(x, dtype)
    if t.dim() == 0:
        t = t.expand(n)
    return t.reshape(n).contiguous()


def init_board(seed: int, env_ids, ctr):
    env = _dev(env_ids, torch.int32).reshape(-1)
    n = env.numel()
    c = _bcast(ctr, n, torch.int64).clone()
    out = torch.empty((n, 8), dtype=torch.int64, device="cuda")
    call("yk_init_board", ptr(out), ptr(c), ptr(env), seed & (2**64 - 1), n, stream_ptr())
    return out, c


def step(states, players, actions, seed: int, env_ids, ctr):
    st = _dev(states, torch.int64).reshape(-1, 8)
    n = st.shape[0]
    pl = _bcast(players, n, torch.int32)
    ac = _bcast(actions, n, torch.int32)
    env = _bcast(env_ids, n, torch.int32)
    c = _bcast(ctr, n, torch.int64).clone()
    out = torch.zeros((n, 8), dtype=torch.int64, device="cuda")
    npl = torch.zeros(n, dtype=torch.int32, device="cuda")
    status = torch.zeros(n, dtype=torch.int8, device="cuda")
    call("yk_step", ptr(st), ptr(pl), ptr(ac), seed & (2**64 - 1), ptr(env), ptr(c), ptr(out), ptr(npl),
         ptr(status), n, stream_ptr())
    return out, npl, status, c


def valid_mask(states, players):
    st = _dev(states, torch.int64).reshape(-1, 8)
    n = st.shape[0]
    pl = _bcast(players, n, torch.int32)
    mask = torch.zeros((n, MASK_WORDS), dtype=torch.int32, device="cuda")
    cnt = torch.zeros(n, dtype=torch.int32, device="cuda")
    call("yk_valid_mask", ptr(st), ptr(pl), ptr(mask), ptr(cnt), n, stream_ptr())
    return mask, cnt


def unpack_mask(mask: torch.Tensor) -> torch.Tensor:
    """[n, 101] int32 bit words -> [n, 3226] uint8 (bit a & 31 of word a >> 5)."""
    bits = torch.arange(32, device=mask.device, dtype=torch.int32)
    dense = ((mask.unsqueeze(-1) >> bits) & 1).reshape(mask.shape[0], -1)[:, :ACTION_SIZE]
    return dense.to(torch.uint8)


def ended(states, players):
    st = _dev(states, torch.int64).reshape(-1, 8)
    n = st.shape[0]
    pl = _bcast(players, n, torch.int32)
    r = torch.zeros(n, dtype=torch.float64, device="cuda")
    tot = torch.zeros((n, 2), dtype=torch.int32, device="cuda")
    call("yk_ended", ptr(st), ptr(pl), ptr(r), ptr(tot), n, stream_ptr())
    return r, tot


def canonical(states, players):
    st = _dev(states, torch.int64).reshape(-1, 8)
    n = st.shape[0]
    pl = _bcast(players, n, torch.int32)
    out = torch.empty_like(st)
    call("yk_canonical", ptr(st), ptr(pl), ptr(out), n, stream_ptr())
    return out


def score_table(states, players):
    st = _dev(states, torch.int64).reshape(-1, 8)
    n = st.shape[0]
    pl = _bcast(players, n, torch.int32)
    out = torch.empty((n, 12, 252), dtype=torch.int32, device="cuda")
    call("yk_score_table", ptr(st), ptr(pl), ptr(out), n, stream_ptr())
    return out


def score_dice(dice):
    d = _dev(dice, torch.int8).reshape(-1, 5)
    out = torch.empty((d.shape[0], 12), dtype=torch.int32, device="cuda")
    call("yk_score_dice", ptr(d), ptr(out), d.shape[0], stream_ptr())
    return out


def featurize(states):
    st = _dev(states, torch.int64).reshape(-1, 8)
    x = torch.empty((st.shape[0], FEATURES), dtype=torch.float32, device="cuda")
    call("yk_featurize", ptr(st), ptr(x), st.shape[0], stream_ptr())
    return x


def key_hash(states):
    st = _dev(states, torch.int64).reshape(-1, 8)
    out = torch.empty(st.shape[0], dtype=torch.int64, device="cuda")
    call("yk_key_hash", ptr(st), ptr(out), st.shape[0], stream_ptr())
    return out


def hash_prior(states):
    st = _dev(states, torch.int64).reshape(-1, 8)
    n = st.shape[0]
    pi = torch.empty((n, ACTION_SIZE), dtype=torch.float32, device="cuda")
    v = torch.empty(n, dtype=torch.float32, device="cuda")
    call("yk_hash_prior", ptr(st), ptr(pi), ptr(v), n, stream_ptr())
    return pi, v


__all__ = ["states_to_device", "states_to_host", "init_board", "step", "valid_mask", "unpack_mask", "ended",
           "canonical", "score_table", "score_dice", "featurize", "key_hash", "hash_prior", "_lib"]


def greedy_action(states):
    """GreedyYachtPlayer's heuristic on canonical boards: the action, or -1 where the player
    falls back to a random legal action (YachtPlayers.py:199-214)."""
    st = _dev(states, torch.int64).reshape(-1, 8)
    out = torch.empty(st.shape[0], dtype=torch.int32, device="cuda")
    call("yk_greedy_action", ptr(st), ptr(out), st.shape[0], stream_ptr())
    return out
