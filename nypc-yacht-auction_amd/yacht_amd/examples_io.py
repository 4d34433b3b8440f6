"""Replay-buffer files (Coach.py:144-170).

The reference writes ``trainExamplesHistory`` - a list of per-iteration deques of
``(YachtState, pi, v)`` - with ``pickle.Pickler`` into ``<checkpoint>.examples``.

* ``save_examples`` / ``load_examples``: this framework's own format, a compressed ``.npz``
  (packed 64-byte boards, sparse policies, values, iteration sizes).  Nothing in it executes.
* ``load_reference_examples``: reads the reference's pickle with a whitelisting unpickler that
  only reconstructs ``yacht.YachtGame.YachtState`` / ``PlayerState`` (as this package's
  field-for-field dataclasses), ``collections.deque`` and numpy scalars; any other global in
  the file is refused, so loading runs no code from it.
* ``save_reference_examples``: writes a pickle the reference's ``loadTrainExamples`` reads
  (class references ``yacht.YachtGame.YachtState`` / ``PlayerState``).
"""
from __future__ import annotations

import collections
import io
import pickle
import sys
import types

import numpy as np

from .state import ACTION_SIZE, PlayerState, YachtState, pack_many, unpack


# ---------------------------------------------------------------- native format
def save_examples(path: str, history) -> None:
    """history: list (iterations) of iterables of (YachtState, pi, v)."""
    write_examples(path, examples_payload(history))


def write_examples(path: str, payload: dict) -> None:
    np.savez_compressed(path, **payload)


def examples_payload(history) -> dict:
    """The arrays save_examples writes (host copies: the history may change after this returns)."""
    from .replay import ExampleShard
    sizes, chunks, rows, cols, vals, values = [], [], [], [], [], []
    k = 0
    for it in history:
        if isinstance(it, ExampleShard):  # the device replay buffer: straight from its arrays
            h = it.host()
            n = len(it)
            sizes.append(n)
            lens = np.diff(h["pi_indptr"])
            rows.append(np.repeat(np.arange(k, k + n, dtype=np.int32), lens))
            cols.append(h["pi_cols"].astype(np.int16))
            vals.append(h["pi_vals"].astype(np.float64))
            chunks.append(np.asarray(h["states"], dtype=np.uint64).reshape(-1, 8))
            values.append(np.asarray(h["values"], dtype=np.float64))
            k += n
            continue
        it = list(it)
        sizes.append(len(it))
        if it:
            chunks.append(pack_many([b for b, _, _ in it]))
        for b, pi, v in it:
            p = np.asarray(pi, dtype=np.float64)
            nz = np.nonzero(p)[0]
            rows.append(np.full(len(nz), k, dtype=np.int32))
            cols.append(nz.astype(np.int16))
            vals.append(p[nz])
            values.append(np.array([float(v)], dtype=np.float64))
            k += 1
    return dict(format=np.array("yacht_amd.examples.v1"), sizes=np.array(sizes, dtype=np.int64),
                states=np.concatenate(chunks) if chunks else np.zeros((0, 8), np.uint64),
                pi_rows=np.concatenate(rows) if rows else np.zeros(0, np.int32),
                pi_cols=np.concatenate(cols) if cols else np.zeros(0, np.int16),
                pi_vals=np.concatenate(vals) if vals else np.zeros(0),
                values=np.concatenate(values) if values else np.zeros(0, np.float64))


def load_examples(path: str, boards: bool = True):
    """Inverse of save_examples: list of lists of (YachtState or packed words, pi list, v)."""
    with np.load(path, allow_pickle=False) as z:
        if str(z["format"]) != "yacht_amd.examples.v1":
            raise ValueError(f"{path}: not a yacht_amd examples file")
        sizes, states, values = z["sizes"], z["states"], z["values"]
        rows, cols, vals = z["pi_rows"], z["pi_cols"].astype(np.int64), z["pi_vals"]
    n = len(values)
    starts = np.searchsorted(rows, np.arange(n + 1))
    out, k = [], 0
    for sz in sizes:
        it = []
        for _ in range(int(sz)):
            pi = [0.0] * ACTION_SIZE
            for c, v in zip(cols[starts[k]:starts[k + 1]], vals[starts[k]:starts[k + 1]]):
                pi[int(c)] = float(v)
            it.append((unpack(states[k]) if boards else states[k], pi, float(values[k])))
            k += 1
        out.append(it)
    return out


def to_device_arrays(history):
    """Flatten to (packed states u64[n, 8], argmax targets i32[n], values f32[n]) for the trainer."""
    flat = [e for it in history for e in it]
    states = pack_many([e[0] for e in flat]) if flat else np.zeros((0, 8), np.uint64)
    targets = np.array([int(np.argmax(np.asarray(e[1]))) for e in flat], dtype=np.int32)
    values = np.array([float(e[2]) for e in flat], dtype=np.float32)
    return states, targets, values


# ---------------------------------------------------------------- the reference's pickle
_NUMPY_SCALAR = {("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar"), ("numpy", "dtype")}
try:
    from numpy._core.multiarray import scalar as _np_scalar
except ImportError:  # numpy < 2
    from numpy.core.multiarray import scalar as _np_scalar


class _ReferenceUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if (module, name) == ("yacht.YachtGame", "YachtState"):
            return YachtState
        if (module, name) == ("yacht.YachtGame", "PlayerState"):
            return PlayerState
        if (module, name) == ("collections", "deque"):
            return collections.deque
        if (module, name) in _NUMPY_SCALAR:  # numpy scalars inside the boards (np.random rolls)
            return np.dtype if name == "dtype" else _np_scalar
        raise pickle.UnpicklingError(f"refusing to load global {module}.{name} from an examples file")


def _plain(x):
    if isinstance(x, np.generic):
        return x.item()
    if isinstance(x, list):
        return [_plain(v) for v in x]
    if isinstance(x, tuple):
        return tuple(_plain(v) for v in x)
    return x


def _normalise_state(b: YachtState) -> YachtState:
    for f in ("rollA", "rollB", "p1_bid", "p2_bid", "round_no", "phase"):
        setattr(b, f, _plain(getattr(b, f)))
    for p in (b.p1, b.p2):
        p.carry = _plain(p.carry)
        p.cat_scores = _plain(p.cat_scores)
        p.used_mask = int(p.used_mask)
        p.bid_score = int(p.bid_score)
    return b


def load_reference_examples(path: str):
    """The reference's ``.examples`` pickle -> list of lists of (YachtState, pi list, v)."""
    with open(path, "rb") as f:
        hist = _ReferenceUnpickler(f).load()
    return [[(_normalise_state(b), [float(x) for x in pi], float(v)) for b, pi, v in it] for it in hist]


def save_reference_examples(path: str, history) -> None:
    """Write history in the reference's format (Pickler(f).dump, Coach.py:150-151)."""
    buf = io.BytesIO()
    saved = {k: sys.modules.get(k) for k in ("yacht", "yacht.YachtGame")}
    ys = type("YachtState", (), {"__module__": "yacht.YachtGame"})
    ps = type("PlayerState", (), {"__module__": "yacht.YachtGame"})
    mod = types.ModuleType("yacht.YachtGame")
    mod.YachtState, mod.PlayerState = ys, ps
    pkg = saved["yacht"] or types.ModuleType("yacht")

    def conv_p(p: PlayerState):
        o = ps.__new__(ps)
        o.__dict__.update(carry=list(p.carry), used_mask=int(p.used_mask), cat_scores=list(p.cat_scores),
                          bid_score=int(p.bid_score))
        return o

    def conv(b: YachtState):
        o = ys.__new__(ys)
        o.__dict__.update(round_no=int(b.round_no), phase=int(b.phase), rollA=list(b.rollA), rollB=list(b.rollB),
                          p1_bid=b.p1_bid, p2_bid=b.p2_bid, p1=conv_p(b.p1), p2=conv_p(b.p2))
        return o

    out = [collections.deque([(conv(b), list(pi), v) for b, pi, v in it]) for it in history]
    try:
        if saved["yacht"] is None:
            sys.modules["yacht"] = pkg
        sys.modules["yacht.YachtGame"] = mod
        pickle.Pickler(buf).dump(out)
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    with open(path, "wb") as f:
        f.write(buf.getvalue())
