"""Pure-Python statement of the engine's data contracts. TEST INFRASTRUCTURE ONLY.

This module is part of the oracle: only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s cpu_baseline leg may import it, and only as the checker.  It states
three contracts that the HIP engine (``nypc-yacht-auction_amd/csrc``) and the C
restatement (``oracle/yk_oracle.c``) both implement:

1. **Packed state** - the 64-byte / 8 x u64 encoding of a reference ``YachtState``
   (``/root/reference/yacht/YachtGame.py:115-147``).  It is injective on exactly the
   fields ``stringRepresentation`` keys on (``YachtGame.py:448-467``), so equal packed
   words <=> equal transposition keys.
2. **RNG contract** - the reference draws from process-global MT19937 / CPython
   ``random`` (``YachtGame.py:154-159``, ``MCTS.py:46``, ``Coach.py:65``).  A batched
   engine needs one stream per game, so every draw is Philox4x32-10 keyed by
   ``seed`` and countered by ``(draw index, env id)``.  Each draw kind consumes one
   counter: ``die = 1 + below(6)`` (``roll_five``), ``below(2)`` (``tiebreak_uniform``),
   ``below(n)`` (``np.random.choice(array)``), ``uniform53`` (``np.random.choice(n, p=)``).
   Running the reference with these four functions patched in gives, per game, the
   exact sequence our engine must reproduce.
3. **Hash prior** - a deterministic stand-in for ``NNetWrapper.predict``
   (``yacht/NNet.py:177-195``) whose outputs are exact f32 values computable
   identically in Python, C and HIP.  It lets whole self-play episodes be compared
   bit-for-bit with the reference's own ``Coach``/``MCTS`` code.
"""
from __future__ import annotations

import numpy as np

M64 = (1 << 64) - 1
M32 = (1 << 32) - 1

NUM_CATEGORIES = 12
BID_LEVELS = 101
NUM_BID_ACTIONS = 202
NUM_COMB = 252
ACTION_SIZE = 3226

# ---------------------------------------------------------------- Philox4x32-10
PHILOX_M0 = 0xD2511F53
PHILOX_M1 = 0xCD9E8D57
PHILOX_W0 = 0x9E3779B9
PHILOX_W1 = 0xBB67AE85


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    for r in range(10):
        p0 = PHILOX_M0 * c0
        p1 = PHILOX_M1 * c2
        hi0, lo0 = p0 >> 32, p0 & M32
        hi1, lo1 = p1 >> 32, p1 & M32
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & M32, lo1, (hi0 ^ c3 ^ k1) & M32, lo0
        k0 = (k0 + PHILOX_W0) & M32
        k1 = (k1 + PHILOX_W1) & M32
    return c0, c1, c2, c3


def draw64(seed: int, env: int, ctr: int) -> int:
    x0, x1, _, _ = philox4x32_10(ctr & M32, (ctr >> 32) & M32, env & M32, 0,
                                 seed & M32, (seed >> 32) & M32)
    return x0 | (x1 << 32)


class Stream:
    """One game's draw stream: (seed, env id, counter)."""

    def __init__(self, seed: int, env: int, ctr: int = 0):
        self.seed, self.env, self.ctr = seed & M64, env & M32, ctr

    def next64(self) -> int:
        x = draw64(self.seed, self.env, self.ctr)
        self.ctr += 1
        return x

    def below(self, n: int) -> int:
        return ((self.next64() >> 32) * n) >> 32

    def die(self) -> int:
        return 1 + self.below(6)

    def uniform53(self) -> float:
        return (self.next64() >> 11) * (1.0 / 9007199254740992.0)


# ---------------------------------------------------------------- packed state
BID_NONE = 0xFF


def _bid_code(bid):
    if bid is None:
        return BID_NONE
    target, amount = bid
    assert amount % 500 == 0 and 0 <= amount <= 50000
    return ((0 if target == "A" else 1) << 7) | (amount // 500)


def _bid_decode(code):
    if code == BID_NONE:
        return None
    return ("A" if (code >> 7) == 0 else "B", 500 * (code & 0x7F))


def _nibbles(dice, nmax):
    assert len(dice) <= nmax
    v = 0
    for i, d in enumerate(dice):
        d = int(d)
        assert 1 <= d <= 6
        v |= d << (4 * i)
    return v


def pack_player(ps):
    carry = [int(d) for d in ps.carry]
    wa = _nibbles(carry, 10) | (len(carry) << 40) | ((int(ps.used_mask) & 0xFFF) << 44)
    cats = [int(c) for c in ps.cat_scores]
    for c in cats:
        assert c % 1000 == 0 and 0 <= c <= 255000
    wb = 0
    for i in range(8):
        wb |= (cats[i] // 1000) << (8 * i)
    wc = 0
    for i in range(4):
        wc |= (cats[8 + i] // 1000) << (8 * i)
    wc |= (int(ps.bid_score) & M32) << 32
    return wa, wb, wc


def pack_state(s) -> list:
    """Reference ``YachtState`` (duck-typed) -> 8 x u64 words."""
    w0 = (int(s.round_no) & 0xF) | ((int(s.phase) & 1) << 4)
    ra = [int(d) for d in s.rollA]
    rb = [int(d) for d in s.rollB]
    assert len(ra) in (0, 5) and len(rb) in (0, 5)
    if ra:
        w0 |= 1 << 5
    if rb:
        w0 |= 1 << 6
    w0 |= _bid_code(s.p1_bid) << 8
    w0 |= _bid_code(s.p2_bid) << 16
    w0 |= _nibbles(ra, 5) << 24
    w0 |= _nibbles(rb, 5) << 44
    return [w0, *pack_player(s.p1), *pack_player(s.p2), 0]


def unpack_words(w):
    """8 x u64 -> plain dict with the reference's field names (for tests)."""
    w0 = int(w[0])

    def dice(v, n):
        return [(v >> (4 * i)) & 0xF for i in range(n)]

    out = dict(round_no=w0 & 0xF, phase=(w0 >> 4) & 1,
               rollA=dice(w0 >> 24, 5) if (w0 >> 5) & 1 else [],
               rollB=dice(w0 >> 44, 5) if (w0 >> 6) & 1 else [],
               p1_bid=_bid_decode((w0 >> 8) & 0xFF), p2_bid=_bid_decode((w0 >> 16) & 0xFF))
    for p, base in (("p1", 1), ("p2", 4)):
        wa, wb, wc = int(w[base]), int(w[base + 1]), int(w[base + 2])
        n = (wa >> 40) & 0xF
        cats = [((wb >> (8 * i)) & 0xFF) * 1000 for i in range(8)] + \
               [((wc >> (8 * i)) & 0xFF) * 1000 for i in range(4)]
        bs = (wc >> 32) & M32
        if bs >= 1 << 31:
            bs -= 1 << 32
        out[p] = dict(carry=dice(wa, n), used_mask=(wa >> 44) & 0xFFF, cat_scores=cats, bid_score=bs)
    return out


# ---------------------------------------------------------------- hashing
def mix64(z: int) -> int:
    z &= M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def key_hash(words) -> int:
    """Transposition-key hash of a packed state (engine hash table + hash prior)."""
    h = 0x243F6A8885A308D3
    for i in range(8):
        h = mix64(h ^ ((int(words[i]) + 0x9E3779B97F4A7C15 * (i + 1)) & M64))
    return h


def hash_prior(words):
    """Deterministic predict() stand-in: (pi f32[3226], v np.float32), both exact f32."""
    h = key_hash(words)
    a = np.arange(1, ACTION_SIZE + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(h) ^ (a * np.uint64(0xD1B54A32D192ED03))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    q = ((z >> np.uint64(40)) & np.uint64(0xFFFF)).astype(np.float32)
    pi = (q + np.float32(1.0)) * np.float32(1.0 / 65536.0)
    zv = mix64(h ^ 0x8CB92BA72F3D8DD7)
    v = np.float32((((zv >> 40) & 0xFFFF) - 32768) / 32768.0)
    return pi.astype(np.float32), v


# ---------------------------------------------------------------- combos
def comb_5_of_10():
    import itertools
    return list(itertools.combinations(range(10), 5))


# ---------------------------------------------------------------- closed-form weights
def closed_form_weights(hidden: int = 256, nblocks: int = 6, input_len: int = 59,
                        action_size: int = ACTION_SIZE):
    """Deterministic YachtNNet parameters (state_dict names of
    ``yacht/pytorch/YachtNNet.py:30-52``), regenerable anywhere without shipping
    megabytes.  Linear weights follow the kaiming-uniform bound of ``_init``
    (``YachtNNet.py:56-60``) but use a sine sequence instead of an RNG; biases and
    LayerNorm affines are made non-trivial so that every term is exercised."""
    names = [("inp.0", "lin", input_len, hidden), ("inp.1", "ln", hidden, hidden)]
    for b in range(nblocks):
        names += [(f"blocks.{b}.fc1", "lin", hidden, hidden), (f"blocks.{b}.ln1", "ln", hidden, hidden),
                  (f"blocks.{b}.fc2", "lin", hidden, hidden), (f"blocks.{b}.ln2", "ln", hidden, hidden)]
    names += [("pi_head.0", "ln", hidden, hidden), ("pi_head.2", "lin", hidden, action_size),
              ("v_head.0", "ln", hidden, hidden), ("v_head.2", "lin", hidden, 128),
              ("v_head.4", "lin", 128, 1)]
    sd = {}
    for t, (name, kind, fan_in, fan_out) in enumerate(names):
        if kind == "lin":
            bound = np.sqrt(6.0 / fan_in)
            i = np.arange(fan_out * fan_in, dtype=np.float64)
            w = bound * np.sin(0.7548776662466927 * (i + 1.0) * (t + 1.0) + 0.3 * t)
            sd[name + ".weight"] = w.reshape(fan_out, fan_in).astype(np.float32)
            j = np.arange(fan_out, dtype=np.float64)
            sd[name + ".bias"] = (0.05 * np.cos(0.5698402909980532 * (j + 1.0) + t)).astype(np.float32)
        else:
            j = np.arange(fan_out, dtype=np.float64)
            sd[name + ".weight"] = (1.0 + 0.1 * np.sin(0.41 * (j + 1.0) + t)).astype(np.float32)
            sd[name + ".bias"] = (0.05 * np.cos(0.23 * (j + 1.0) + 2.0 * t)).astype(np.float32)
    return sd
