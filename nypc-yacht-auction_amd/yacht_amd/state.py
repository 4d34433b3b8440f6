"""Host-side game state objects and their 64-byte packed form.

``YachtState`` / ``PlayerState`` mirror the reference dataclasses field for field
(yacht/YachtGame.py:115-147), so code written against the reference keeps working.
``pack`` / ``unpack`` convert to the device layout of include/yacht_hip.h (8 x u64):

  w0 : round[0:4] phase[4] hasA[5] hasB[6] p1_bid[8:16] p2_bid[16:24] rollA[24:44] rollB[44:64]
  w1..w3 = p1, w4..w6 = p2:  carry nibbles[0:40] len[40:44] used[44:56] | cat[0..7] bytes |
                            cat[8..11] bytes, bid_score int32[32:64]
  w7 : 0

A bid byte is 0xFF (None) or target<<7 | amount/500; category scores are stored /1000.
The packing is injective on exactly the fields of ``stringRepresentation``
(YachtGame.py:448-467): equal words <=> same MCTS node.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import numpy as np

NUM_CATEGORIES = 12
CATEGORIES = ["ONE", "TWO", "THREE", "FOUR", "FIVE", "SIX", "CHOICE", "FOUR_OF_A_KIND", "FULL_HOUSE",
              "SMALL_STRAIGHT", "LARGE_STRAIGHT", "YACHT"]
BASIC_BONUS_THRESHOLD = 63000
BASIC_BONUS = 35000
BID_STEP = 500
BID_LEVELS = 101
BID_AMOUNTS = [i * BID_STEP for i in range(BID_LEVELS)]
NUM_BID_ACTIONS = 202
NUM_COMB = 252
NUM_SCORE_ACTIONS = NUM_CATEGORIES * NUM_COMB
ACTION_SIZE = NUM_BID_ACTIONS + NUM_SCORE_ACTIONS
PHASE_BID, PHASE_SCORE = 0, 1
FIRST_ROUND, LAST_ROUND = 1, 13
M32 = (1 << 32) - 1


def _combos():
    import itertools
    return list(itertools.combinations(range(10), 5))


COMB_5_OF_10 = _combos()


@dataclass
class PlayerState:
    carry: List[int] = field(default_factory=list)
    used_mask: int = 0
    cat_scores: List[int] = field(default_factory=lambda: [0] * NUM_CATEGORIES)
    bid_score: int = 0

    def basic_total(self) -> int:
        return sum(self.cat_scores[0:6])

    def total_with_bonus(self) -> int:
        bonus = BASIC_BONUS if self.basic_total() >= BASIC_BONUS_THRESHOLD else 0
        return sum(self.cat_scores) + bonus + self.bid_score


@dataclass
class YachtState:
    round_no: int = FIRST_ROUND
    phase: int = PHASE_BID
    rollA: List[int] = field(default_factory=list)
    rollB: List[int] = field(default_factory=list)
    p1_bid: Optional[Tuple[str, int]] = None
    p2_bid: Optional[Tuple[str, int]] = None
    p1: PlayerState = field(default_factory=PlayerState)
    p2: PlayerState = field(default_factory=PlayerState)


def decode_bid_action(a: int) -> Tuple[str, int]:  # YachtGame.py:168-171
    return ("A" if a // BID_LEVELS == 0 else "B", BID_AMOUNTS[a % BID_LEVELS])


def encode_bid_action(target: str, amount: int) -> int:  # YachtGame.py:162-165
    return (0 if target == "A" else 1) * BID_LEVELS + amount // BID_STEP


def decode_score_action(a: int):  # YachtGame.py:174-178
    base = a - NUM_BID_ACTIONS
    return base // NUM_COMB, COMB_5_OF_10[base % NUM_COMB]


def _bid_code(bid) -> int:
    if bid is None:
        return 0xFF
    target, amount = bid
    amount = int(amount)
    if amount % BID_STEP or not 0 <= amount <= 50000 or target not in ("A", "B"):
        raise ValueError(f"bid {bid!r} is not representable")
    return ((0 if target == "A" else 1) << 7) | (amount // BID_STEP)


def _nibbles(dice, nmax) -> int:
    if len(dice) > nmax:
        raise ValueError(f"{len(dice)} dice do not fit the packed state (max {nmax})")
    v = 0
    for i, d in enumerate(dice):
        d = int(d)
        if not 1 <= d <= 6:
            raise ValueError(f"die value {d} out of range")
        v |= d << (4 * i)
    return v


def _pack_player(ps: PlayerState):
    wa = _nibbles(ps.carry, 10) | (len(ps.carry) << 40) | ((int(ps.used_mask) & 0xFFF) << 44)
    wb = wc = 0
    for i, c in enumerate(ps.cat_scores):
        c = int(c)
        if c % 1000 or not 0 <= c <= 255000:
            raise ValueError(f"category score {c} is not representable")
        if i < 8:
            wb |= (c // 1000) << (8 * i)
        else:
            wc |= (c // 1000) << (8 * (i - 8))
    wc |= (int(ps.bid_score) & M32) << 32
    return wa, wb, wc


def pack(s: YachtState) -> np.ndarray:
    """YachtState -> uint64[8]."""
    if len(s.rollA) not in (0, 5) or len(s.rollB) not in (0, 5):
        raise ValueError("rolls hold 0 or 5 dice")
    w0 = (int(s.round_no) & 0xF) | ((int(s.phase) & 1) << 4)
    w0 |= (1 << 5) if len(s.rollA) else 0
    w0 |= (1 << 6) if len(s.rollB) else 0
    w0 |= _bid_code(s.p1_bid) << 8
    w0 |= _bid_code(s.p2_bid) << 16
    w0 |= _nibbles(s.rollA, 5) << 24
    w0 |= _nibbles(s.rollB, 5) << 44
    return np.array([w0, *_pack_player(s.p1), *_pack_player(s.p2), 0], dtype=np.uint64)


def pack_many(states) -> np.ndarray:
    return np.stack([pack(s) for s in states]) if len(states) else np.zeros((0, 8), dtype=np.uint64)


def _unpack_player(wa, wb, wc) -> PlayerState:
    n = (wa >> 40) & 0xF
    cats = [((wb >> (8 * i)) & 0xFF) * 1000 for i in range(8)] + [((wc >> (8 * i)) & 0xFF) * 1000 for i in range(4)]
    bs = (wc >> 32) & M32
    if bs >= 1 << 31:
        bs -= 1 << 32
    return PlayerState(carry=[(wa >> (4 * i)) & 0xF for i in range(n)], used_mask=(wa >> 44) & 0xFFF,
                       cat_scores=cats, bid_score=bs)


def unpack(w) -> YachtState:
    """uint64[8] -> YachtState."""
    w = [int(x) for x in w]
    w0 = w[0]

    def bid(code):
        return None if code == 0xFF else ("A" if code >> 7 == 0 else "B", 500 * (code & 0x7F))

    return YachtState(
        round_no=w0 & 0xF, phase=(w0 >> 4) & 1,
        rollA=[(w0 >> (24 + 4 * i)) & 0xF for i in range(5)] if (w0 >> 5) & 1 else [],
        rollB=[(w0 >> (44 + 4 * i)) & 0xF for i in range(5)] if (w0 >> 6) & 1 else [],
        p1_bid=bid((w0 >> 8) & 0xFF), p2_bid=bid((w0 >> 16) & 0xFF),
        p1=_unpack_player(w[1], w[2], w[3]), p2=_unpack_player(w[4], w[5], w[6]))


def string_representation(s: YachtState) -> str:
    """YachtGame.stringRepresentation (YachtGame.py:448-467), host-side."""
    p1, p2 = s.p1, s.p2
    return "|".join([
        f"r{s.round_no}", f"ph{s.phase}",
        f"A{''.join(map(str, s.rollA)) if s.rollA else '-'}",
        f"B{''.join(map(str, s.rollB)) if s.rollB else '-'}",
        f"p1b{s.p1_bid[0]}{s.p1_bid[1]}" if s.p1_bid else "p1b-",
        f"p2b{s.p2_bid[0]}{s.p2_bid[1]}" if s.p2_bid else "p2b-",
        f"p1c{''.join(map(str, p1.carry))}", f"p2c{''.join(map(str, p2.carry))}",
        f"p1u{p1.used_mask}", f"p2u{p2.used_mask}",
        f"p1s{','.join(map(str, p1.cat_scores))}", f"p2s{','.join(map(str, p2.cat_scores))}",
        f"p1bid{p1.bid_score}", f"p2bid{p2.bid_score}",
    ])
