"""YachtGame on the MI355X kernels: the reference Game plugin surface, unchanged.

Mirrors ``yacht/YachtGame.py:210-467`` behind ``Game.py:14-113``: same method names,
argument meaning, return types and exceptions.  Each call is a batch of one on the GPU
(``yacht_amd.kernels``); the batched engine (``yacht_amd.engine``) is the fast path.

Randomness: the reference reseeds process-global numpy / ``random`` generators
(YachtGame.py:222-225).  Here a game owns one Philox stream ``(seed, env_id, counter)``
(include/yacht_hip.h) that MCTS and Coach also draw from, which is the single-game
equivalent of the reference's shared global RNG.
"""
from __future__ import annotations

import os
from typing import List, Optional, Tuple

import numpy as np

from . import kernels as K
from ._lib import ST_ASSERT, ST_CAPACITY, ST_OK, ST_RUNTIME, ST_VALUE_BID, ST_VALUE_SCORE
from .state import ACTION_SIZE, YachtState, pack, string_representation, unpack


class RngStream:
    """Host view of one game's draw stream (the counter lives here between calls)."""

    def __init__(self, seed: int, env: int = 0, ctr: int = 0):
        self.seed, self.env, self.ctr = int(seed) & (2**64 - 1), int(env) & (2**32 - 1), int(ctr)

    def draw64(self) -> int:
        from . import rng
        x = rng.draw64(self.seed, self.env, self.ctr)
        self.ctr += 1
        return x

    def below(self, n: int) -> int:
        return ((self.draw64() >> 32) * n) >> 32

    def uniform53(self) -> float:
        return (self.draw64() >> 11) * (1.0 / 9007199254740992.0)


def _raise_status(st: int):
    if st == ST_VALUE_BID:
        raise ValueError("Invalid action in BID phase")
    if st == ST_VALUE_SCORE:
        raise ValueError("Invalid action in SCORE phase")
    if st == ST_RUNTIME:
        raise RuntimeError("Invalid phase/state")
    if st == ST_ASSERT:
        raise AssertionError("both bids must be present to resolve")
    if st == ST_CAPACITY:
        raise OverflowError("a carry would exceed 10 dice (not reachable from getInitBoard)")


class YachtGame:
    """AlphaZero-General game wrapper for 13-round Yacht with bidding (GPU kernels)."""

    def __init__(self, seed: Optional[int] = None, env_id: int = 0):
        if seed is None:
            seed = int.from_bytes(os.urandom(8), "little")
        self.rng = RngStream(seed, env_id, 0)

    # ---- Game.py API
    def getInitBoard(self) -> YachtState:  # YachtGame.py:232-237
        out, c = K.init_board(self.rng.seed, [self.rng.env], self.rng.ctr)
        self.rng.ctr = int(c[0].item())
        return unpack(K.states_to_host(out)[0])

    def getBoardSize(self) -> Tuple[int, int]:
        return (1, 59)

    def getActionSize(self) -> int:
        return ACTION_SIZE

    def getNextState(self, board: YachtState, player: int, action: int) -> Tuple[YachtState, int]:
        out, npl, st, c = K.step(K.states_to_device(pack(board)), int(player), int(action), self.rng.seed,
                                 self.rng.env, self.rng.ctr)
        status = int(st[0].item())
        if status != ST_OK:
            _raise_status(status)
        self.rng.ctr = int(c[0].item())
        return unpack(K.states_to_host(out)[0]), int(npl[0].item())

    def getValidMoves(self, board: YachtState, player: int) -> np.ndarray:
        mask, _ = K.valid_mask(K.states_to_device(pack(board)), int(player))
        return K.unpack_mask(mask)[0].cpu().numpy()

    def getGameEnded(self, board: YachtState, player: int) -> float:
        r, _ = K.ended(K.states_to_device(pack(board)), int(player))
        return float(r[0].item())

    def getCanonicalForm(self, board: YachtState, player: int) -> YachtState:
        if player == 1:
            return board  # alias, as the reference (YachtGame.py:435-436)
        out = K.canonical(K.states_to_device(pack(board)), int(player))
        return unpack(K.states_to_host(out)[0])

    def getSymmetries(self, board: YachtState, pi) -> List[Tuple[YachtState, object]]:
        return [(board, pi)]

    def stringRepresentation(self, board: YachtState) -> str:
        return string_representation(board)

    def display(self, board: YachtState):
        pass
