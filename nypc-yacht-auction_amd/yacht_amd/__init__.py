"""yacht_amd - MI355X-native batched self-play for Yacht Auction.

Drop-in for the reference hot path Coach.executeEpisode -> MCTS.getActionProb ->
MCTS.search -> YachtGame / NNetWrapper.predict, implemented as hand-written gfx950 HIP
kernels behind a C ABI (include/yacht_hip.h, libyacht_hip.so).  The classes keep the
reference's plugin surface: YachtGame, NNetWrapper, MCTS, Coach.
"""
from ._lib import LIB_PATH, YkError, build, lib
from .state import ACTION_SIZE, PlayerState, YachtState, pack, pack_many, string_representation, unpack
from .utils import dotdict

__all__ = ["LIB_PATH", "YkError", "build", "lib", "ACTION_SIZE", "PlayerState", "YachtState", "pack", "pack_many",
           "unpack", "string_representation", "dotdict", "YachtGame", "NNetWrapper", "YachtNNet", "HashPriorNet",
           "MCTS", "Coach", "SelfPlayEngine"]


def __getattr__(name):  # lazy: torch-dependent modules
    if name == "YachtGame":
        from .game import YachtGame
        return YachtGame
    if name in ("NNetWrapper", "YachtNNet", "HashPriorNet", "YkNet"):
        from . import nnet
        return getattr(nnet, name)
    if name == "MCTS":
        from .mcts import MCTS
        return MCTS
    if name == "Coach":
        from .coach import Coach
        return Coach
    if name == "SelfPlayEngine":
        from .engine import SelfPlayEngine
        return SelfPlayEngine
    raise AttributeError(name)
