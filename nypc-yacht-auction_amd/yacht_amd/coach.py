"""Coach self-play on the MI355X engine (Coach.py:17-72).

``executeEpisode`` keeps the reference's return value - a list of
``(canonicalBoard, pi, v)`` - and ``executeEpisodes(n)`` plays n games in one lock-step
batch on the GPU (``SelfPlayEngine``).  Episode k of a Coach uses the RNG stream
``(game seed, game env_id + k)``; every episode starts from a fresh tree (Coach.py:93).
"""
from __future__ import annotations

import numpy as np

from .engine import SelfPlayEngine
from .mcts import MCTS
from .state import ACTION_SIZE, unpack


def examples_from_records(rec: dict, n_envs: int):
    """Engine records -> per-game lists of (YachtState, pi list, v) as Coach.py:72 returns."""
    out = []
    M = rec["states"].shape[1]
    for e in range(n_envs):
        ex = []
        for m in range(int(rec["n_moves"][e])):
            temp, _player, action = (int(x) for x in rec["info"][e, m, :3])
            a0, a1 = int(rec["visits_off"][e * M + m]), int(rec["visits_off"][e * M + m + 1])
            if temp == 0:
                pi = [0] * ACTION_SIZE
                pi[action] = 1
            else:
                counts = [0] * ACTION_SIZE
                for a, c in rec["visits"][a0:a1]:
                    counts[int(a)] = int(c)
                counts = [x ** 1.0 for x in counts]
                s = float(sum(counts))
                pi = [x / s for x in counts]
            ex.append((unpack(rec["states"][e, m]), pi, float(rec["values"][e, m])))
        out.append(ex)
    return out


class Coach:
    def __init__(self, game, nnet, args):
        self.game, self.nnet, self.args = game, nnet, args
        self.mcts = MCTS(game, nnet, args)
        self.trainExamplesHistory = []
        self.skipFirstSelfPlay = False
        self._episodes = 0

    def _engine(self, n):
        prior = "hash" if getattr(self.nnet, "yk_prior", None) == "hash" else "net"
        net = None if prior == "hash" else self.nnet.yk_net()
        return SelfPlayEngine(n, self.args.numMCTSSims, self.args.cpuct, self.args.tempThreshold, net=net,
                              prior=prior, max_moves=64)

    def executeEpisodes(self, n: int):
        eng = self._engine(n)
        eng.run(self.game.rng.seed, self.game.rng.env + self._episodes)
        self._episodes += n
        rec = eng.records()
        eng.close()
        return examples_from_records(rec, n)

    def executeEpisode(self):
        return self.executeEpisodes(1)[0]
