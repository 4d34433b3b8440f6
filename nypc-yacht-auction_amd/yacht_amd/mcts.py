"""MCTS plugin on the MI355X engine: MCTS(game, nnet, args).getActionProb (MCTS.py:28-54).

The search itself (``MCTS.search``, MCTS.py:56-164) runs on the device through
``yk_mcts_search`` with a persistent per-instance tree, drawing from the game's RNG
stream exactly where the reference draws from its global RNG.  The visit-count policy
and the temperature-0 tie pick (``np.random.choice(bestAs)``) are done here on the host.
"""
from __future__ import annotations

import torch

from . import kernels as K
from ._lib import call, stream_ptr
from .engine import SelfPlayEngine
from .state import ACTION_SIZE, pack


class MCTS:
    def __init__(self, game, nnet, args):
        self.game, self.nnet, self.args = game, nnet, args
        self._engine = None
        self._round = 0  # round of the last root: a lower one starts a new game (fresh tree)

    def _eng(self):
        if self._engine is None:
            if getattr(self.nnet, "yk_prior", None) == "hash":
                self._engine = SelfPlayEngine(1, self.args.numMCTSSims, self.args.cpuct, prior="hash", max_moves=1)
            else:
                self._engine = SelfPlayEngine(1, self.args.numMCTSSims, self.args.cpuct, net=self.nnet.yk_net(),
                                              max_moves=1)
            call("yk_mcts_reset", self._engine.handle)
        return self._engine

    def search_counts(self, canonicalBoard, sims=None):
        """Run `sims` searches from the root; return the root's visit counts (list)."""
        eng = self._eng()
        rng = self.game.rng
        if canonicalBoard.round_no < self._round:
            # a new game (Arena.playGames reuses one MCTS, Coach.py:124-125): the device trees
            # only keep rounds >= the root's, so the new game starts from a fresh tree
            call("yk_mcts_reset", eng.handle)
        self._round = canonicalBoard.round_no
        roots = K.states_to_device(pack(canonicalBoard))
        env = torch.tensor([rng.env], dtype=torch.int32, device="cuda")
        ctr = torch.tensor([rng.ctr], dtype=torch.int64, device="cuda")
        counts = torch.zeros((1, ACTION_SIZE), dtype=torch.int32, device="cuda")
        call("yk_mcts_search", eng.handle, roots.data_ptr(), rng.seed, env.data_ptr(), ctr.data_ptr(),
             int(self.args.numMCTSSims if sims is None else sims), counts.data_ptr(), stream_ptr())
        rng.ctr = int(ctr.item())
        return counts[0].cpu().tolist()

    def getActionProb(self, canonicalBoard, temp=1):
        counts = self.search_counts(canonicalBoard)
        if temp == 0:
            m = max(counts)
            best = [a for a, c in enumerate(counts) if c == m]
            best_a = best[self.game.rng.below(len(best))]  # np.random.choice(bestAs), MCTS.py:46
            probs = [0] * len(counts)
            probs[best_a] = 1
            return probs
        counts = [x ** (1. / temp) for x in counts]
        counts_sum = float(sum(counts))
        return [x / counts_sum for x in counts]
