"""Arena on the MI355X engine (Arena.py:8-130, YachtPlayers.py:174-214).

``Arena(player1, player2, game)`` keeps the reference's sequential host loop for arbitrary
duck-typed players (``RandomYachtPlayer``, ``GreedyYachtPlayer`` - its heuristic runs on the
GPU, ``yk_greedy_action`` - or an MCTS lambda).  ``MCTSArena(game, nnet, args).playGames(num)``
is the batched form of config 4 - by default the MCTS agent
(``np.argmax(getActionProb(x, temp=0))``, Coach.py:124-125) against ``RandomYachtPlayer``, or
any pairing of "mcts" / "random" / "greedy" - with all ``num`` games played in one lock-step
device batch (``yk_arena``).  Randomness comes from per-game streams: game k of a playGames call uses
``(game seed, game env_id + k)``; the first num/2 games seat the agent as player 1, the
rest as player 2 (the reference swaps players after num/2 games, Arena.py:118).
Every game gets a fresh agent tree (the reference shares one MCTS across the games of a
playGames call; the two differ only when a game revisits a canonical state of an earlier one).
"""
from __future__ import annotations

import logging

import numpy as np

from .engine import SelfPlayEngine

log = logging.getLogger(__name__)


class RandomYachtPlayer:
    """Uniform random legal move from the game's stream (YachtPlayers.py:174-183)."""

    def __init__(self, game):
        self.game = game

    def play(self, board) -> int:
        legal = np.nonzero(self.game.getValidMoves(board, 1))[0]  # canonical player = 1
        return int(legal[self.game.rng.below(len(legal))]) if len(legal) else 0


class GreedyYachtPlayer:
    """Heuristic bidder + greedy scorer (YachtPlayers.py:186-214) on the canonical board; the
    heuristic runs on the GPU, a random-legal fallback draws from the game's stream."""

    def __init__(self, game, seed=None):
        self.game = game  # seed: the reference reseeds the global RNGs; streams are per game here

    def play(self, board) -> int:
        from . import kernels as K
        from .state import pack
        a = int(K.greedy_action(K.states_to_device(pack(board)))[0].item())
        if a >= 0:
            return a
        legal = np.nonzero(self.game.getValidMoves(board, 1))[0]
        return int(legal[self.game.rng.below(len(legal))]) if len(legal) else 0


class Arena:
    """Arena.py:8-130: the reference's sequential loop over duck-typed players."""

    def __init__(self, player1, player2, game, display=None):
        self.player1, self.player2, self.game, self.display = player1, player2, game, display

    def playGame(self, verbose=False):  # Arena.py:30-93
        players = [self.player2, None, self.player1]
        cur = 1
        board = self.game.getInitBoard()
        it = 0
        for p in (players[0], players[2]):
            if hasattr(p, "startGame"):
                p.startGame()
        while self.game.getGameEnded(board, cur) == 0:
            it += 1
            if verbose:
                assert self.display
                print("Turn ", str(it), "Player ", str(cur))
                self.display(board)
            canon = self.game.getCanonicalForm(board, cur)
            action = players[cur + 1](canon)
            valids = self.game.getValidMoves(canon, 1)
            if valids[action] == 0:
                log.error(f"Action {action} is not valid!")
                assert valids[action] > 0
            opponent = players[-cur + 1]
            if hasattr(opponent, "notify"):
                opponent.notify(board, action)
            board, cur = self.game.getNextState(board, cur, action)
        for p in (players[0], players[2]):
            if hasattr(p, "endGame"):
                p.endGame()
        result = self.game.getGameEnded(board, cur)
        log.info(f"Game finished: P1={board.p1.total_with_bonus()}, P2={board.p2.total_with_bonus()}")
        if verbose:
            assert self.display
            print("Game over: Turn ", str(it), "Result ", str(result))
            self.display(board)
        return cur * result

    def playGames(self, num, verbose=False):  # Arena.py:95-130
        num = int(num / 2)
        one = two = draws = 0
        for _ in range(num):
            r = self.playGame(verbose=verbose)
            one, two, draws = (one + 1, two, draws) if r == 1 else (one, two + 1, draws) if r == -1 else \
                (one, two, draws + 1)
        self.player1, self.player2 = self.player2, self.player1
        for _ in range(num):
            r = self.playGame(verbose=verbose)
            one, two, draws = (one + 1, two, draws) if r == -1 else (one, two + 1, draws) if r == 1 else \
                (one, two, draws + 1)
        return one, two, draws


class MCTSArena:
    """Batched Arena.playGames(num): `agent` (player1; default the MCTS agent over `nnet`) vs
    `opponent` (player2; default RandomYachtPlayer), each "mcts", "random" or "greedy"."""

    def __init__(self, game, nnet, args, agent="mcts", opponent="random"):
        self.game, self.nnet, self.args = game, nnet, args
        self.agent, self.opponent = agent, opponent
        self._games = 0
        self.last = None

    def _engine(self, n):
        uses_net = "mcts" in (self.agent, self.opponent) and self.nnet is not None
        prior = "hash" if not uses_net or getattr(self.nnet, "yk_prior", None) == "hash" else "net"
        net = None if prior == "hash" else self.nnet.yk_net()
        sims = self.args.numMCTSSims if "mcts" in (self.agent, self.opponent) else 1
        return SelfPlayEngine(n, sims, self.args.get("cpuct", 1.0), 0, net=net, prior=prior, max_moves=64)

    def play_batch(self, agent_seats) -> dict:
        """One device batch; agent_seats[i] in {1, -1}.  Returns the engine's arena results."""
        seats = np.asarray(agent_seats, dtype=np.int32)
        eng = self._engine(len(seats))
        try:
            eng.arena(seats, self.game.rng.seed, self.game.rng.env + self._games, agent=self.agent,
                      opponent=self.opponent)
            self._games += len(seats)
            self.last = eng.arena_results()
        finally:
            eng.close()
        return self.last

    def playGames(self, num, verbose=False):
        """Returns (oneWon, twoWon, draws) with the agent as player one, as Arena.py:95-130."""
        half = int(num / 2)
        seats = np.array([1] * half + [-1] * half, dtype=np.int32)
        r = self.play_batch(seats)["result"]
        agent = r * seats  # +1: the agent won
        one = int((agent == 1).sum())
        two = int((agent == -1).sum())
        return one, two, len(seats) - one - two


class GatingArena:
    """Coach.learn's gating arena (Coach.py:117-139): ``Arena(pmcts, nmcts).playGames(num)`` with
    pmcts = MCTS over the previous net and nmcts = MCTS over the new one, each
    ``np.argmax(getActionProb(x, temp=0))``, as ONE device batch on a dual-tree engine (one tree
    per seat, each seat its own net).  pmcts is player one of the first num/2 games and player
    two of the rest (Arena.py:118).  Game k uses stream (game seed, env_base + k).

    Under torch.distributed the games are sharded over the ranks (rank r plays games
    [r*c, (r+1)*c)) and the tallies summed, so every rank gets the single-GPU result."""

    def __init__(self, game, pnet, nnet, args):
        self.game, self.pnet, self.nnet, self.args = game, pnet, nnet, args
        self.last = None

    def playGames(self, num, env_base: int = None):
        """-> (pwins, nwins, draws): (oneWon, twoWon, draws) of Arena.playGames with pmcts as one."""
        from . import dist as D
        rank, world = D.rank_world()
        half = int(num / 2)
        total = 2 * half
        base = self.game.rng.env if env_base is None else env_base
        c, lo, hi = D.shard(total, rank, world)
        one = two = 0
        self.last = None
        if hi > lo:
            seats = np.where(np.arange(lo, hi) < half, 1, -1).astype(np.int32)
            hashed = getattr(self.pnet, "yk_prior", None) == "hash" and getattr(self.nnet, "yk_prior", None) == "hash"
            a = self.args
            eng = SelfPlayEngine(hi - lo, a.numMCTSSims, a.get("cpuct", 1.0), 0,
                                 net=None if hashed else self.pnet.yk_net(), prior="hash" if hashed else "net",
                                 opponent_net=None if hashed else self.nnet.yk_net(), max_moves=48, dual_trees=True)
            try:
                eng.arena(seats, self.game.rng.seed, base + lo, agent="mcts", opponent="mcts")
                self.last = eng.arena_results()
            finally:
                eng.close()
            p = self.last["result"] * seats  # +1: pmcts won
            one, two = int((p == 1).sum()), int((p == -1).sum())
        one, two, n = D.allreduce_counts([one, two, hi - lo], device="cuda")
        return one, two, n - one - two
