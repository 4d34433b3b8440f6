"""Coach self-play on the MI355X engine (Coach.py:17-72).

``executeEpisode`` keeps the reference's return value - a list of
``(canonicalBoard, pi, v)`` - and ``executeEpisodes(n)`` plays n games in one lock-step
batch on the GPU (``SelfPlayEngine``).  Episode k of a Coach uses the RNG stream
``(game seed, game env_id + k)``; every episode starts from a fresh tree (Coach.py:93).
"""
from __future__ import annotations

import logging
import os
import random
from collections import deque

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


log = logging.getLogger(__name__)


class Coach:
    def __init__(self, game, nnet, args):
        self.game, self.nnet, self.args = game, nnet, args
        # the competitor network with the same args (Coach.py:26-27)
        self.pnet = nnet.__class__(game, args) if hasattr(nnet, "train") else None
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

    # ---- Coach.learn (Coach.py:74-139)
    def learn(self):
        """numIters iterations: numEps self-play episodes (one device batch), the replay history
        (numItersForTrainExamplesHistory iterations), NNetWrapper.train, then arenaCompare games of
        the previous net against the new one (MCTS temp 0 each), accepting the new net when it
        wins >= updateThreshold of the decided games."""
        from .arena import Arena
        a = self.args
        for i in range(1, a.numIters + 1):
            log.info(f"Starting Iter #{i} ...")
            if not self.skipFirstSelfPlay or i > 1:
                it = deque([], maxlen=a.maxlenOfQueue)
                for ep in self.executeEpisodes(a.numEps):
                    it += ep
                self.trainExamplesHistory.append(it)
            if len(self.trainExamplesHistory) > a.numItersForTrainExamplesHistory:
                log.warning(f"Removing the oldest entry in trainExamples. len(trainExamplesHistory) = "
                            f"{len(self.trainExamplesHistory)}")
                self.trainExamplesHistory.pop(0)
            self.saveTrainExamples(i - 1)
            trainExamples = [e for h in self.trainExamplesHistory for e in h]
            random.Random(self.game.rng.seed + i).shuffle(trainExamples)
            self.nnet.save_checkpoint(folder=a.checkpoint, filename="temp.pth.tar")
            self.pnet.load_checkpoint(folder=a.checkpoint, filename="temp.pth.tar")
            pmcts = MCTS(self.game, self.pnet, a)
            self.nnet.train(trainExamples)
            nmcts = MCTS(self.game, self.nnet, a)
            log.info("PITTING AGAINST PREVIOUS VERSION")
            arena = Arena(lambda x: int(np.argmax(pmcts.getActionProb(x, temp=0))),
                          lambda x: int(np.argmax(nmcts.getActionProb(x, temp=0))), self.game)
            pwins, nwins, draws = arena.playGames(a.arenaCompare)
            log.info("NEW/PREV WINS : %d / %d ; DRAWS : %d" % (nwins, pwins, draws))
            if pwins + nwins == 0 or float(nwins) / (pwins + nwins) < a.updateThreshold:
                log.info("REJECTING NEW MODEL")
                self.nnet.load_checkpoint(folder=a.checkpoint, filename="temp.pth.tar")
            else:
                log.info("ACCEPTING NEW MODEL")
                self.nnet.save_checkpoint(folder=a.checkpoint, filename=self.getCheckpointFile(i))
                self.nnet.save_checkpoint(folder=a.checkpoint, filename="best.pth.tar")
            self.last_pit = (pwins, nwins, draws)

    def getCheckpointFile(self, iteration):
        return "checkpoint_" + str(iteration) + ".pth.tar"

    # ---- the replay buffer on disk (Coach.py:144-170): the reference's pickle (readable by the
    # reference) and this framework's npz next to it
    def saveTrainExamples(self, iteration):
        from .examples_io import save_examples, save_reference_examples
        folder = self.args.checkpoint
        os.makedirs(folder, exist_ok=True)
        base = os.path.join(folder, self.getCheckpointFile(iteration) + ".examples")
        fmt = self.args.get("examples_format", "both")  # the dense reference pickle grows ~29 KB / example
        if fmt in ("both", "reference"):
            save_reference_examples(base, self.trainExamplesHistory)
        if fmt in ("both", "npz"):
            save_examples(base + ".npz", self.trainExamplesHistory)

    def loadTrainExamples(self):
        from .examples_io import load_examples, load_reference_examples
        modelFile = os.path.join(self.args.load_folder_file[0], self.args.load_folder_file[1])
        examplesFile = modelFile + ".examples"
        if os.path.isfile(examplesFile + ".npz"):
            self.trainExamplesHistory = load_examples(examplesFile + ".npz")
        elif os.path.isfile(examplesFile):
            self.trainExamplesHistory = load_reference_examples(examplesFile)
        else:
            log.warning(f'File "{examplesFile}" with trainExamples not found!')
            return
        log.info("Loading done!")
        self.skipFirstSelfPlay = True  # examples based on the model were already collected
