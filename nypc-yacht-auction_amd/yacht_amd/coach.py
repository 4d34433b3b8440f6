"""Coach self-play and learning on the MI355X engine (Coach.py:17-170).

``executeEpisode`` keeps the reference's return value - a list of
``(canonicalBoard, pi, v)`` - and ``executeEpisodes(n)`` plays n games in one lock-step
batch on the GPU (``SelfPlayEngine``).  ``learn`` is the reference loop at device scale and on
any number of ranks (one process per GPU, torch.distributed):

* self-play: the iteration's numEps games are sharded over the ranks by global env id, each
  rank's trajectory records are all-gathered (RCCL) and turned into device examples
  (``replay.ExampleShard``) - the same pooled buffer a single GPU playing every game builds;
* train: ``NNetWrapper.train`` on the pooled history, each minibatch split over the ranks with
  an all-reduce of the gradients (DDP), so every rank holds the same new net;
* gating: ``arena.GatingArena`` - pmcts vs nmcts as one dual-tree device batch, games sharded,
  tallies summed - then accept / reject as Coach.py:127-139.

Randomness comes from per-game Philox streams ``(game seed, env id)``: the Coach hands out
consecutive env ids starting at the game's own (``_streams``), episodes first, then each
iteration's arena games, so no two games ever share a stream.  Every episode starts from a
fresh tree (Coach.py:93).
"""
from __future__ import annotations

import logging
import os

from .engine import SelfPlayEngine
from .mcts import MCTS
from .state import ACTION_SIZE, unpack

# every real game has exactly 48 moves (2 bids in round 1, 2 bids + 2 scores in rounds 2-12,
# 2 scores in round 13; YachtGame.py:266-370): the record capacity of the Coach's engines, so
# the all-gathered images carry no padding moves (a longer game would be a move-cap error)
GAME_MOVES = 48


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
        self._next_env = game.rng.env
        self.last_pit = None

    def _streams(self, n: int) -> int:
        """Allocate n consecutive env ids (game streams); returns the first."""
        base = self._next_env
        self._next_env += n
        return base

    def _engine(self, n):
        prior = "hash" if getattr(self.nnet, "yk_prior", None) == "hash" else "net"
        net = None if prior == "hash" else self.nnet.yk_net()
        return SelfPlayEngine(n, self.args.numMCTSSims, self.args.cpuct, self.args.tempThreshold, net=net,
                              prior=prior, max_moves=GAME_MOVES)

    def executeEpisodes(self, n: int):
        """n episodes as the reference's per-game lists of (YachtState, pi, v) (this process only)."""
        eng = self._engine(n)
        eng.run(self.game.rng.seed, self._streams(n))
        rec = eng.records()
        eng.close()
        return examples_from_records(rec, n)

    def executeEpisode(self):
        return self.executeEpisodes(1)[0]

    def selfPlayExamples(self, n: int, maxlen: int = None):
        """One iteration's self-play (Coach.py:84-90) on every rank: game k of the n uses stream
        env0 + k and is played by rank k // ceil(n / world); the records are all-gathered and
        become the pooled ExampleShard (the last `maxlen` examples, the deque's maxlen)."""
        from . import dist as D
        from .replay import examples_from_images
        rank, world = D.rank_world()
        base = self._streams(n)
        c, lo, _hi = D.shard(n, rank, world)
        eng = self._engine(c)
        try:
            eng.run(self.game.rng.seed, base + lo)
            img = eng.pack_records()
        finally:
            eng.close()
        gathered = D.allgather_records(img)
        return examples_from_images(gathered, c, GAME_MOVES, self.args.numMCTSSims, n_games=n, maxlen=maxlen)

    # ---- Coach.learn (Coach.py:74-139)
    def learn(self):
        """numIters iterations: numEps self-play episodes (sharded over the ranks), the replay
        history (numItersForTrainExamplesHistory iterations), NNetWrapper.train, then
        arenaCompare games of the previous net against the new one (MCTS temp 0 each),
        accepting the new net when it wins >= updateThreshold of the decided games.  Rank 0
        writes the files; every rank reads the checkpoints back, so all ranks stay identical."""
        from . import dist as D
        from .arena import GatingArena
        import time

        import torch
        a = self.args
        rank, _world = D.rank_world()

        def clock():
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            return time.perf_counter()
        for i in range(1, a.numIters + 1):
            log.info(f"Starting Iter #{i} ...")
            t = {"t0": clock()}  # phase wall times of this iteration (self.phase_times)
            if not self.skipFirstSelfPlay or i > 1:
                self.trainExamplesHistory.append(self.selfPlayExamples(a.numEps, maxlen=a.maxlenOfQueue))
            t["selfplay"] = clock()
            if len(self.trainExamplesHistory) > a.numItersForTrainExamplesHistory:
                log.warning(f"Removing the oldest entry in trainExamples. len(trainExamplesHistory) = "
                            f"{len(self.trainExamplesHistory)}")
                self.trainExamplesHistory.pop(0)
            if rank == 0:
                self.saveTrainExamples(i - 1)
                self.nnet.save_checkpoint(folder=a.checkpoint, filename="temp.pth.tar")
            D.barrier()
            self.pnet.load_checkpoint(folder=a.checkpoint, filename="temp.pth.tar")
            t["save"] = clock()
            # the reference shuffles the pooled examples here (Coach.py:104-108) and its
            # DataLoader(shuffle=True) reshuffles every epoch; train's per-epoch permutation is
            # that reshuffle
            self.nnet.train(self.trainExamplesHistory)
            t["train"] = clock()
            log.info("PITTING AGAINST PREVIOUS VERSION")
            pwins, nwins, draws = GatingArena(self.game, self.pnet, self.nnet, a).playGames(
                a.arenaCompare, env_base=self._streams(2 * int(a.arenaCompare / 2)))
            t["arena"] = clock()
            log.info("NEW/PREV WINS : %d / %d ; DRAWS : %d" % (nwins, pwins, draws))
            D.barrier()  # every rank has read temp.pth.tar before it can be rewritten
            if pwins + nwins == 0 or float(nwins) / (pwins + nwins) < a.updateThreshold:
                log.info("REJECTING NEW MODEL")
                self.nnet.load_checkpoint(folder=a.checkpoint, filename="temp.pth.tar")
            else:
                log.info("ACCEPTING NEW MODEL")
                if rank == 0:
                    self.nnet.save_checkpoint(folder=a.checkpoint, filename=self.getCheckpointFile(i))
                    self.nnet.save_checkpoint(folder=a.checkpoint, filename="best.pth.tar")
            self.last_pit = (pwins, nwins, draws)
            D.barrier()
            t["gate"] = clock()
            keys = ["t0", "selfplay", "save", "train", "arena", "gate"]
            self.phase_times = {k + "_s": t[k] - t[p] for p, k in zip(keys, keys[1:])}
            self.phase_times["iteration_s"] = t["gate"] - t["t0"]
        self.wait_saves()

    def getCheckpointFile(self, iteration):
        return "checkpoint_" + str(iteration) + ".pth.tar"

    # ---- the replay buffer on disk (Coach.py:144-170): this framework's npz and, when asked
    # for (examples_format "reference" / "both"), the reference's pickle next to it
    def saveTrainExamples(self, iteration):
        """Coach.py:144-152.  The npz's arrays are copied to the host here; the compressed write
        runs on a background thread (joined before the next write, a load, and at the end of
        learn), so the iteration's training does not wait for the disk."""
        import threading

        from .examples_io import examples_payload, save_reference_examples, write_examples
        folder = self.args.checkpoint
        os.makedirs(folder, exist_ok=True)
        base = os.path.join(folder, self.getCheckpointFile(iteration) + ".examples")
        fmt = self.args.get("examples_format", "npz")  # the dense reference pickle grows ~29 KB / example
        if fmt in ("both", "reference"):
            save_reference_examples(base, self.trainExamplesHistory)
        if fmt in ("both", "npz"):
            payload = examples_payload(self.trainExamplesHistory)
            self.wait_saves()
            self._saver = threading.Thread(target=write_examples, args=(base + ".npz", payload))
            self._saver.start()

    def wait_saves(self):
        """Join the background examples write, if one is running."""
        t = getattr(self, "_saver", None)
        if t is not None:
            t.join()
            self._saver = None

    def loadTrainExamples(self):
        from .examples_io import load_examples, load_reference_examples
        self.wait_saves()
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
