"""Config 5 at its per-GPU shape: two Coach.learn iterations (Coach.py:74-139)
on one rank with main.py's args (main.py:17-43): 8192 self-play games x 25 sims per iteration (the
65,536 games of config 5 over 8 GPUs), YachtNNet 256 x 6, maxlenOfQueue 200,000, 15 epochs of
batch 512 in the reference's GPU train arithmetic (args.cuda: autocast + GradScaler, NNet.py:113-116),
dropout 0.3, numItersForTrainExamplesHistory 5, arenaCompare 10.  Checked:

* every 128th self-play game of both iterations is replayed bit for bit by the oracle from the
  predictions the engine expanded with (visit counts of every move, actions, RNG counters, values,
  final boards), and the first iteration's recorded priors are held against a float64 forward
  (helpers.check_recorded_priors);
* the pooled history: each iteration's ExampleShard equals the host restatement
  (helpers.host_examples) of that iteration's record image, trimmed to the maxlenOfQueue deque's
  newest 200,000 examples (Coach.py:86-90), and the second iteration trains on both entries
  (Coach.py:99-111);
* the trainer Coach.learn itself ran: its first 3 amp steps (dropout 0.3) are recorded as they
  happen (minibatch indices, losses, parameters, GradScaler state), a standalone Trainer given the
  same examples, indices, seed and dropout reproduces them bit for bit, and those recorded steps
  are held against torch autocast('cuda') + GradScaler('cuda') on the same minibatches WITH THE
  SAME DROPOUT MASKS (helpers.dropout_keep_np restates the trainer's Philox keep bits; torch's
  nn.Dropout modules replaced by those fixed masks x 1/(1-p)), within
  test_amp_steps_vs_torch_autocast_gradscaler's tolerance;
* each iteration's gate tally equals a fresh, unsharded GatingArena run on the same two nets and
  env ids (Coach.py:117-139)."""
import os

import numpy as np
import pytest

from oracle import oracle as O
from helpers import check_recorded_priors, dropout_keep_np, host_examples

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

GAMES, SIMS, STRIDE, MAXLEN = 8192, 25, 128, 200000


def _dense_counts(rec, e, m):
    M = rec["states"].shape[1]
    a0, a1 = rec["visits_off"][e * M + m], rec["visits_off"][e * M + m + 1]
    c = np.zeros(3226, dtype=np.int32)
    v = rec["visits"][a0:a1]
    c[v[:, 0]] = v[:, 1]
    return c


def _replay_sampled_games(play):
    """The oracle replays the recorded games (every STRIDE-th) from the engine's own predictions."""
    rec, pi, v, cnt = play["rec"], play["pi"], play["v"], play["cnt"]
    pick = np.arange(0, GAMES, STRIDE)
    replay = [(pi[r, :cnt[r]], v[r, :cnt[r]]) for r in range(len(pick))]
    orc = O.selfplay(play["base"] + pick, play["seed"], SIMS, 1.5, 15, O.MODE_REPLAY, replay=replay, max_moves=48,
                     threads=16)
    assert orc["nerr"] == 0
    assert np.array_equal(orc["stats"][:, 1], cnt)
    for r, e in enumerate(pick):
        M = int(orc["stats"][r, 0])
        assert rec["n_moves"][e] == M == 48
        assert np.array_equal(rec["states"][e, :M], orc["canon"][r, :M])
        assert np.array_equal(rec["info"][e, :M, :7], orc["mv"][r, :M, :7]), e
        assert np.array_equal(rec["ctr"][e, :M], orc["ctr"][r, :M])
        for m in range(M):
            assert np.array_equal(_dense_counts(rec, e, m), orc["counts"][r, m]), (e, m)
        assert np.array_equal(rec["values"][e, :M], orc["values"][r, :M])
        assert np.array_equal(rec["final"][e], orc["final"][r])


def _same_as_host(shard, img):
    """The pooled device examples == helpers.host_examples of the record image, deque-trimmed."""
    from yacht_amd import replay as R
    h = host_examples(img[None], GAMES, 48, SIMS)
    total = len(h["targets"])
    assert total == GAMES * 48
    skip = total - MAXLEN
    assert len(shard) == MAXLEN
    assert np.array_equal(shard.states.cpu().numpy().view(np.uint64), h["states"][skip:])
    assert np.array_equal(shard.targets.cpu().numpy(), h["targets"][skip:])
    assert np.array_equal(shard.values.cpu().numpy(), h["values"][skip:].astype(np.float32))
    got = shard.host()
    ip = h["pi_indptr"]
    a0, a1 = int(ip[skip]), int(ip[total])
    assert np.array_equal(got["pi_indptr"], ip[skip:] - a0)
    assert np.array_equal(got["pi_cols"], h["pi_cols"][a0:a1])
    assert np.array_equal(got["pi_vals"], h["pi_vals"][a0:a1])
    assert np.array_equal(got["values"], h["values"][skip:])


def test_config5_two_coach_iterations(tmp_path, monkeypatch):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from test_gpu_train import _relnorm, _torch_train_steps
    from yacht_amd import arena as AM
    from yacht_amd import coach as CM
    from yacht_amd import engine as EM
    from yacht_amd import kernels as K
    from yacht_amd.coach import Coach
    from yacht_amd.game import YachtGame
    from yacht_amd.nnet import NNetWrapper, YkNet
    from yacht_amd.train import Trainer
    from yacht_amd.utils import dotdict
    d = str(tmp_path)
    args = dotdict(numIters=2, numEps=GAMES, tempThreshold=15, updateThreshold=0.55, maxlenOfQueue=MAXLEN,
                   numMCTSSims=SIMS, arenaCompare=10, cpuct=1.5, checkpoint=d, load_folder_file=(d, "best.pth.tar"),
                   numItersForTrainExamplesHistory=5, lr=2e-3, weight_decay=1e-4, epochs=15, batch_size=512,
                   vloss_weight=1.5, cuda=True, hidden=256, nblocks=6, dropout=0.3, examples_format="npz", seed=5)
    torch.manual_seed(17)
    game = YachtGame(seed=41, env_id=3 * 10**6)
    nn = NNetWrapper(game, args)
    assert nn.uses_amp()  # args.cuda: the reference's autocast + GradScaler arithmetic
    sd0 = {k: v.detach().clone() for k, v in nn.nnet.state_dict().items()}
    c = Coach(game, nn, args)

    plays, gates = [], []

    class RecordingEngine(EM.SelfPlayEngine):
        """The Coach's self-play engine, recording every STRIDE-th game's predictions (the path
        does not change) and keeping the records, the image and the weights when it closes."""

        def __init__(self, n, sims, cpuct, temp, net=None, prior="net", max_moves=48, **kw):
            super().__init__(n, sims, cpuct, temp, net=net, prior=prior, max_moves=max_moves, record_predictions=True,
                             max_expansions=48 * sims + 8, record_stride=STRIDE)
            self._sd = {k: v.detach().cpu().numpy().copy() for k, v in c.nnet.nnet.state_dict().items()}

        def run(self, seed, env_base=0, stream=None):
            self._seed, self._base = seed, env_base
            super().run(seed, env_base, stream)

        def close(self):
            if getattr(self, "handle", None):
                assert self.stats()["errors"] == 0
                pi, v, cnt, leaves = self.predictions(leaves=True)
                plays.append(dict(rec=self.records(), pi=pi, v=v, cnt=cnt, leaves=leaves, seed=self._seed,
                                  base=self._base, img=self.pack_records().cpu().numpy(), sd=self._sd))
            super().close()

    class RecordingGate(AM.GatingArena):
        def playGames(self, num, env_base=None):
            tally = super().playGames(num, env_base=env_base)
            gates.append(dict(num=num, env_base=env_base, tally=tally,
                              p={k: v.detach().clone() for k, v in self.pnet.nnet.state_dict().items()},
                              n={k: v.detach().clone() for k, v in self.nnet.nnet.state_dict().items()}))
            return tally

    # the Coach's own trainer: its first 3 steps as they happen
    from yacht_amd import train as TM
    rec_steps = dict(trainer=None, idx=[], losses=[], amp=[])
    real_step = TM.Trainer.step

    def recording_step(self, states, targets, values, idx=None, batch=None, stream=None):
        out = real_step(self, states, targets, values, idx=idx, batch=batch, stream=stream)
        if rec_steps["trainer"] is None:
            rec_steps.update(trainer=id(self), arrays=(states, targets, values))
        if rec_steps["trainer"] == id(self) and len(rec_steps["idx"]) < 3:
            rec_steps["idx"].append(idx.clone())
            rec_steps["losses"].append(self.losses())
            rec_steps["amp"].append(self.amp_state())
            if len(rec_steps["idx"]) == 3:
                rec_steps["params"] = self.params().clone()
        return out
    monkeypatch.setattr(TM.Trainer, "step", recording_step)

    sizes = []
    train = nn.train

    def counting_train(examples, verbose=True):
        from yacht_amd.replay import as_device_examples
        sizes.append(int(as_device_examples(examples)[1].numel()))
        return train(examples, verbose)
    nn.train = counting_train
    monkeypatch.setattr(CM, "SelfPlayEngine", RecordingEngine)
    real_gate = AM.GatingArena
    monkeypatch.setattr(AM, "GatingArena", RecordingGate)
    c.learn()
    monkeypatch.undo()

    # ---- the two iterations ran at the shape, and the history pooled (Coach.py:86-111)
    assert len(plays) == 2 and len(gates) == 2
    assert len(c.trainExamplesHistory) == 2 and all(len(x) == MAXLEN for x in c.trainExamplesHistory)
    tr = c.nnet._trainer()
    assert tr.amp and tr.amp_state()["steps"] > 0
    assert sizes == [MAXLEN, 2 * MAXLEN]  # iteration 2 trains on both history entries
    for f in ("checkpoint_0.pth.tar.examples.npz", "checkpoint_1.pth.tar.examples.npz", "temp.pth.tar"):
        assert os.path.exists(os.path.join(d, f)), f

    # ---- self-play: sampled games bit for bit through the oracle; the recorded priors
    for play in plays:
        assert play["rec"]["n_moves"].min() == 48
        _replay_sampled_games(play)
    assert check_recorded_priors(plays[0]["pi"], plays[0]["v"], plays[0]["cnt"], plays[0]["leaves"],
                                 plays[0]["sd"], every=16, net=YkNet(plays[0]["sd"], 256, 6)) > 3000

    # ---- the pooled examples, per iteration, against the host restatement of its image
    for k in range(2):
        _same_as_host(c.trainExamplesHistory[k], plays[k]["img"])

    # ---- the Coach's first 3 amp steps: a standalone twin reproduces them bit for bit, and they
    # are held against torch autocast + GradScaler on the same minibatches and dropout masks
    assert len(rec_steps["idx"]) == 3 and all(len(i) == args.batch_size for i in rec_steps["idx"])
    S_all, T_all, V_all = rec_steps["arrays"]
    B, P_DROP = args.batch_size, float(args.dropout)
    twin = Trainer(sd0, 256, 6, lr=2e-3, weight_decay=1e-4, max_batch=B, vloss_weight=1.5, dropout=P_DROP,
                   seed=int(args.seed), amp=True)
    for k in range(3):
        twin.step(S_all, T_all, V_all, idx=rec_steps["idx"][k])
        assert np.array_equal(twin.losses()[:2], rec_steps["losses"][k][:2]), k
        assert twin.amp_state() == rec_steps["amp"][k], k
    assert torch.equal(twin.params().view(torch.int32), rec_steps["params"].view(torch.int32))
    params = {k: v.numpy() for k, v in twin.state_dict().items()}  # = the Coach's, bit for bit (above)
    twin.close()
    idx = torch.cat(rec_steps["idx"]).long()
    S = S_all[idx].contiguous()
    X = K.featurize(S)
    tg = T_all[idx].contiguous()
    vv = V_all[idx].contiguous()
    # the trainer's keep masks of dropout step k (a fresh trainer: steps 0, 1, 2; rows = the
    # minibatch rows), layer 0 = inp, 1 + b = block b
    masks = [[torch.tensor(dropout_keep_np(int(args.seed), L, k, B, 256, P_DROP), device="cuda") for L in range(7)]
             for k in range(3)]
    torch.backends.cuda.matmul.allow_tf32 = False
    p_amp, l_amp, g_amp, scale_amp = _torch_train_steps(sd0, 256, 6, X, tg, vv, B, 3, True, masks=masks, p=P_DROP)
    p_f32, l_f32, g_f32, _ = _torch_train_steps(sd0, 256, 6, X, tg, vv, B, 3, False, masks=masks, p=P_DROP)
    # step-1 gradients of the Coach's trainer = a backward at dropout step 0 on minibatch 0
    gtr = Trainer(sd0, 256, 6, lr=2e-3, weight_decay=1e-4, max_batch=B, vloss_weight=1.5, dropout=P_DROP,
                  seed=int(args.seed), amp=True)
    gtr.backward(S_all, T_all, V_all, idx=rec_steps["idx"][0])
    sc = gtr.amp_state()["scale"]
    g1 = {n: v.numpy() / sc for n, v in gtr.gradients().items()}
    gtr.close()
    ours_l = [(l[0] / B, l[1] / B) for l in rec_steps["losses"]]
    tol = lambda gap, ref: 1.5 * gap + 1e-4 * abs(ref) + 1e-7
    for k in range(3):
        for j in range(2):
            assert abs(ours_l[k][j] - l_amp[k][j]) <= tol(abs(l_f32[k][j] - l_amp[k][j]), l_amp[k][j]), (k, j)
    for name in g_amp:
        assert _relnorm(g1[name], g_amp[name]) <= 1.5 * _relnorm(g_f32[name], g_amp[name]) + 2e-3, name
    for name in p_amp:
        p0 = sd0[name].numpy()
        d_ours = _relnorm(params[name] - p0, p_amp[name] - p0)
        assert d_ours <= 1.5 * _relnorm(p_f32[name] - p0, p_amp[name] - p0) + 2e-2, name
    assert rec_steps["amp"][2]["scale"] == scale_amp

    # ---- the gates: a fresh unsharded GatingArena on the same nets and env ids, same tally
    for gt in gates:
        pw, nw = NNetWrapper(game, args), NNetWrapper(game, args)
        pw.nnet.load_state_dict(gt["p"])
        nw.nnet.load_state_dict(gt["n"])
        assert tuple(real_gate(game, pw, nw, args).playGames(gt["num"], env_base=gt["env_base"])) == tuple(gt["tally"])
        assert sum(gt["tally"]) == 10
