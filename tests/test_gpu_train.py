"""GPU parity of the native trainer (NNetWrapper.train, NNet.py:118-174).

* against the REFERENCE's own train() (tests/golden/train_h64_b1.npz: one AdamW step on one
  batch, dropout 0, CPU float32);
* against a plain torch fp32 step of the same architecture at hidden 256 x 6 blocks, over three
  steps: losses, clipped gradients, parameters and both Adam moments;
* dropout determinism, the NNetWrapper train / checkpoint round trip, and DDP gradient
  averaging (2 processes, gloo) equal to one process on the union of the shards.
Tolerances: f32 reductions in a different order (rocBLAS / torch CPU), amplified on the first
Adam step only where |grad| ~ eps; stated per test."""
import os

import numpy as np
import pytest

from oracle import spec

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def T():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from yacht_amd import kernels as K
    from yacht_amd import nnet, train
    return K, nnet, train


def _sd(hidden, nblocks):
    return {k: torch.tensor(np.asarray(v, dtype=np.float32)) for k, v in spec.closed_form_weights(hidden, nblocks).items()}


def _relnorm(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def _dense_targets(pidx, pval):
    n = len(pidx)
    pi = np.zeros((n, 3226), dtype=np.float32)
    for i in range(n):
        pi[i, pidx[i]] = pval[i]
    return np.argmax(pi, axis=1).astype(np.int32)


def test_one_step_matches_reference_train(T, golden):
    K, N, TR = T
    g = golden("train_h64_b1.npz")
    H, NB = int(g["hidden"]), int(g["nblocks"])
    n = len(g["values"])
    tr = TR.Trainer(_sd(H, NB), H, NB, lr=2e-3, weight_decay=1e-4, max_batch=n, vloss_weight=1.5, dropout=0.0)
    S = K.states_to_device(g["states"])
    t = torch.tensor(_dense_targets(g["pidx"], g["pval"]), device="cuda")
    v = torch.tensor(g["values"], device="cuda")
    tr.step(S, t, v)
    after = tr.state_dict()
    # the first AdamW step moves each weight by lr * g / (|g| + eps) ~ +-2e-3; f32 reductions in
    # another order (rocBLAS vs torch CPU) shift g slightly, which matters only where |g| ~ eps:
    # 1e-5 = 0.5 % of one step
    for k, ref in after.items():
        np.testing.assert_allclose(ref.numpy(), g["after/" + k], rtol=1e-4, atol=1e-5, err_msg=k)


def _torch_step_reference(model, opt, x, t, v, vw=1.5):
    import torch.nn.functional as F
    opt.zero_grad(set_to_none=True)
    out_pi, out_v = model(x)
    lp = F.cross_entropy(out_pi, t.long())
    lv = F.mse_loss(out_v, v.reshape(-1, 1))
    loss = lp + vw * lv
    loss.backward()
    torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=5.0)
    opt.step()
    return float(lp), float(lv)


def test_three_steps_vs_torch_fp32(T, golden):
    K, N, TR = T
    H, NB, B = 256, 6, 128
    torch.manual_seed(3)
    model = N.YachtNNet(hidden=H, nblocks=NB, dropout=0.0).cuda().float().train()
    with torch.no_grad():
        for m in model.modules():
            if isinstance(m, torch.nn.LayerNorm):
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.2, 0.2)
    sd0 = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    opt = torch.optim.AdamW(model.parameters(), lr=2e-3, weight_decay=1e-4)
    tr = TR.Trainer(sd0, H, NB, lr=2e-3, weight_decay=1e-4, max_batch=B, vloss_weight=1.5, dropout=0.0)
    W = golden("states.npz")["states"]
    rng = np.random.RandomState(0)
    torch.backends.cuda.matmul.allow_tf32 = False
    S = K.states_to_device(W[:3 * B])
    X = K.featurize(S)
    tg = torch.tensor(rng.randint(0, 3226, 3 * B), dtype=torch.int32, device="cuda")
    vv = torch.tensor(rng.rand(3 * B) * 2 - 1, dtype=torch.float32, device="cuda")
    tr.epoch_loss_begin(1.5)
    total = 0.0
    for k in range(3):
        sl = slice(k * B, (k + 1) * B)
        idx = torch.arange(k * B, (k + 1) * B, dtype=torch.int32, device="cuda")
        tr.step(S, tg, vv, idx=idx)
        lp, lv = _torch_step_reference(model, opt, X[sl], tg[sl], vv[sl])
        ce, se, _ = tr.losses()
        assert abs(ce / B - lp) <= 1e-5 * abs(lp) + 1e-6 and abs(se / B - lv) <= 1e-5 * abs(lv) + 1e-6
        total += ce / B + 1.5 * se / B
    # the device-side report-epoch sum (NNetWrapper.train's "Avg Loss") is the host sum, bit for bit
    assert tr.epoch_loss_end() == (total, 3)
    # gradients and moments: per-tensor relative error (f32 reductions in another order through
    # 13 layers); parameters: the update p - p0 agrees to 0.1 % in norm, and at most 1e-4 of the
    # weights are off by more than 0.5 % of one AdamW step (1e-5): Adam normalises each element,
    # so a gradient near eps whose rounding differs can move its weight by up to 2 lr
    grads = tr.gradients()  # clipped, of the last step
    params = tr.state_dict()
    m, v2 = tr.moments()
    for name, p in model.named_parameters():
        assert _relnorm(grads[name].numpy(), p.grad.detach().cpu().numpy()) < 1e-4, "grad " + name
        p_ref = p.detach().cpu().numpy()
        assert _relnorm(params[name].numpy() - sd0[name].numpy(), p_ref - sd0[name].numpy()) < 1e-3, "update " + name
        assert (np.abs(params[name].numpy() - p_ref) > 1e-5).mean() <= 1e-4, "param " + name
        st = opt.state[p]
        assert _relnorm(m[name].numpy(), st["exp_avg"].cpu().numpy()) < 1e-4, "exp_avg " + name
        assert _relnorm(v2[name].numpy(), st["exp_avg_sq"].cpu().numpy()) < 2e-4, "exp_avg_sq " + name
    assert tr.step_count == 3


def test_dropout_masks_are_deterministic_and_active(T, golden):
    K, N, TR = T
    H, NB, B = 64, 2, 64
    sd = _sd(H, NB)
    W = golden("states.npz")["states"][:B]
    S = K.states_to_device(W)
    tg = torch.zeros(B, dtype=torch.int32, device="cuda")
    vv = torch.zeros(B, dtype=torch.float32, device="cuda")
    res = []
    for p, seed in ((0.3, 7), (0.3, 7), (0.3, 8), (0.0, 7)):
        tr = TR.Trainer(sd, H, NB, max_batch=B, dropout=p, seed=seed)
        tr.backward(S, tg, vv)
        res.append(tr.gradients()["inp.0.weight"].numpy())
    assert np.array_equal(res[0], res[1])
    assert not np.allclose(res[0], res[2]) and not np.allclose(res[0], res[3])


@pytest.mark.parametrize("amp", [False, True])
def test_nnetwrapper_train_and_checkpoint(T, tmp_path, amp):
    """NNetWrapper.train + save/load_checkpoint (NNet.py:118-213) in both modes: the float32 step
    and the default under args.cuda, autocast + GradScaler (the AMP path through the
    wrapper and its checkpoint round trip).  AMP counts the steps GradScaler did not skip."""
    K, N, TR = T
    from yacht_amd.coach import Coach
    from yacht_amd.game import YachtGame
    from yacht_amd.nnet import HashPriorNet, NNetWrapper
    from yacht_amd.utils import dotdict
    game = YachtGame(seed=1, env_id=0)
    coach = Coach(game, HashPriorNet(game), dotdict(numMCTSSims=4, cpuct=1.5, tempThreshold=15))
    examples = [ex for ep in coach.executeEpisodes(4) for ex in ep]
    args = dotdict(lr=2e-3, weight_decay=1e-4, epochs=2, batch_size=64, vloss_weight=1.5, cuda=True, hidden=64,
                   nblocks=1, dropout=0.3)
    # args.cuda selects the reference's GPU arithmetic (autocast + GradScaler, NNet.py:113-116),
    # args.amp False the float32 step
    assert NNetWrapper(game, args).uses_amp() and not NNetWrapper(game, dotdict(args, cuda=False)).uses_amp()
    args = dotdict(args, amp=amp)
    w = NNetWrapper(game, args)
    assert w._trainer().amp == amp
    pi0, _ = w.predict(examples[0][0])
    w.train(examples, verbose=False)
    pi1, v1 = w.predict(examples[0][0])
    assert not np.allclose(pi0, pi1)
    steps = -(-len(examples) // 64) * 2
    if amp:  # a GradScaler skip leaves AdamW's count alone (torch's scaler.step)
        st = w._trainer().amp_state()
        assert 1 <= st["steps"] <= steps and st["steps"] == w._trainer().step_count
        steps = st["steps"]
    assert w._trainer().step_count == steps
    w.save_checkpoint(str(tmp_path), "best.pth.tar")
    ck = torch.load(os.path.join(tmp_path, "best.pth.tar"), map_location="cpu", weights_only=True)
    assert set(ck) == {"state_dict", "optimizer", "args"} and len(ck["optimizer"]["state"]) == len(ck["state_dict"])
    w2 = NNetWrapper(game, args)
    w2.load_checkpoint(str(tmp_path), "best.pth.tar", load_optimizer=True)
    pi2, v2 = w2.predict(examples[0][0])
    assert np.array_equal(pi1, pi2) and v1 == v2
    m1, s1 = w._trainer().moments()
    m2, s2 = w2._trainer().moments()
    assert all(torch.equal(m1[k], m2[k]) and torch.equal(s1[k], s2[k]) for k in m1)
    assert w2._trainer().step_count == steps


def _ddp_worker(rank, world, port, H, NB, B, W, tg, vv, out, dropout=0.0):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "nypc-yacht-auction_amd"))
    from yacht_amd import kernels as K
    from yacht_amd.dist import allreduce_grads
    from yacht_amd.train import Trainer
    tr = Trainer(_sd(H, NB), H, NB, max_batch=B, dropout=dropout, seed=5)
    sl = slice(rank * B, (rank + 1) * B)
    S = K.states_to_device(W[sl])
    tr.backward(S, torch.tensor(tg[sl], device="cuda"), torch.tensor(vv[sl], device="cuda"), row0=rank * B)
    allreduce_grads(tr)
    out["g%d" % rank] = tr.grads().cpu().numpy().copy()
    tr.apply()
    out["p%d" % rank] = tr.params().cpu().numpy().copy()
    dist.destroy_process_group()


@pytest.mark.parametrize("dropout", [0.0, 0.3])
def test_ddp_gradient_average_equals_union_batch(T, golden, dropout):
    """With dropout on, each rank draws the masks of its rows of the whole minibatch (row offset =
    the rank's start), so the averaged gradient is still the single-process one."""
    import torch.multiprocessing as mp
    K, N, TR = T
    H, NB, B = 64, 1, 32
    W = golden("states.npz")["states"][:2 * B]
    rng = np.random.RandomState(1)
    tg = rng.randint(0, 3226, 2 * B).astype(np.int32)
    vv = (rng.rand(2 * B) * 2 - 1).astype(np.float32)
    mgr = mp.get_context("spawn").Manager()
    out = mgr.dict()
    mp.start_processes(_ddp_worker, args=(2, 29577 + int(dropout * 10), H, NB, B, W, tg, vv, out, dropout), nprocs=2,
                       start_method="spawn")
    ref = TR.Trainer(_sd(H, NB), H, NB, max_batch=2 * B, dropout=dropout, seed=5)
    ref.backward(K.states_to_device(W), torch.tensor(tg, device="cuda"), torch.tensor(vv, device="cuda"))
    single = ref.grads().cpu().numpy()
    # every rank steps on the same averaged gradient, equal to the union batch's gradient up to
    # f32 summation order
    assert np.array_equal(out["g0"], out["g1"]) and np.array_equal(out["p0"], out["p1"])
    assert _relnorm(out["g0"], single) < 1e-5


def test_coach_learn_iteration_and_resume(T, tmp_path):
    """Coach.learn (Coach.py:74-139) end to end: batched self-play, examples files, train, the
    previous-vs-new arena with two MCTS plugins, accept/reject; then loadTrainExamples resumes."""
    from yacht_amd.coach import Coach
    from yacht_amd.game import YachtGame
    from yacht_amd.nnet import NNetWrapper
    from yacht_amd.utils import dotdict
    d = str(tmp_path)
    args = dotdict(numIters=1, numEps=8, tempThreshold=15, updateThreshold=0.55, maxlenOfQueue=200000,
                   numMCTSSims=4, arenaCompare=2, cpuct=1.5, checkpoint=d, load_folder_file=(d, "checkpoint_0.pth.tar"),
                   numItersForTrainExamplesHistory=5, lr=2e-3, weight_decay=1e-4, epochs=1, batch_size=64,
                   vloss_weight=1.5, cuda=True, hidden=64, nblocks=1, dropout=0.3, examples_format="both")
    game = YachtGame(seed=3, env_id=0)
    c = Coach(game, NNetWrapper(game, args), args)
    c.learn()
    assert sum(c.last_pit) == 2
    for f in ("temp.pth.tar", "checkpoint_0.pth.tar.examples", "checkpoint_0.pth.tar.examples.npz"):
        assert os.path.exists(os.path.join(d, f)), f
    assert len(c.trainExamplesHistory) == 1 and len(c.trainExamplesHistory[0]) == 8 * 48
    c2 = Coach(game, NNetWrapper(game, args), args)
    c2.loadTrainExamples()
    assert c2.skipFirstSelfPlay and len(c2.trainExamplesHistory[0]) == 8 * 48
    os.remove(os.path.join(d, "checkpoint_0.pth.tar.examples.npz"))  # the reference-format file alone
    c3 = Coach(game, NNetWrapper(game, args), args)
    c3.loadTrainExamples()
    a, b = c2.trainExamplesHistory[0][5], c3.trainExamplesHistory[0][5]
    assert a[0] == b[0] and a[1] == b[1] and a[2] == b[2]


@pytest.mark.parametrize("amp", [False, True])
@pytest.mark.parametrize("B", [64, 63])
def test_dropout_rows_split_over_calls_equal_the_whole_batch(T, golden, amp, B):
    """Two backwards of part of a minibatch each (row offsets 0 and B//2, gradients weighted by
    their shares) take the whole minibatch's dropout masks: the gradient equals one backward over
    all B rows.  An odd B leaves a row alone in its wave in one call but not in the other, which is
    where a mask cache shared across layers would hand a row the previous layer's mask."""
    K, N, TR = T
    H, NB = 64, 2
    W = golden("states.npz")["states"][:B]
    rng = np.random.RandomState(2)
    S = K.states_to_device(W)
    tg = torch.tensor(rng.randint(0, 3226, B), dtype=torch.int32, device="cuda")
    vv = torch.tensor(rng.rand(B) * 2 - 1, dtype=torch.float32, device="cuda")
    # (amp: a small loss scale - 65536 / 32 rows would overflow fp16 gradients, a step GradScaler skips)
    kw = dict(max_batch=B, dropout=0.3, seed=9, amp=amp, init_scale=256.0)
    whole = TR.Trainer(_sd(H, NB), H, NB, **kw)
    whole.backward(S, tg, vv)
    g_whole = whole.grads().cpu().numpy().copy()
    half = TR.Trainer(_sd(H, NB), H, NB, **kw)
    acc = 0
    cuts = (0, B // 2, B)
    for k in range(2):
        idx = torch.arange(cuts[k], cuts[k + 1], dtype=torch.int32, device="cuda")
        half.backward(S, tg, vv, idx=idx, row0=cuts[k])
        acc = acc + (cuts[k + 1] - cuts[k]) / B * half.grads().cpu().numpy().astype(np.float64)
    # f32 (or fp16-rounded, amp) sums in another grouping
    assert _relnorm(acc, g_whole) < (2e-3 if amp else 1e-4)  # wrong masks would be O(1) off
    other = TR.Trainer(_sd(H, NB), H, NB, **kw)
    other.backward(S, tg, vv, idx=torch.arange(B // 2, B, dtype=torch.int32, device="cuda"), row0=0)
    g_wrong = other.grads().cpu().numpy()
    half.backward(S, tg, vv, idx=torch.arange(B // 2, B, dtype=torch.int32, device="cuda"), row0=B // 2)
    assert not np.allclose(g_wrong, half.grads().cpu().numpy())  # the offset selects other masks


class _FixedDropout(torch.nn.Module):
    """nn.Dropout with given keep masks: x * keep * 1/(1-p), as torch's dropout kernel scales."""

    def __init__(self, p):
        super().__init__()
        self.scale, self.keep = 1.0 / (1.0 - p), None

    def forward(self, x):
        return x * (self.keep.to(x.dtype) * self.scale)


def _torch_train_steps(sd0, H, NB, X, tg, vv, B, steps, amp, vw=1.5, masks=None, p=0.0):
    """The reference's train() inner loop (NNet.py:132-165) on the GPU: autocast('cuda') +
    GradScaler('cuda') (amp) or float32, AdamW(2e-3, 1e-4), clip 5.0; dropout 0, or - masks[k][L]
    given - the nn.Dropout layers (L = 0: inp, 1 + b: block b) applying those keep masks at step k."""
    import torch.nn.functional as F
    from yacht_amd.nnet import YachtNNet
    model = YachtNNet(hidden=H, nblocks=NB, dropout=0.0).cuda().float()
    model.load_state_dict(sd0)
    drops = None
    if masks is not None:
        drops = [_FixedDropout(p) for _ in range(1 + NB)]
        model.inp[3] = drops[0]
        for b, blk in enumerate(model.blocks):
            blk.dropout = drops[1 + b]
    model.train()
    opt = torch.optim.AdamW(model.parameters(), lr=2e-3, weight_decay=1e-4)
    scaler = torch.amp.GradScaler("cuda") if amp else None
    losses, grads1 = [], None
    for k in range(steps):
        sl = slice(k * B, (k + 1) * B)
        if drops is not None:
            for L, d in enumerate(drops):
                d.keep = masks[k][L]
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", enabled=amp):
            out_pi, out_v = model(X[sl])
            lp = F.cross_entropy(out_pi, tg[sl].long())
            lv = F.mse_loss(out_v, vv[sl].reshape(-1, 1))
            loss = lp + vw * lv
        if amp:
            scaler.scale(loss).backward()
            scaler.unscale_(opt)
        else:
            loss.backward()
        if k == 0:
            grads1 = {n: p.grad.detach().float().cpu().numpy().copy() for n, p in model.named_parameters()}
        torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=5.0)
        if amp:
            scaler.step(opt)
            scaler.update()
        else:
            opt.step()
        losses.append((float(lp), float(lv)))
    params = {n: p.detach().cpu().numpy().copy() for n, p in model.named_parameters()}
    return params, losses, grads1, (scaler.get_scale() if amp else None)


@pytest.mark.parametrize("H,NB,B", [(256, 6, 512), (64, 1, 128)])
def test_amp_steps_vs_torch_autocast_gradscaler(T, golden, H, NB, B):
    """The mixed-precision mode against the reference's own GPU train step: torch autocast('cuda')
    + GradScaler('cuda') (NNet.py:141-155) on the same weights and minibatches, 3 steps.
    Stated tolerance, per quantity: the amp trainer may be no further from torch-AMP than torch's
    float32 step is (the gap the fp16 rounding itself opens), x1.5 plus a floor: losses (each
    step), step-1 gradients (per tensor, unscaled, before the clip), parameters after 3 steps
    (the update p - p0 per tensor).  And the GradScaler state (scale, steps taken) is torch's."""
    K, N, TR = T
    torch.manual_seed(11)
    model = N.YachtNNet(hidden=H, nblocks=NB, dropout=0.0)
    with torch.no_grad():
        for m in model.modules():
            if isinstance(m, torch.nn.LayerNorm):
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.2, 0.2)
    sd0 = {k: v.detach().clone() for k, v in model.state_dict().items()}
    W = golden("states.npz")["states"]
    W = np.concatenate([W] * (3 * B // len(W) + 1))[:3 * B]
    rng = np.random.RandomState(4)
    S = K.states_to_device(W)
    X = K.featurize(S)
    tg = torch.tensor(rng.randint(0, 3226, 3 * B), dtype=torch.int32, device="cuda")
    vv = torch.tensor(rng.rand(3 * B) * 2 - 1, dtype=torch.float32, device="cuda")
    torch.backends.cuda.matmul.allow_tf32 = False
    p_amp, l_amp, g_amp, scale_amp = _torch_train_steps(sd0, H, NB, X, tg, vv, B, 3, True)
    p_f32, l_f32, g_f32, _ = _torch_train_steps(sd0, H, NB, X, tg, vv, B, 3, False)
    tr = TR.Trainer(sd0, H, NB, lr=2e-3, weight_decay=1e-4, max_batch=B, vloss_weight=1.5, dropout=0.0, amp=True)
    ours_l = []
    g1 = None
    for k in range(3):
        idx = torch.arange(k * B, (k + 1) * B, dtype=torch.int32, device="cuda")
        tr.backward(S, tg, vv, idx=idx)
        if k == 0:
            scale = tr.amp_state()["scale"]
            g1 = {n: v.numpy() / scale for n, v in tr.gradients().items()}
        tr.apply()
        ce, se, _ = tr.losses()
        ours_l.append((ce / B, se / B))
    tol = lambda ref_gap, ref: 1.5 * ref_gap + 1e-4 * abs(ref) + 1e-7
    for k in range(3):
        for j in range(2):
            gap = abs(l_f32[k][j] - l_amp[k][j])
            print(f"step {k} loss[{j}]: ours {ours_l[k][j]:.7f} torch-amp {l_amp[k][j]:.7f} torch-f32 {l_f32[k][j]:.7f}")
            assert abs(ours_l[k][j] - l_amp[k][j]) <= tol(gap, l_amp[k][j]), (k, j)
    worst = []
    for name in g_amp:
        d_ours = _relnorm(g1[name], g_amp[name])
        d_f32 = _relnorm(g_f32[name], g_amp[name])
        worst.append((d_ours / max(d_f32, 1e-12), name, d_ours, d_f32))
        assert d_ours <= 1.5 * d_f32 + 2e-3, ("grad", name, d_ours, d_f32)
    print("worst grad ratios:", sorted(worst)[-3:])
    params = tr.state_dict()
    for name in p_amp:
        p0 = sd0[name].numpy()
        d_ours = _relnorm(params[name].numpy() - p0, p_amp[name] - p0)
        d_f32 = _relnorm(p_f32[name] - p0, p_amp[name] - p0)
        assert d_ours <= 1.5 * d_f32 + 2e-2, ("update", name, d_ours, d_f32)
    st = tr.amp_state()
    assert st["scale"] == scale_amp and tr.step_count == st["steps"]


def test_amp_skipped_step_gradients_as_torch_leaves_them(T, golden):
    """A step GradScaler skips (the scaled fp16 gradients overflow) leaves the parameters alone, and
    the gradient buffer as torch leaves p.grad: unscale_, then clip_grad_norm_'s
    multiply by min(1, 5 / (norm + 1e-6)) - 0 for an infinite norm, so finite entries become 0
    and infinite ones nan; all nan for a nan norm."""
    K, N, TR = T
    H, NB, B = 64, 1, 32
    W = golden("states.npz")["states"][:B]
    rng = np.random.RandomState(6)
    S = K.states_to_device(W)
    tg = torch.tensor(rng.randint(0, 3226, B), dtype=torch.int32, device="cuda")
    vv = torch.tensor(rng.rand(B) * 2 - 1, dtype=torch.float32, device="cuda")
    tr = TR.Trainer(_sd(H, NB), H, NB, max_batch=B, dropout=0.0, amp=True, init_scale=2.0 ** 40)
    p0 = tr.params().cpu().numpy().copy()
    tr.backward(S, tg, vv)
    g_scaled = tr.grads().cpu().numpy().copy()
    assert not np.isfinite(g_scaled).all()
    tr.apply()
    st = tr.amp_state()
    assert st["found_inf"] and st["steps"] == 0 and st["scale"] == 2.0 ** 39
    assert np.array_equal(tr.params().cpu().numpy(), p0)
    u = g_scaled * np.float32(2.0 ** -40)
    total = float(np.sum(u.astype(np.float64) ** 2))
    assert not np.isfinite(total)
    with np.errstate(invalid="ignore"):
        want = u * np.float32(0.0) if np.isinf(total) else np.full_like(u, np.nan)
    got = tr.grads().cpu().numpy()
    np.testing.assert_array_equal(got, want)
    assert np.isnan(got).any() and (np.isnan(total) or (got == 0).any())


@pytest.mark.parametrize("H,NB,B,scale", [(256, 6, 512, None), (64, 1, 32, 2.0 ** 40)])
def test_amp_fused_norm_step_equals_backward_then_apply(T, golden, H, NB, B, scale):
    """yk_trainer_step (one call) sums the gradient norm inside the gradient launches instead of
    re-reading G; backward() + apply() (the DDP split, an all-reduce may sit between) re-reads it.
    Same grad sq-norm (double sums in another order: rel 1e-12), same GradScaler state and the same
    parameters (the clip coefficient may move by an ulp: rtol 1e-6) over 3 steps, and an overflowing
    step (scale 2^40) is skipped the same way."""
    K, N, TR = T
    W = golden("states.npz")["states"]
    W = np.concatenate([W] * (3 * B // len(W) + 1))[:3 * B]
    rng = np.random.RandomState(9)
    S = K.states_to_device(W)
    tg = torch.tensor(rng.randint(0, 3226, 3 * B), dtype=torch.int32, device="cuda")
    vv = torch.tensor(rng.rand(3 * B) * 2 - 1, dtype=torch.float32, device="cuda")
    kw = dict(max_batch=B, dropout=0.1, amp=True)
    if scale:
        kw["init_scale"] = scale
    fused = TR.Trainer(_sd(H, NB), H, NB, **kw)
    split = TR.Trainer(_sd(H, NB), H, NB, **kw)
    for k in range(3):
        idx = torch.arange(k * B, (k + 1) * B, dtype=torch.int32, device="cuda")
        fused.step(S, tg, vv, idx=idx)
        split.backward(S, tg, vv, idx=idx)
        split.apply()
        lf, ls = fused.losses(), split.losses()
        assert lf[0] == ls[0] and lf[1] == ls[1], k
        if np.isfinite(ls[2]):
            assert abs(lf[2] - ls[2]) <= 1e-12 * ls[2], (k, lf[2], ls[2])
        else:
            assert not np.isfinite(lf[2]), k
        assert fused.amp_state() == split.amp_state(), k
        np.testing.assert_allclose(fused.params().cpu().numpy(), split.params().cpu().numpy(), rtol=1e-6, atol=1e-9)
    if scale:
        assert fused.amp_state()["steps"] < 3


@pytest.mark.parametrize("H,NB,B", [(64, 2, 64), (256, 6, 512)])
def test_amp_update_made_masks_equal_k_amp_masks(T, golden, H, NB, B):
    """Every AMP step after the first reads dropout keep bits that the previous step's k_amp_update
    made ahead (row offset 0).  Trainer A: step() then backward() at dropout step 1 (the update-made
    bits).  Trainer B: A's parameters and step count 1 through yk_trainer_set, so its backward makes
    the bits with k_amp_masks.  Same gradients bit for bit, and both differ from dropout step 0's
    masks."""
    K, N, TR = T
    W = golden("states.npz")["states"]
    W = np.concatenate([W] * (2 * B // len(W) + 1))[:2 * B]
    rng = np.random.RandomState(12)
    S = K.states_to_device(W)
    tg = torch.tensor(rng.randint(0, 3226, 2 * B), dtype=torch.int32, device="cuda")
    vv = torch.tensor(rng.rand(2 * B) * 2 - 1, dtype=torch.float32, device="cuda")
    i0 = torch.arange(0, B, dtype=torch.int32, device="cuda")
    i1 = torch.arange(B, 2 * B, dtype=torch.int32, device="cuda")
    kw = dict(max_batch=B, dropout=0.3, seed=13, amp=True, init_scale=256.0)  # (no skipped step)
    a = TR.Trainer(_sd(H, NB), H, NB, **kw)
    a.step(S, tg, vv, idx=i0)
    assert a.amp_state()["steps"] == 1
    a.backward(S, tg, vv, idx=i1)
    ga = a.grads().clone()
    b = TR.Trainer(_sd(H, NB), H, NB, **kw)
    b.load_params(a.state_dict())
    m, v = a.moments()
    b.set_moments(m, v, 1)
    b.backward(S, tg, vv, idx=i1)
    assert torch.equal(ga.view(torch.int32), b.grads().view(torch.int32))
    c = TR.Trainer(_sd(H, NB), H, NB, **kw)  # the same parameters at dropout step 0: other masks
    c.load_params(a.state_dict())
    c.backward(S, tg, vv, idx=i1)
    assert not torch.equal(ga, c.grads())
    for t in (a, b, c):
        t.close()
