"""GPU parity of NNetWrapper.predict (f32 MFMA): within 1e-5 of the reference's own torch
float32 CPU outputs (tests/golden) and of a plain torch fp32 forward on the same weights."""
import numpy as np
import pytest

from oracle import oracle as O
from oracle import spec

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

RTOL_PI, ATOL_PI, ATOL_V = 1e-5, 1e-7, 1e-5  # north-star tolerance on policy/value


@pytest.fixture(scope="module")
def mods():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from yacht_amd import kernels, nnet
    return kernels, nnet


@pytest.mark.parametrize("hidden,nblocks", [(256, 6), (64, 1)])
def test_predict_vs_reference(mods, golden, hidden, nblocks):
    K, N = mods
    g = golden(f"predict_h{hidden}_b{nblocks}.npz")
    net = N.YkNet(spec.closed_form_weights(hidden, nblocks), hidden, nblocks)
    pi, v = net.predict_states(K.states_to_device(g["states"]))
    np.testing.assert_allclose(pi.cpu().numpy(), g["pi"], rtol=RTOL_PI, atol=ATOL_PI)
    np.testing.assert_allclose(v.cpu().numpy(), g["v"], rtol=0, atol=ATOL_V)
    pi2, v2 = net.predict_features(torch.from_numpy(g["x"]))
    assert torch.equal(pi, pi2) and torch.equal(v, v2)


@pytest.mark.parametrize("hidden,nblocks", [(256, 6), (128, 2), (512, 1)])
def test_predict_vs_torch_fp32(mods, golden, hidden, nblocks):
    K, N = mods
    torch.manual_seed(hidden + nblocks)
    model = N.YachtNNet(hidden=hidden, nblocks=nblocks).eval()
    with torch.no_grad():  # non-trivial LayerNorm affines
        for m in model.modules():
            if isinstance(m, torch.nn.LayerNorm):
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.2, 0.2)
    net = N.YkNet(model.state_dict(), hidden, nblocks)
    W = golden("states.npz")["states"][:1000]
    S = K.states_to_device(W)
    pi, v = net.predict_states(S)
    m = model.to("cuda").float()
    with torch.no_grad():
        torch.backends.cuda.matmul.allow_tf32 = False
        logits, vr = m(K.featurize(S))
        pr = torch.nn.functional.log_softmax(logits, dim=1).exp()
    np.testing.assert_allclose(pi.cpu().numpy(), pr.cpu().numpy(), rtol=RTOL_PI, atol=ATOL_PI)
    np.testing.assert_allclose(v.cpu().numpy(), vr[:, 0].cpu().numpy(), rtol=0, atol=ATOL_V)


def test_predict_large_batch_vs_oracle(mods, golden):
    K, N = mods
    sd = spec.closed_form_weights(256, 6)
    net = N.YkNet(sd, 256, 6)
    W = golden("states.npz")["states"]
    W = np.concatenate([W] * (4096 // len(W) + 1))[:4099]  # > one 4096-game lock-step, ragged tail
    pi, v = net.predict_states(K.states_to_device(W))
    pick = np.r_[0:64, 4000:4099]
    opi, ov = O.Net(sd, 256, 6).predict_states(W[pick])
    np.testing.assert_allclose(pi.cpu().numpy()[pick], opi, rtol=RTOL_PI, atol=ATOL_PI)
    np.testing.assert_allclose(v.cpu().numpy()[pick], ov, rtol=0, atol=ATOL_V)
    assert torch.isfinite(pi).all() and torch.allclose(pi.sum(1), torch.ones(len(W), device="cuda"), atol=1e-4)


def _masked_renorm(pi, ok):
    p = np.where(ok, pi, 0.0).astype(np.float64)
    s = p.sum(1, keepdims=True)
    return np.divide(p, s, out=np.zeros_like(p), where=s > 0)


@pytest.mark.parametrize("hidden,nblocks", [(256, 6), (64, 1)])
def test_leaf_prior_is_the_renormalised_reference_policy(mods, golden, hidden, nblocks):
    """The engine's valid-only leaf prior (yk_net_leaf_prior, the softmax over the valid actions)
    renormalised == the masked, renormalised exp(log_softmax) of MCTS.py:86-91: within 1e-5 of the
    same renormalisation of the GPU's full predict pi (the same logits), and within 3e-5 of the
    reference's own (pi within 1e-5 per element, test_predict_vs_reference, and the renormalising
    sum within 1e-5 again)."""
    K, N = mods
    g = golden(f"predict_h{hidden}_b{nblocks}.npz")
    net = N.YkNet(spec.closed_form_weights(hidden, nblocks), hidden, nblocks)
    S = K.states_to_device(g["states"])
    pi, v = net.leaf_prior(S)
    full, _ = net.predict_states(S)
    ok, cnt = O.valid(g["states"], 1)
    ok = ok.astype(bool)
    pi = pi.cpu().numpy()
    assert not pi[~ok].any()
    P = _masked_renorm(pi, ok)
    np.testing.assert_allclose(P, _masked_renorm(full.cpu().numpy(), ok), rtol=RTOL_PI, atol=ATOL_PI)
    np.testing.assert_allclose(P, _masked_renorm(g["pi"], ok), rtol=3 * RTOL_PI, atol=ATOL_PI)
    np.testing.assert_allclose(v.cpu().numpy(), g["v"], rtol=0, atol=ATOL_V)
    assert (pi.sum(1) <= 1.0 + 1e-5).all()  # a softmax over a superset of the valid set


def test_leaf_prior_keeps_the_full_softmax_when_underflow_is_possible(mods, golden):
    """A bias spread past the bound: every row takes the full softmax, so the leaf prior is the
    predict pi at the valid actions (to the ulps between the expand's hardware exp and expf), and
    the reference's uniform fallback stays reachable exactly as in MCTS.py:93-107."""
    K, N = mods
    sd = spec.closed_form_weights(256, 6)
    b = np.asarray(sd["pi_head.2.bias"], dtype=np.float32).copy()
    b[202:] += 120.0  # score actions far above the bids
    sd = dict(sd)
    sd["pi_head.2.bias"] = b
    net = N.YkNet(sd, 256, 6)
    W = golden("states.npz")["states"][:512]
    S = K.states_to_device(W)
    lp, _ = net.leaf_prior(S)
    pp, _ = net.predict_states(S)
    ok = O.valid(W, 1)[0].astype(bool)
    lp, pp = lp.cpu().numpy(), pp.cpu().numpy()
    np.testing.assert_allclose(lp, np.where(ok, pp, 0.0).astype(np.float32), rtol=1e-6, atol=0)
    bid = ok[:, :202].any(1)
    assert bid.any() and (lp[bid].sum(1) < 1e-30).all()  # the bids underflow: uniform fallback


def _torch_model(N, hidden, nblocks, seed):
    torch.manual_seed(seed)
    model = N.YachtNNet(hidden=hidden, nblocks=nblocks).eval()
    with torch.no_grad():  # non-trivial LayerNorm affines
        for m in model.modules():
            if isinstance(m, torch.nn.LayerNorm):
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.2, 0.2)
    return model


def _torch_fp32(K, model, S):
    m = model.to("cuda").float()
    with torch.no_grad():
        torch.backends.cuda.matmul.allow_tf32 = False
        logits, vr = m(K.featurize(S))
        pr = torch.nn.functional.log_softmax(logits, dim=1).exp()
    return pr.cpu().numpy(), vr[:, 0].cpu().numpy()


@pytest.mark.parametrize("hidden", [256, 64])
def test_predict_no_residual_blocks(mods, golden, hidden):
    """nblocks = 0 (YachtNNet with an empty ModuleList: inp -> heads): the value head's v_head.2
    weights come from their own load, not from a last trunk GEMM's ring (there is none)."""
    K, N = mods
    model = _torch_model(N, hidden, 0, 7)
    net = N.YkNet(model.state_dict(), hidden, 0)
    S = K.states_to_device(golden("states.npz")["states"][:1000])
    pi, v = net.predict_states(S)
    lp, lv = net.leaf_prior(S)
    pr, vr = _torch_fp32(K, model, S)
    np.testing.assert_allclose(pi.cpu().numpy(), pr, rtol=RTOL_PI, atol=ATOL_PI)
    np.testing.assert_allclose(v.cpu().numpy(), vr, rtol=0, atol=ATOL_V)
    assert torch.equal(v, lv)
    assert net.errors() == 0


def test_split_range_guard(mods, golden):
    """yk_net_create refuses a finite weight the fp16 hi plane cannot hold (|w| >= 65520) with
    YK_ERR_RANGE, in every packed matrix; weights at +-6e4 (inside the range) still predict within
    1e-5 of torch fp32.  The mixed-precision trainer (fp16 weight casts) refuses the same."""
    K, N = mods
    from yacht_amd._lib import YK_ERR_RANGE, YkError
    from yacht_amd.train import Trainer
    model = _torch_model(N, 256, 6, 11)
    base = {k: t.detach().clone() for k, t in model.state_dict().items()}
    for name in ("inp.0.weight", "blocks.0.fc1.weight", "blocks.5.fc2.weight", "pi_head.2.weight",
                 "v_head.2.weight"):
        sd = {k: t.clone() for k, t in base.items()}
        sd[name][3, 7] = 1e5 if name != "blocks.5.fc2.weight" else -65520.0
        with pytest.raises(YkError) as e:
            N.YkNet(sd, 256, 6)
        assert e.value.code == YK_ERR_RANGE, name
        with pytest.raises(YkError) as e:
            Trainer(sd, 256, 6, max_batch=64, dropout=0.0, seed=0, amp=True)
        assert e.value.code == YK_ERR_RANGE, name
    # +-6e4 in the heads' products (well-conditioned there): within 1e-5 of torch fp32
    sd = {k: t.clone() for k, t in base.items()}
    sd["pi_head.2.weight"][3, 7] = 6e4
    sd["pi_head.2.weight"][100, 9] = -6e4
    sd["v_head.2.weight"][5, 9] = -6e4
    sd["inp.0.weight"][11, 2] = 65504.0
    model.load_state_dict(sd)
    net = N.YkNet(sd, 256, 6)
    W = golden("states.npz")["states"][:1000]
    S = K.states_to_device(W)
    pi, v = net.predict_states(S)
    pr, vr = _torch_fp32(K, model, S)
    np.testing.assert_allclose(pi.cpu().numpy(), pr, rtol=RTOL_PI, atol=ATOL_PI)
    np.testing.assert_allclose(v.cpu().numpy(), vr, rtol=0, atol=ATOL_V)
    assert net.errors() == 0
    # +-6e4 inside the trunk: one column of fc1 / fc2 dominates its LayerNorm, which then cancels
    # ~12 bits of every other column - ill-conditioned for any f32 arithmetic (torch fp32's own
    # pi is ~1e-3 off float64 there).  Checked against a float64 forward: no further from it than
    # torch fp32 x 4 (the split's operands carry 22 bits to float32's 24)
    from helpers import torch_predict
    sd = {k: t.clone() for k, t in base.items()}
    sd["blocks.0.fc1.weight"][3, 7] = 6e4
    sd["blocks.2.fc2.weight"][5, 9] = -6e4
    net = N.YkNet(sd, 256, 6)
    pi, v = net.predict_states(S)
    sdn = {k: t.numpy() for k, t in sd.items()}
    p64, v64 = torch_predict(sdn, 256, 6, W, torch.float64)
    p32, v32 = torch_predict(sdn, 256, 6, W, torch.float32)
    big = p64 > 1e-4
    e_gpu = float((np.abs(pi.cpu().numpy() - p64)[big] / p64[big]).max())
    e_t32 = float((np.abs(p32 - p64)[big] / p64[big]).max())
    ev_gpu, ev_t32 = float(np.abs(v.cpu().numpy() - v64).max()), float(np.abs(v32 - v64).max())
    print(f"trunk weights +-6e4: pi max rel err vs float64 {e_gpu:.2e} (torch fp32 {e_t32:.2e}), "
          f"v {ev_gpu:.2e} ({ev_t32:.2e})")
    assert e_gpu <= 4 * e_t32 and ev_gpu <= max(ATOL_V, 4 * ev_t32)
