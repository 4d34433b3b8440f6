"""The opt-in fp16 predict mode (YK_PREDICT_F16): the arithmetic of the reference's own GPU path,
NNetWrapper.predict under autocast('cuda') (yacht/NNet.py:186-189), against torch on the box.

Tolerance (stated): the mode must be at least as close to a float64 forward of the same weights
as torch's autocast('cuda') predict is - the reference's own CUDA numbers - on every output
(max |pi - pi64| and max |v - v64| over 1000 fixture states), and within twice that bound of the
autocast outputs themselves.  The search given the fp16 priors stays exact: the oracle replays a
small fp16-mode self-play batch bit for bit."""
import numpy as np
import pytest

from oracle import oracle as O
from oracle import spec

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def mods():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from yacht_amd import engine, kernels, nnet
    return kernels, nnet, engine


def _model(N, hidden, nblocks, seed):
    torch.manual_seed(seed)
    model = N.YachtNNet(hidden=hidden, nblocks=nblocks).eval()
    with torch.no_grad():  # non-trivial LayerNorm affines
        for m in model.modules():
            if isinstance(m, torch.nn.LayerNorm):
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.2, 0.2)
    return model


@pytest.mark.parametrize("hidden,nblocks", [(256, 6), (64, 1), (512, 1)])
def test_f16_predict_vs_torch_autocast(mods, golden, hidden, nblocks):
    K, N, _ = mods
    model = _model(N, hidden, nblocks, 7 + hidden + nblocks)
    net = N.YkNet(model.state_dict(), hidden, nblocks, precision="f16")
    S = K.states_to_device(golden("states.npz")["states"][:1000])
    pi, v = net.predict_states(S)
    x = K.featurize(S)
    m = model.to("cuda")
    with torch.no_grad():
        m64 = _model(N, hidden, nblocks, 7 + hidden + nblocks).double().to("cuda")
        l64, v64 = m64(x.double())
        p64 = torch.log_softmax(l64, 1).exp()
        with torch.autocast("cuda"):  # NNet.py:186-189
            lac, vac = m(x)
        pac = torch.nn.functional.log_softmax(lac, dim=1).exp()  # NNet.py:193 (outside autocast)
    p64, v64 = p64.cpu().numpy(), v64[:, 0].cpu().numpy()
    pac, vac = pac.double().cpu().numpy(), vac[:, 0].double().cpu().numpy()
    pi, v = pi.double().cpu().numpy(), v.double().cpu().numpy()
    e_ac_pi, e_ac_v = np.abs(pac - p64).max(), np.abs(vac - v64).max()
    e_pi, e_v = np.abs(pi - p64).max(), np.abs(v - v64).max()
    print(f"\nH{hidden}x{nblocks}: max|pi - pi64| fp16 mode {e_pi:.3e} autocast {e_ac_pi:.3e}; "
          f"max|v - v64| fp16 mode {e_v:.3e} autocast {e_ac_v:.3e}")
    assert e_pi <= e_ac_pi and e_v <= e_ac_v
    assert np.abs(pi - pac).max() <= 2 * e_ac_pi and np.abs(v - vac).max() <= 2 * e_ac_v
    assert np.allclose(pi.sum(1), 1.0, atol=1e-4)


def test_f16_selfplay_replayed_by_oracle(mods):
    """Self-play with the fp16 forward: the oracle's MCTS given the recorded fp16 priors
    reproduces every move (visit counts, actions, counters, values)."""
    _, N, E = mods
    n, sims, seed, base = 8, 16, 91, 40
    net = N.YkNet(spec.closed_form_weights(256, 6), 256, 6, precision="f16")
    eng = E.SelfPlayEngine(n, sims, 1.5, 15, net=net, max_moves=64, record_predictions=True,
                           max_expansions=64 * sims)
    eng.run(seed, base)
    assert eng.stats()["errors"] == 0
    rec = eng.records()
    pi, v, cnt, leaves = eng.predictions(leaves=True)
    orc = O.selfplay(np.arange(base, base + n), seed, sims, 1.5, 15, O.MODE_REPLAY,
                     replay=[(pi[e, :cnt[e]], v[e, :cnt[e]]) for e in range(n)])
    assert orc["nerr"] == 0
    assert np.array_equal(orc["stats"][:, 1], cnt)
    for e in range(n):
        M = int(orc["stats"][e, 0])
        assert rec["n_moves"][e] == M == 48
        assert np.array_equal(rec["info"][e, :M, :7], orc["mv"][e, :M, :7])
        assert np.array_equal(rec["values"][e, :M], orc["values"][e, :M])
        assert np.array_equal(rec["final"][e], orc["final"][e])
    eng.close()
