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
