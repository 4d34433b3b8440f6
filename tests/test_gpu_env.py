"""GPU parity of the Game-plugin kernels: bit-exact against the reference's own vectors
(tests/golden, produced by running /root/reference) and against the C oracle on large
random batches."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def K():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from yacht_amd import kernels
    return kernels


def test_score_dice_exhaustive(K, golden):
    g = golden("score_table.npz")
    out = K.score_dice(torch.from_numpy(g["dice"]))
    assert np.array_equal(out.cpu().numpy(), g["score"])


def test_transitions_vs_reference(K, golden):
    g = golden("transitions.npz")
    out, npl, st, c = K.step(K.states_to_device(g["state"]), g["player"], g["action"], int(g["seed"]),
                             g["env"].astype(np.int32), g["ctr"].astype(np.int64))
    st = st.cpu().numpy()
    assert np.array_equal(st, g["status"].astype(np.int8))
    ok = g["status"] == 0
    assert np.array_equal(K.states_to_host(out)[ok], g["next_state"][ok])
    assert np.array_equal(npl.cpu().numpy()[ok], g["next_player"][ok])
    assert np.array_equal(c.cpu().numpy().astype(np.uint64)[ok], g["ctr_after"][ok])


def test_state_functions_vs_reference(K, golden):
    g = golden("states.npz")
    W = g["states"]
    S = K.states_to_device(W)
    valid = np.unpackbits(g["valid"], axis=-1, bitorder="little")[..., :3226]
    for j, p in enumerate((1, -1)):
        mask, cnt = K.valid_mask(S, p)
        assert np.array_equal(K.unpack_mask(mask).cpu().numpy(), valid[:, j])
        assert np.array_equal(cnt.cpu().numpy(), valid[:, j].sum(-1))
        r, tot = K.ended(S, p)
        assert np.array_equal(r.cpu().numpy(), g["ended"][:, j])
    assert np.array_equal(tot.cpu().numpy(), g["totals"].astype(np.int32))
    assert np.array_equal(K.states_to_host(K.canonical(S, -1)), g["canon"])
    assert np.array_equal(K.states_to_host(K.canonical(S, 1)), W)
    x = K.featurize(S).cpu().numpy()
    assert np.array_equal(x.view(np.uint32), g["feat"].view(np.uint32))


def test_score_table_hash_and_prior_vs_oracle(K, golden):
    W = golden("states.npz")["states"]
    S = K.states_to_device(W)
    for p in (1, -1):
        assert np.array_equal(K.score_table(S, p).cpu().numpy(), O.score_table(W, p))
    assert np.array_equal(K.key_hash(S).cpu().numpy().view(np.uint64), O.key_hash(W))
    pi, v = K.hash_prior(S[:256])
    opi, ov = O.hash_prior(W[:256])
    assert np.array_equal(pi.cpu().numpy(), opi) and np.array_equal(v.cpu().numpy(), ov)


def test_init_board_vs_oracle(K):
    envs = np.arange(5000, dtype=np.uint32)
    out, c = K.init_board(99, envs.astype(np.int32), 0)
    ow, oc = O.init_board(99, envs, 0)
    assert np.array_equal(K.states_to_host(out), ow)
    assert np.array_equal(c.cpu().numpy().astype(np.uint64), oc)


def _random_walk_states(n_games, seed=3):
    """States from real-game and MCTS-style (player 1 + canonical) random walks via the oracle."""
    rng = np.random.default_rng(seed)
    envs = np.arange(n_games, dtype=np.uint32)
    s, ctr = O.init_board(seed, envs, 0)
    players = np.ones(n_games, dtype=np.int32)
    alls = []
    for t in range(60):
        alls.append((s.copy(), players.copy(), ctr.copy()))
        v, cnt = O.valid(s, players)
        live = cnt > 0
        if not live.any():
            break
        u = rng.random(n_games)
        a = np.zeros(n_games, dtype=np.int32)
        for i in np.nonzero(live)[0]:
            idx = np.nonzero(v[i])[0]
            a[i] = idx[int(u[i] * len(idx))]
        ns, npl, st, nc = O.step(s, players, a, seed, envs, ctr)
        assert (st[live] == 0).all()
        mcts_style = rng.random(n_games) < 0.3
        can = O.canonical(ns, npl)
        s = np.where(live[:, None], np.where(mcts_style[:, None], can, ns), s)
        players = np.where(live, np.where(mcts_style, 1, npl), players).astype(np.int32)
        ctr = np.where(live, nc, ctr)
    return alls


def test_random_transitions_vs_oracle(K):
    seed = 3
    for s, players, ctr in _random_walk_states(2048, seed)[::3]:
        n = len(s)
        rng = np.random.default_rng(len(s) + int(ctr.sum() % 1000))
        actions = rng.integers(0, 3226, n).astype(np.int32)  # valid and invalid alike
        envs = np.arange(n, dtype=np.uint32)
        ow, onp, ost, oc = O.step(s, players, actions, seed, envs, ctr)
        gw, gnp, gst, gc = K.step(K.states_to_device(s), players, actions, seed, envs.astype(np.int32),
                                  ctr.astype(np.int64))
        gst = gst.cpu().numpy()
        assert np.array_equal(gst, ost)
        ok = ost == 0
        assert np.array_equal(K.states_to_host(gw)[ok], ow[ok])
        assert np.array_equal(gnp.cpu().numpy()[ok], onp[ok])
        assert np.array_equal(gc.cpu().numpy().astype(np.uint64)[ok], oc[ok])
        ov, ocnt = O.valid(s, players)
        m, cnt = K.valid_mask(K.states_to_device(s), players)
        assert np.array_equal(K.unpack_mask(m).cpu().numpy(), ov) and np.array_equal(cnt.cpu().numpy(), ocnt)
        assert np.array_equal(K.featurize(K.states_to_device(s)).cpu().numpy().view(np.uint32),
                              O.featurize(s).view(np.uint32))


def test_empty_and_single_batches(K):
    from yacht_amd._lib import call, stream_ptr
    call("yk_step", 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, stream_ptr())  # n == 0 is a no-op
    out, c = K.init_board(1, [7], 0)
    assert K.states_to_host(out).shape == (1, 8)
