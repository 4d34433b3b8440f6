"""Pin the C restatement (oracle/) against vectors produced by the reference itself.

Fixtures come from tests/golden/make_golden.py (reference imported read-only, RNG
entry points replaced by the per-game Philox stream of oracle/spec.py)."""
import numpy as np
import pytest

from oracle import oracle as O
from oracle import spec


def test_philox_python_matches_c():
    for seed, env in ((0, 0), (20251015, 7), (2**63 + 5, 2**32 - 1)):
        c = O.draws(seed, env, 12345, 16)
        py = [spec.draw64(seed, env, 12345 + i) for i in range(16)]
        assert [int(x) for x in c] == py


def test_philox_known_answer():
    # Random123 philox4x32-10 known-answer vector: ctr=0, key=0
    assert spec.philox4x32_10(0, 0, 0, 0, 0, 0) == (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)
    assert spec.philox4x32_10(0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF) == \
        (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)


def test_score_table_exhaustive(golden):
    g = golden("score_table.npz")
    assert np.array_equal(O.score_dice(g["dice"]), g["score"])


def test_transitions_bit_exact(golden):
    g = golden("transitions.npz")
    seed = int(g["seed"])
    out, npl, st, ctr = O.step(g["state"], g["player"], g["action"], seed, g["env"].astype(np.uint32),
                               g["ctr"])
    assert np.array_equal(st, g["status"].astype(np.int8))
    ok = g["status"] == 0
    assert np.array_equal(out[ok], g["next_state"][ok])
    assert np.array_equal(npl[ok], g["next_player"][ok].astype(np.int32))
    assert np.array_equal(ctr[ok], g["ctr_after"][ok])


def test_state_functions(golden):
    g = golden("states.npz")
    W = g["states"]
    valid = np.unpackbits(g["valid"], axis=-1, bitorder="little")[..., :3226]
    for j, p in enumerate((1, -1)):
        v, cnt = O.valid(W, p)
        assert np.array_equal(v, valid[:, j])
        assert np.array_equal(cnt, valid[:, j].sum(-1))
        r, tot = O.ended(W, p)
        assert np.array_equal(r, g["ended"][:, j])
    assert np.array_equal(tot, g["totals"].astype(np.int32))
    assert np.array_equal(O.canonical(W, -1), g["canon"])
    assert np.array_equal(O.canonical(W, 1), W)
    x = O.featurize(W)
    assert np.array_equal(x.view(np.uint32), g["feat"].view(np.uint32))


def test_pack_roundtrip(golden):
    g = golden("states.npz")
    for w in g["states"][:500]:
        d = spec.unpack_words(w)

        class P:
            pass
        s = P()
        for k in ("round_no", "phase", "rollA", "rollB", "p1_bid", "p2_bid"):
            setattr(s, k, d[k])
        for k in ("p1", "p2"):
            q = P()
            for kk, vv in d[k].items():
                setattr(q, kk, vv)
            setattr(s, k, q)
        assert spec.pack_state(s) == [int(x) for x in w]


def test_hash_prior_python_matches_c(golden):
    W = golden("states.npz")["states"][:64]
    pi, v = O.hash_prior(W)
    assert [int(h) for h in O.key_hash(W)] == [spec.key_hash(w) for w in W]
    for i in range(len(W)):
        p2, v2 = spec.hash_prior(W[i])
        assert np.array_equal(pi[i], p2) and v[i] == v2


def test_pairwise_sum_matches_numpy():
    rng = np.random.default_rng(0)
    for n in (1, 7, 8, 9, 127, 128, 129, 1000, 3226):
        for _ in range(20):
            a = (rng.random(n) * rng.integers(0, 2, n) * 10.0 ** rng.integers(-4, 4)).astype(np.float32)
            assert O.pairwise_sum(a) == np.sum(a)


@pytest.mark.parametrize("hidden,nblocks", [(256, 6), (64, 1)])
def test_predict_vs_reference(golden, hidden, nblocks):
    g = golden(f"predict_h{hidden}_b{nblocks}.npz")
    net = O.Net(spec.closed_form_weights(hidden, nblocks), hidden, nblocks)
    x = O.featurize(g["states"])
    assert np.array_equal(x, g["x"])
    pi, v = net.predict_states(g["states"])
    np.testing.assert_allclose(pi, g["pi"], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(v, g["v"], rtol=0, atol=1e-5)


def test_reverse_sum_order_is_another_valid_f32_forward(golden):
    """oracle.Net(reverse_sums=True) (the f32-vs-f32 divergence baseline of
    test_gpu_selfplay.py) sums every Linear last to first: its outputs differ from the forward
    order's in the last bits and hold the same tolerance to the reference."""
    g = golden("predict_h256_b6.npz")
    sd = spec.closed_form_weights(256, 6)
    pi, v = O.Net(sd, 256, 6).predict_states(g["states"])
    pr, vr = O.Net(sd, 256, 6, reverse_sums=True).predict_states(g["states"])
    assert (pi != pr).mean() > 0.5
    np.testing.assert_allclose(pr, g["pi"], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(vr, g["v"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(pr, pi, rtol=1e-5, atol=1e-7)


def _episode_case(g, i):
    meta = g["meta"][i]
    return dict(seed=int(meta[0]), env=int(meta[1]), sims=int(meta[2]), tt=int(meta[3]), nmoves=int(meta[4]),
                ctr_end=int(meta[5]), expansions=int(meta[6]), nodes=int(meta[7]), cpuct=float(g["cpuct"][i]))


def test_selfplay_hash_prior_matches_reference(golden):
    g = golden("episodes_hash.npz")
    for i in range(len(g["meta"])):
        c = _episode_case(g, i)
        r = O.selfplay([c["env"]], c["seed"], c["sims"], c["cpuct"], c["tt"], O.MODE_HASH)
        assert r["nerr"] == 0
        st = r["stats"][0]
        M = c["nmoves"]
        assert st[0] == M and st[1] == c["expansions"] and st[2] == c["nodes"] and st[4] == c["ctr_end"]
        assert np.array_equal(r["canon"][0, :M], g["canon"][i, :M])
        mv = g["moves"][i, :M]  # temp, player, action, ctr_search, ctr_step, n_ps, root_ns, ncounts
        assert np.array_equal(r["mv"][0, :M, 0], mv[:, 0])
        assert np.array_equal(r["mv"][0, :M, 1], mv[:, 1])
        assert np.array_equal(r["mv"][0, :M, 2], mv[:, 2])
        assert np.array_equal(r["ctr"][0, :M, 0].astype(np.int64), mv[:, 3])
        assert np.array_equal(r["ctr"][0, :M, 1].astype(np.int64), mv[:, 4])
        assert np.array_equal(r["mv"][0, :M, 3], mv[:, 5])
        assert np.array_equal(r["mv"][0, :M, 4], mv[:, 6])
        off = g["count_off"][i]
        for j in range(M):
            a = g["count_action"][off[j]:off[j + 1]]
            n = g["count_n"][off[j]:off[j + 1]]
            dense = np.zeros(3226, dtype=np.int32)
            dense[a] = n
            assert np.array_equal(r["counts"][0, j], dense), (i, j)
        assert np.array_equal(r["values"][0, :M], g["values"][i, :M])


def test_arena_hash_prior_matches_reference(golden):
    """Arena.playGame (Arena.py:30-93): MCTS agent at temp 0 vs RandomYachtPlayer, both seats."""
    g = golden("arena_hash.npz")
    r = O.arena(g["env"], g["seat"], int(g["seed"]), int(g["sims"]))
    assert r["nerr"] == 0
    assert np.array_equal(r["result"], g["result"])
    assert np.array_equal(r["stats"][:, 0], g["n_moves"])
    assert np.array_equal(r["stats"][:, 1], g["expansions"])
    assert np.array_equal(r["stats"][:, 4], g["ctr_end"])
    for i, n in enumerate(g["n_moves"]):
        assert np.array_equal(r["actions"][i, :n], g["actions"][i, :n])


def test_greedy_player_matches_reference(golden):
    """GreedyYachtPlayer.play (YachtPlayers.py:186-214) on all 11,403 fixture states: bid
    heuristic (float64, round-half-even, index overflow past 100), greedy scorer, and the
    random-legal fallback drawn from the state's stream."""
    g = golden("greedy.npz")
    n = len(g["action"])
    acts, ctr = O.greedy_play(g["states"], int(g["seed"]), np.arange(n), 0)
    assert np.array_equal(acts, g["action"])
    assert np.array_equal(ctr, g["draws"].astype(np.uint64))
    # the heuristic alone: the played action, or -1 where play fell back (a draw, or no legal move)
    h = O.greedy_heuristic(g["states"])
    drew = g["draws"] > 0
    _, counts = O.valid(g["states"], np.ones(n, dtype=np.int32))
    assert ((h == g["action"]) | (h == -1)).all()
    assert (h[drew] == -1).all() and (h[(counts == 0)] == -1).all()
    assert ((h != -1) | drew | (counts == 0)).all()


@pytest.mark.parametrize("fixture,agent,opponent", [("arena_greedy_random.npz", "greedy", "random"),
                                                     ("arena_mcts_greedy.npz", "mcts", "greedy")])
def test_arena_player_pairings_match_reference(golden, fixture, agent, opponent):
    g = golden(fixture)
    r = O.arena(g["env"], g["seat"], int(g["seed"]), int(g["sims"]), agent=agent, opponent=opponent)
    assert r["nerr"] == 0
    assert np.array_equal(r["result"], g["result"])
    assert np.array_equal(r["stats"][:, 4], g["ctr_end"])
    for i, n in enumerate(g["n_moves"]):
        assert np.array_equal(r["actions"][i, :n], g["actions"][i, :n])


def test_prior_checker_accepts_the_oracle_net_and_rejects_a_perturbed_one(golden):
    """tests/helpers.check_recorded_priors (the GPU tests' prior check) on the CPU: the oracle's
    f32 net, recorded the way the engine records (Ps * valids), passes against the float64
    forward; the same priors with one logit moved by 1e-3 do not."""
    from helpers import check_recorded_priors
    sd = spec.closed_form_weights(64, 1)
    W = golden("states.npz")["states"][::23][:400]
    pi, v = O.Net(sd, 64, 1).predict_states(W)
    ok = O.valid(W, 1)[0].astype(bool)
    rec = np.where(ok, pi, 0.0).astype(np.float32)[None]
    cnt = np.array([len(W)])
    assert check_recorded_priors(rec, v[None], cnt, W[None], sd, 64, 1) == len(W)
    bad = rec.copy()
    r = int(np.argmax((ok.sum(1) > 1) & (ok.sum(1) < 20)))
    a = int(np.flatnonzero(ok[r])[0])
    bad[0, r, a] *= np.float32(np.exp(1e-3))
    with pytest.raises(AssertionError):
        check_recorded_priors(bad, v[None], cnt, W[None], sd, 64, 1)


@pytest.mark.parametrize("tag", ["shared", "fresh"])
def test_gating_arena_matches_reference(golden, tag):
    """The oracle's dual-tree arena (Coach.learn's pmcts vs nmcts, Coach.py:117-139) against the
    REFERENCE's games: trees kept across the games of playGames (shared) and fresh per game."""
    g = golden("arena_gating_hash.npz")
    o = O.arena_dual(g["env"], g["seat"], int(g["seed"]), int(g["sims"]), float(g["cpuct"]), shared=tag == "shared")
    assert o["nerr"] == 0
    assert np.array_equal(o["result"], g[tag + "_result"])
    assert np.array_equal(o["stats"][:, 4], g[tag + "_ctr_end"])
    assert np.array_equal(o["stats"][:, 1], g[tag + "_expansions"])
    for i, m in enumerate(g[tag + "_n_moves"]):
        assert np.array_equal(o["actions"][i, :m], g[tag + "_actions"][i, :m]), i


def test_gating_arena_fresh_trees_equal_shared_trees():
    """Where the engine differs from the reference by construction - one tree per game instead of
    pmcts / nmcts kept across the games of playGames - the oracle plays both ways: no game differs
    (96 games here; 400 games at 25 sims measured identical too)."""
    n = 96
    env = np.arange(n) + 123
    seats = np.where(np.arange(n) < n // 2, 1, -1)
    a = O.arena_dual(env, seats, 17, 10, 1.5, shared=True)
    b = O.arena_dual(env, seats, 17, 10, 1.5, shared=False, threads=8)
    assert a["nerr"] == 0 and b["nerr"] == 0
    for k in ("result", "totals", "final", "actions"):
        assert np.array_equal(a[k], b[k]), k
    assert np.array_equal(a["stats"][:, 1], b["stats"][:, 1]) and np.array_equal(a["stats"][:, 4], b["stats"][:, 4])
