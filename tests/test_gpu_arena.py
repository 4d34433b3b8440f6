"""GPU parity of the batched Arena (Arena.playGame, Arena.py:30-93): the MCTS agent at
temperature 0 (Coach.py:124-125) against RandomYachtPlayer (YachtPlayers.py:174-183).

* hash prior: the engine reproduces, bit for bit, the games that the REFERENCE's own
  Arena / MCTS / RandomYachtPlayer / YachtGame played (tests/golden/arena_hash.npz), and the
  C oracle on further games (results, both totals, actions, final states, RNG counters);
* YachtNNet prior: the oracle replays the engine's recorded predictions and must end every
  game identically;
* the plugin classes (MCTSArena.playGames, sequential Arena with the MCTS plugin) agree.
"""
import numpy as np
import pytest

from oracle import oracle as O
from oracle import spec
from helpers import check_recorded_priors

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def Y():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from yacht_amd import engine, nnet
    return engine, nnet


def test_arena_hash_prior_matches_reference_games(Y, golden):
    E, _ = Y
    g = golden("arena_hash.npz")
    env = g["env"]
    assert np.array_equal(env, np.arange(env[0], env[0] + len(env)))
    eng = E.SelfPlayEngine(len(env), int(g["sims"]), 1.5, 0, prior="hash", max_moves=64)
    eng.arena(g["seat"], int(g["seed"]), int(env[0]))
    r = eng.arena_results()
    assert np.array_equal(r["result"], g["result"])
    assert np.array_equal(r["n_moves"], g["n_moves"])
    assert np.array_equal(r["ctr"], g["ctr_end"].astype(np.uint64))
    for i, n in enumerate(g["n_moves"]):
        assert np.array_equal(r["actions"][i, :n], g["actions"][i, :n]), i
    assert eng.stats()["expansions"] == int(g["expansions"].sum())


@pytest.mark.parametrize("sims,cpuct", [(25, 1.5), (4, 1.0), (2, 1.5)])
def test_arena_hash_prior_matches_oracle(Y, sims, cpuct):
    E, _ = Y
    n, seed, base = 96, 4242, 3000
    seats = np.where(np.arange(n) % 3 == 0, -1, 1).astype(np.int32)
    eng = E.SelfPlayEngine(n, sims, cpuct, 0, prior="hash", max_moves=64)
    eng.arena(seats, seed, base)
    r = eng.arena_results()
    o = O.arena(np.arange(base, base + n), seats, seed, sims, cpuct, threads=8)
    assert o["nerr"] == 0
    assert np.array_equal(r["result"], o["result"])
    assert np.array_equal(r["totals"], o["totals"])
    assert np.array_equal(r["final"], o["final"])
    assert np.array_equal(r["n_moves"], o["stats"][:, 0].astype(np.int32))
    assert np.array_equal(r["ctr"], o["stats"][:, 4].astype(np.uint64))
    for i in range(n):
        m = int(r["n_moves"][i])
        assert np.array_equal(r["actions"][i, :m], o["actions"][i, :m]), i
    # the totals are the final board's, and result is curPlayer * getGameEnded from player 1's view
    ended, tot = O.ended(r["final"], np.ones(n, dtype=np.int32))
    assert np.array_equal(tot, r["totals"])
    assert np.array_equal(ended, r["result"])


def test_arena_one_sim_picks_an_illegal_action_like_the_reference(Y):
    """With 1 simulation the root has no visited child: every count is 0, the tie set is all
    3226 actions, and the pick is usually illegal - the reference's Arena asserts
    (Arena.py:58-64); the engine reports a transition error, the oracle an error per game."""
    from yacht_amd._lib import YkError
    E, _ = Y
    n = 8
    eng = E.SelfPlayEngine(n, 1, 1.5, 0, prior="hash", max_moves=64)
    with pytest.raises(YkError, match="transition status"):
        eng.arena(np.ones(n, dtype=np.int32), 3, 0)
    o = O.arena(np.arange(n), np.ones(n, dtype=np.int32), 3, 1)
    assert o["nerr"] == n


def test_arena_net_prior_replayed_by_oracle(Y):
    E, N = Y
    n, sims, seed, base = 8, 10, 91, 40
    sd = spec.closed_form_weights(256, 6)
    net = N.YkNet(sd, 256, 6)
    seats = np.array([1, -1] * (n // 2), dtype=np.int32)
    eng = E.SelfPlayEngine(n, sims, 1.5, 0, net=net, max_moves=64, record_predictions=True,
                           max_expansions=64 * sims)
    eng.arena(seats, seed, base)
    r = eng.arena_results()
    pi, v, cnt = eng.predictions()
    replay = [(pi[e, :cnt[e]], v[e, :cnt[e]]) for e in range(n)]
    o = O.arena(np.arange(base, base + n), seats, seed, sims, 1.5, O.MODE_REPLAY, replay=replay)
    assert o["nerr"] == 0
    assert np.array_equal(o["stats"][:, 1], cnt)
    assert np.array_equal(r["result"], o["result"])
    assert np.array_equal(r["totals"], o["totals"])
    assert np.array_equal(r["final"], o["final"])
    assert np.array_equal(r["ctr"], o["stats"][:, 4].astype(np.uint64))


def _compare_arena(r, o, n):
    assert o["nerr"] == 0
    assert np.array_equal(r["result"], o["result"])
    assert np.array_equal(r["totals"], o["totals"])
    assert np.array_equal(r["final"], o["final"])
    assert np.array_equal(r["n_moves"], o["stats"][:, 0].astype(np.int32))
    assert np.array_equal(r["ctr"], o["stats"][:, 4].astype(np.uint64))
    for i in range(n):
        m = int(r["n_moves"][i])
        assert np.array_equal(r["actions"][i, :m], o["actions"][i, :m]), i


def test_arena_1000_games_hash_prior_vs_oracle(Y):
    """Config 4's shape: Arena.playGames(1000) (Arena.py:95-130: half the games in each seat),
    MCTS temp 0 at 25 sims vs RandomYachtPlayer, every result, both totals, every action and
    final board bit-exact against the oracle's own independent run."""
    E, _ = Y
    n, sims, seed, base = 1000, 25, 31337, 0
    seats = np.where(np.arange(n) < n // 2, 1, -1).astype(np.int32)
    eng = E.SelfPlayEngine(n, sims, 1.5, 0, prior="hash", max_moves=48)
    eng.arena(seats, seed, base)
    r = eng.arena_results()
    o = O.arena(np.arange(base, base + n), seats, seed, sims, 1.5, max_moves=48, threads=16)
    _compare_arena(r, o, n)
    ended, tot = O.ended(r["final"], np.ones(n, dtype=np.int32))
    assert np.array_equal(tot, r["totals"]) and np.array_equal(ended, r["result"])


def test_arena_1000_games_net_prior_replayed_by_oracle(Y):
    """Config 4 as bench.py runs it (1000 games, 25 sims, random-init YachtNNet 256 x 6 on the
    production valid-only forward): every game's predictions recorded, the oracle replays them
    and ends all 1000 games identically; the recorded priors match the oracle net."""
    E, N = Y
    n, sims, seed, base = 1000, 25, 4711, 100000
    sd = spec.closed_form_weights(256, 6)
    seats = np.where(np.arange(n) < n // 2, 1, -1).astype(np.int32)
    ynet = N.YkNet(sd, 256, 6)
    eng = E.SelfPlayEngine(n, sims, 1.5, 0, net=ynet, max_moves=48, record_predictions=True,
                           max_expansions=24 * sims + 16)
    eng.arena(seats, seed, base)
    r = eng.arena_results()
    pi, v, cnt, leaves = eng.predictions(leaves=True)
    replay = [(pi[e, :cnt[e]], v[e, :cnt[e]]) for e in range(n)]
    o = O.arena(np.arange(base, base + n), seats, seed, sims, 1.5, O.MODE_REPLAY, replay=replay, max_moves=48,
                threads=16)
    assert np.array_equal(o["stats"][:, 1], cnt)
    _compare_arena(r, o, n)
    assert check_recorded_priors(pi, v, cnt, leaves, sd, every=40, net=ynet) > 10000


def test_arena_after_selfplay_and_back(Y):
    """The engine switches modes cleanly (idle flags, trees, records)."""
    E, _ = Y
    n, sims, seed = 16, 6, 5
    eng = E.SelfPlayEngine(n, sims, 1.5, 15, prior="hash", max_moves=64)
    eng.run(seed, 0)
    rec1 = eng.records()
    eng.arena(np.ones(n, dtype=np.int32), seed, 100)
    r = eng.arena_results()
    o = O.arena(np.arange(100, 100 + n), np.ones(n, dtype=np.int32), seed, sims)
    assert np.array_equal(r["result"], o["result"])
    eng.run(seed, 0)
    rec2 = eng.records()
    for k in ("states", "info", "ctr", "values", "final", "n_moves"):
        assert np.array_equal(rec1[k], rec2[k]), k


def test_mcts_arena_playgames_and_sequential_arena(Y):
    from yacht_amd.arena import Arena, MCTSArena, RandomYachtPlayer
    from yacht_amd.game import YachtGame
    from yacht_amd.mcts import MCTS
    from yacht_amd.nnet import HashPriorNet
    from yacht_amd.utils import dotdict
    args = dotdict(numMCTSSims=6, cpuct=1.5)
    game = YachtGame(seed=11, env_id=200)
    one, two, draws = MCTSArena(game, HashPriorNet(game), args).playGames(20)
    assert one + two + draws == 20
    seats = np.array([1] * 10 + [-1] * 10, dtype=np.int32)
    o = O.arena(np.arange(200, 220), seats, 11, 6)
    agent = o["result"] * seats
    assert (one, two) == (int((agent == 1).sum()), int((agent == -1).sum()))
    # one game through the sequential host loop with the MCTS plugin: same as the oracle
    g2 = YachtGame(seed=11, env_id=200)
    mcts = MCTS(g2, HashPriorNet(g2), args)
    res = Arena(lambda x: int(np.argmax(mcts.getActionProb(x, temp=0))), RandomYachtPlayer(g2).play,
                g2).playGame()
    assert res == o["result"][0]


def test_mcts_plugin_resets_its_tree_for_a_new_game(Y):
    """One MCTS object over two games (Arena.playGames reuses pmcts / nmcts, Coach.py:120-125):
    when the next root has a lower round the plugin resets its tree
    and plays the second game exactly as a fresh MCTS object does; the raw C call refuses the
    lower round without the reset."""
    from yacht_amd._lib import YkError, call
    from yacht_amd.arena import Arena, RandomYachtPlayer
    from yacht_amd.game import YachtGame
    from yacht_amd.mcts import MCTS
    from yacht_amd.nnet import HashPriorNet
    from yacht_amd.utils import dotdict
    args = dotdict(numMCTSSims=6, cpuct=1.5)

    def play(game, mcts):
        return Arena(lambda x: int(np.argmax(mcts.getActionProb(x, temp=0))), RandomYachtPlayer(game).play,
                     game).playGame(), game.rng.ctr

    g1 = YachtGame(seed=12, env_id=300)
    shared = MCTS(g1, HashPriorNet(g1), args)
    play(g1, shared)                     # game 1 leaves a tree of late rounds behind
    g1.rng.env, g1.rng.ctr = 301, 0      # game 2 on its own stream
    reused = play(g1, shared)
    g2 = YachtGame(seed=12, env_id=301)
    fresh = play(g2, MCTS(g2, HashPriorNet(g2), args))
    assert reused == fresh
    # the C ABI itself: a lower-round root without yk_mcts_reset is an engine state error
    import torch as T
    from yacht_amd import kernels as K
    from yacht_amd.state import ACTION_SIZE, pack
    eng = shared._eng()
    late = K.states_to_device(pack(g1.getInitBoard()))
    counts = T.zeros((1, ACTION_SIZE), dtype=T.int32, device="cuda")
    env = T.tensor([301], dtype=T.int32, device="cuda")
    ctr = T.tensor([0], dtype=T.int64, device="cuda")
    with pytest.raises(YkError):
        call("yk_mcts_search", eng.handle, late.data_ptr(), 12, env.data_ptr(), ctr.data_ptr(), 2,
             counts.data_ptr(), 0)


def test_greedy_heuristic_kernel_matches_reference(Y, golden):
    """yk_greedy_action on all 11,403 fixture states against the reference GreedyYachtPlayer's
    choices (tests/golden/greedy.npz) and the C restatement."""
    from yacht_amd import kernels as K
    g = golden("greedy.npz")
    h = K.greedy_action(K.states_to_device(g["states"])).cpu().numpy()
    assert np.array_equal(h, O.greedy_heuristic(g["states"]))
    ok = h >= 0
    assert np.array_equal(h[ok], g["action"][ok])
    assert (g["draws"][~ok] > 0).sum() == (g["draws"] > 0).sum()  # every fallback draw is a -1 here


@pytest.mark.parametrize("fixture,agent,opponent", [("arena_greedy_random.npz", "greedy", "random"),
                                                     ("arena_mcts_greedy.npz", "mcts", "greedy")])
def test_arena_pairings_match_reference_games(Y, golden, fixture, agent, opponent):
    E, _ = Y
    g = golden(fixture)
    env = g["env"]
    eng = E.SelfPlayEngine(len(env), max(int(g["sims"]), 1), 1.5, 0, prior="hash", max_moves=64)
    eng.arena(g["seat"], int(g["seed"]), int(env[0]), agent=agent, opponent=opponent)
    r = eng.arena_results()
    assert np.array_equal(r["result"], g["result"])
    assert np.array_equal(r["ctr"], g["ctr_end"].astype(np.uint64))
    for i, n in enumerate(g["n_moves"]):
        assert np.array_equal(r["actions"][i, :n], g["actions"][i, :n]), i


@pytest.mark.parametrize("agent,opponent,sims,n", [("greedy", "random", 1, 256), ("random", "greedy", 1, 128),
                                                   ("mcts", "greedy", 4, 64), ("greedy", "mcts", 6, 48),
                                                   ("greedy", "greedy", 1, 64)])
def test_arena_pairings_match_oracle(Y, agent, opponent, sims, n):
    E, _ = Y
    seed, base = 9100 + sims, 40000
    seats = np.where(np.arange(n) % 2 == 0, 1, -1).astype(np.int32)
    eng = E.SelfPlayEngine(n, sims, 1.5, 0, prior="hash", max_moves=64)
    eng.arena(seats, seed, base, agent=agent, opponent=opponent)
    r = eng.arena_results()
    o = O.arena(np.arange(base, base + n), seats, seed, sims, 1.5, agent=agent, opponent=opponent, threads=8)
    assert o["nerr"] == 0
    assert np.array_equal(r["result"], o["result"])
    assert np.array_equal(r["totals"], o["totals"])
    assert np.array_equal(r["final"], o["final"])
    assert np.array_equal(r["ctr"], o["stats"][:, 4].astype(np.uint64))


def test_sequential_arena_with_greedy_plugin(Y, golden):
    from yacht_amd.arena import Arena, GreedyYachtPlayer, MCTSArena, RandomYachtPlayer
    from yacht_amd.game import YachtGame
    from yacht_amd.utils import dotdict
    g = golden("arena_greedy_random.npz")
    game = YachtGame(seed=int(g["seed"]), env_id=int(g["env"][0]))
    res = Arena(GreedyYachtPlayer(game).play, RandomYachtPlayer(game).play, game).playGame()
    assert res == g["result"][0] and game.rng.ctr == int(g["ctr_end"][0])
    one, two, draws = MCTSArena(YachtGame(seed=5, env_id=0), None, dotdict(), agent="greedy",
                                opponent="random").playGames(200)
    assert one + two + draws == 200 and one > 180  # the greedy player beats random almost always


def test_gating_arena_matches_reference_games(Y, golden):
    """The gating arena of Coach.learn (Coach.py:117-139) on the engine's dual trees: the REFERENCE
    played these games with pmcts / nmcts kept across all games of Arena.playGames (and again with
    fresh MCTS objects per game: identical, tests/golden/arena_gating_hash.npz); the engine (one tree
    per seat per game) reproduces results, actions, counters and expansions bit for bit."""
    E, _ = Y
    g = golden("arena_gating_hash.npz")
    n = len(g["env"])
    for k in ("result", "actions", "ctr_end", "expansions"):  # the reference: shared trees change nothing here
        assert np.array_equal(g["shared_" + k], g["fresh_" + k]), k
    eng = E.SelfPlayEngine(n, int(g["sims"]), float(g["cpuct"]), 0, prior="hash", max_moves=48, dual_trees=True)
    eng.arena(g["seat"], int(g["seed"]), int(g["env"][0]), agent="mcts", opponent="mcts")
    r = eng.arena_results()
    assert np.array_equal(r["result"], g["shared_result"])
    assert np.array_equal(r["n_moves"], g["shared_n_moves"])
    assert np.array_equal(r["ctr"], g["shared_ctr_end"].astype(np.uint64))
    for i, m in enumerate(g["shared_n_moves"]):
        assert np.array_equal(r["actions"][i, :m], g["shared_actions"][i, :m]), i
    assert eng.stats()["expansions"] == int(g["shared_expansions"].sum())


def test_gating_arena_two_nets_replayed_by_oracle(Y):
    """Two different nets, one per seat, each its own tree: the oracle (dual trees) replays the
    engine's recorded predictions and ends every game identically; every recorded value is the
    value of one of the two nets at that leaf, and both nets are used."""
    from helpers import torch_predict
    E, N = Y
    n, sims, seed, base = 256, 10, 515, 7000
    sd_a = spec.closed_form_weights(256, 6)
    sd_b = {k: (np.asarray(v, dtype=np.float32) * np.float32(0.9) if k.endswith("weight") else v)
            for k, v in sd_a.items()}
    seats = np.where(np.arange(n) < n // 2, 1, -1).astype(np.int32)
    eng = E.SelfPlayEngine(n, sims, 1.5, 0, net=N.YkNet(sd_a, 256, 6), opponent_net=N.YkNet(sd_b, 256, 6),
                           max_moves=48, record_predictions=True, max_expansions=48 * sims + 16, dual_trees=True)
    eng.arena(seats, seed, base, agent="mcts", opponent="mcts")
    r = eng.arena_results()
    pi, v, cnt, leaves = eng.predictions(leaves=True)
    o = O.arena_dual(np.arange(base, base + n), seats, seed, sims, 1.5, O.MODE_REPLAY,
                     replay=[(pi[e, :cnt[e]], v[e, :cnt[e]]) for e in range(n)], max_moves=48, threads=16)
    assert np.array_equal(o["stats"][:, 1], cnt)
    _compare_arena(r, o, n)
    S = np.concatenate([leaves[e, :cnt[e]:7] for e in range(n)])
    V = np.concatenate([v[e, :cnt[e]:7] for e in range(n)])
    import torch
    _, va = torch_predict(sd_a, 256, 6, S, torch.float64)
    _, vb = torch_predict(sd_b, 256, 6, S, torch.float64)
    is_a, is_b = np.abs(V - va) <= 2e-5, np.abs(V - vb) <= 2e-5
    assert (is_a | is_b).all() and (is_a & ~is_b).any() and (is_b & ~is_a).any()
