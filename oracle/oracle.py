"""ctypes front-end of the C restatement (``oracle/liboracle.so``).

TEST INFRASTRUCTURE ONLY: imported by ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s cpu_baseline leg, never by the product package.  Every array is numpy;
states are ``uint64[n, 8]`` packed words (``oracle/spec.py``).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from . import spec

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
ASIZE = spec.ACTION_SIZE

_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH) or \
            os.path.getmtime(LIB_PATH) < os.path.getmtime(os.path.join(HERE, "yk_oracle.c")):
        subprocess.run(["make", "-C", HERE, "-B" if force else "all"], check=True,
                       stdout=subprocess.DEVNULL)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = C.CDLL(LIB_PATH)
        _lib.or_net_create.restype = C.c_void_p
        _lib.or_net_create.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_void_p)]
        _lib.or_net_destroy.argtypes = [C.c_void_p]
        _lib.or_net_set_order.argtypes = [C.c_void_p, C.c_int]
        _lib.or_net_predict.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        _lib.or_net_forward_x.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        _lib.or_draw64.restype = C.c_uint64
        _lib.or_draw64.argtypes = [C.c_uint64, C.c_uint32, C.c_uint64]
        _lib.or_pairwise_sum.restype = C.c_float
        _lib.or_pairwise_sum.argtypes = [C.c_void_p, C.c_long]
        _lib.or_selfplay.restype = C.c_int
        _lib.or_selfplay.argtypes = [C.c_int, C.c_void_p, C.c_uint64, C.c_int, C.c_double, C.c_int, C.c_int,
                                     C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                     C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                     C.c_void_p, C.c_void_p, C.c_int]
        _lib.or_arena.restype = C.c_int
        _lib.or_arena.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_uint64, C.c_int, C.c_double,
                                  C.c_int, C.c_int,
                                  C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                  C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        _lib.or_arena_dual.restype = C.c_int
        _lib.or_arena_dual.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_int, C.c_double, C.c_int,
                                       C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                       C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        for name in ("or_step", "or_valid", "or_ended", "or_canonical", "or_featurize", "or_score_table",
                     "or_score_dice", "or_key_hash_batch", "or_hash_prior", "or_init_board", "or_draws",
                     "or_greedy_heuristic", "or_greedy_play"):
            getattr(_lib, name).restype = None
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def _w(states):
    return np.ascontiguousarray(np.asarray(states, dtype=np.uint64).reshape(-1, 8))


def _i32(x, n):
    return np.ascontiguousarray(np.broadcast_to(np.asarray(x, dtype=np.int32), (n,)))


def step(states, players, actions, seed, envs, ctr):
    w = _w(states)
    n = len(w)
    out = np.zeros_like(w)
    npl = np.zeros(n, dtype=np.int32)
    st = np.zeros(n, dtype=np.int8)
    c = np.ascontiguousarray(np.broadcast_to(np.asarray(ctr, dtype=np.uint64), (n,))).copy()
    e = np.ascontiguousarray(np.broadcast_to(np.asarray(envs, dtype=np.uint32), (n,)))
    lib().or_step(_p(w), _p(_i32(players, n)), _p(_i32(actions, n)), C.c_uint64(seed), _p(e), _p(c),
                  _p(out), _p(npl), _p(st), C.c_int(n))
    return out, npl, st, c


def valid(states, players):
    w = _w(states)
    n = len(w)
    out = np.zeros((n, ASIZE), dtype=np.uint8)
    cnt = np.zeros(n, dtype=np.int32)
    lib().or_valid(_p(w), _p(_i32(players, n)), _p(out), _p(cnt), C.c_int(n))
    return out, cnt


def ended(states, players):
    w = _w(states)
    n = len(w)
    r = np.zeros(n, dtype=np.float64)
    tot = np.zeros((n, 2), dtype=np.int32)
    lib().or_ended(_p(w), _p(_i32(players, n)), _p(r), _p(tot), C.c_int(n))
    return r, tot


def canonical(states, players):
    w = _w(states)
    out = np.zeros_like(w)
    lib().or_canonical(_p(w), _p(_i32(players, len(w))), _p(out), C.c_int(len(w)))
    return out


def featurize(states):
    w = _w(states)
    x = np.zeros((len(w), 59), dtype=np.float32)
    lib().or_featurize(_p(w), _p(x), C.c_int(len(w)))
    return x


def score_table(states, players):
    w = _w(states)
    out = np.zeros((len(w), 12, 252), dtype=np.int32)
    lib().or_score_table(_p(w), _p(_i32(players, len(w))), _p(out), C.c_int(len(w)))
    return out


def score_dice(dice):
    d = np.ascontiguousarray(np.asarray(dice, dtype=np.int8).reshape(-1, 5))
    out = np.zeros((len(d), 12), dtype=np.int32)
    lib().or_score_dice(_p(d), _p(out), C.c_int(len(d)))
    return out


def key_hash(states):
    w = _w(states)
    out = np.zeros(len(w), dtype=np.uint64)
    lib().or_key_hash_batch(_p(w), _p(out), C.c_int(len(w)))
    return out


def hash_prior(states):
    w = _w(states)
    pi = np.zeros((len(w), ASIZE), dtype=np.float32)
    v = np.zeros(len(w), dtype=np.float32)
    lib().or_hash_prior(_p(w), _p(pi), _p(v), C.c_int(len(w)))
    return pi, v


def init_board(seed, envs, ctr=0):
    e = np.ascontiguousarray(np.asarray(envs, dtype=np.uint32).reshape(-1))
    c = np.ascontiguousarray(np.broadcast_to(np.asarray(ctr, dtype=np.uint64), e.shape)).copy()
    out = np.zeros((len(e), 8), dtype=np.uint64)
    lib().or_init_board(C.c_uint64(seed), _p(e), _p(c), _p(out), C.c_int(len(e)))
    return out, c


def draws(seed, env, ctr0, n):
    out = np.zeros(n, dtype=np.uint64)
    lib().or_draws(C.c_uint64(seed), C.c_uint32(env), C.c_uint64(ctr0), _p(out), C.c_int(n))
    return out


def pairwise_sum(a):
    a = np.ascontiguousarray(a, dtype=np.float32)
    return np.float32(lib().or_pairwise_sum(_p(a), C.c_long(len(a))))


class Net:
    """C restatement of YachtNNet.forward + exp(log_softmax) (NNet.py:177-195)."""

    def __init__(self, state_dict, hidden, nblocks, reverse_sums=False):
        """reverse_sums: every Linear adds its inputs last to first - another valid float32
        evaluation order, for measuring how much float32 rounding alone changes a search."""
        self._keep = [np.ascontiguousarray(np.asarray(v, dtype=np.float32)) for v in state_dict.values()]
        arr = (C.c_void_p * len(self._keep))(*[a.ctypes.data for a in self._keep])
        self.h = lib().or_net_create(hidden, nblocks, arr)
        if reverse_sums:
            lib().or_net_set_order(C.c_void_p(self.h), 1)
        self.hidden, self.nblocks = hidden, nblocks

    def predict_states(self, states):
        w = _w(states)
        pi = np.zeros((len(w), ASIZE), dtype=np.float32)
        v = np.zeros(len(w), dtype=np.float32)
        lib().or_net_predict(C.c_void_p(self.h), _p(w), _p(pi), _p(v), C.c_int(len(w)))
        return pi, v

    def forward_x(self, x):
        x = np.ascontiguousarray(x, dtype=np.float32).reshape(-1, 59)
        pi = np.zeros((len(x), ASIZE), dtype=np.float32)
        v = np.zeros(len(x), dtype=np.float32)
        lib().or_net_forward_x(C.c_void_p(self.h), _p(x), _p(pi), _p(v), C.c_int(len(x)))
        return pi, v

    def __del__(self):
        try:
            if self.h:
                lib().or_net_destroy(C.c_void_p(self.h))
                self.h = None
        except Exception:
            pass


def policy_action(net, states):
    """The submission bot's move (yacht/submission/agent.py:248-280) for canonical states: the
    valid (== decodable, agent.py:150-187) action of highest softmax probability, the lowest index
    among equals (its stable descending sort); -1 when none.  Also returns each row's margin to
    the runner-up as a log-probability (= logit) difference (inf with a single valid action)."""
    pi, _ = net.predict_states(states)
    ok, cnt = valid(states, 1)
    p = np.where(ok.astype(bool), pi, -1.0)
    a = p.argmax(1).astype(np.int64)  # first maximum
    top2 = -np.sort(-p, 1)[:, :2]
    with np.errstate(divide="ignore", invalid="ignore"):
        margin = np.where(cnt > 1, np.log(top2[:, 0].astype(np.float64)) - np.log(top2[:, 1].astype(np.float64)),
                          np.inf)
    a[cnt == 0] = -1
    return a, margin


def mcts_prior(pi, states):
    """MCTS.py:86-111 for given predict outputs: P = Ps * valids / np.sum (numpy's float32
    pairwise sum of the masked 3226-vector), the uniform-over-valid fallback when that sum is 0,
    action 0 when nothing is valid.  pi f32[n, 3226], canonical states [n, 8] -> f32[n, 3226]."""
    ok, cnt = valid(states, 1)
    p = np.asarray(pi, dtype=np.float32) * ok.astype(np.float32)
    out = np.zeros_like(p)
    for i in range(len(p)):
        s = pairwise_sum(p[i])
        if s > 0:
            out[i] = p[i] / s
        elif cnt[i] > 0:
            out[i] = ok[i].astype(np.float32) / np.float32(cnt[i])
        else:
            out[i, 0] = 1.0
    return out


MODE_HASH, MODE_MLP, MODE_REPLAY = 0, 1, 2
PLAYERS = {"mcts": 0, "random": 1, "greedy": 2}


def greedy_play(states, seed, envs, ctr=0):
    """GreedyYachtPlayer.play (YachtPlayers.py:199-214) per state, drawing any fallback from the
    state's stream; returns (actions, counters after)."""
    w = _w(states)
    n = len(w)
    e = np.ascontiguousarray(np.broadcast_to(np.asarray(envs, dtype=np.uint32), (n,)))
    c = np.ascontiguousarray(np.broadcast_to(np.asarray(ctr, dtype=np.uint64), (n,))).copy()
    out = np.zeros(n, dtype=np.int32)
    lib().or_greedy_play(_p(w), C.c_uint64(seed), _p(e), _p(c), _p(out), C.c_int(n))
    return out, c


def greedy_heuristic(states):
    """GreedyYachtPlayer's heuristic action for canonical boards (-1: it would fall back to a
    random legal action)."""
    w = _w(states)
    out = np.zeros(len(w), dtype=np.int32)
    lib().or_greedy_heuristic(_p(w), _p(out), C.c_int(len(w)))
    return out


def _replay_ptrs(replay, keep):
    pis = [np.ascontiguousarray(p, dtype=np.float32) for p, _ in replay]
    vs = [np.ascontiguousarray(v, dtype=np.float32) for _, v in replay]
    rn_arr = np.array([len(v) for v in vs], dtype=np.int64)
    keep += pis + vs + [rn_arr]
    n = len(pis)
    return (C.c_void_p * n)(*[p.ctypes.data for p in pis]), (C.c_void_p * n)(*[v.ctypes.data for v in vs]), _p(rn_arr)


def selfplay(envs, seed, sims, cpuct=1.5, temp_threshold=15, mode=MODE_HASH, net=None, replay=None,
             max_moves=64, want_counts=True, threads=1):
    """Coach.executeEpisode for each env id (fresh MCTS per game, Coach.py:93).

    replay: list (per env) of (pi f32[k,3226], v f32[k]) predictions consumed in call order.
    Returns a dict of numpy arrays (see ep_out_t in yk_oracle.c)."""
    e = np.ascontiguousarray(np.asarray(envs, dtype=np.uint32).reshape(-1))
    n = len(e)
    M = max_moves
    canon = np.zeros((n, M, 8), dtype=np.uint64)
    mv = np.zeros((n, M, 8), dtype=np.int32)
    ctr = np.zeros((n, M, 2), dtype=np.uint64)
    counts = np.zeros((n, M, ASIZE), dtype=np.int32) if want_counts else None
    values = np.zeros((n, M), dtype=np.float64)
    stats = np.zeros((n, 8), dtype=np.int64)
    final = np.zeros((n, 8), dtype=np.uint64)
    rpi = rv = rn = None
    keep = []
    if mode == MODE_REPLAY:
        rpi, rv, rn = _replay_ptrs(replay, keep)
    nerr = lib().or_selfplay(n, _p(e), C.c_uint64(seed), sims, C.c_double(cpuct), temp_threshold, M, mode,
                             C.c_void_p(net.h if net is not None else None), rpi, rv, rn,
                             _p(canon), _p(mv), _p(ctr), _p(counts) if counts is not None else None,
                             _p(values), _p(stats), _p(final), threads)
    return dict(canon=canon, mv=mv, ctr=ctr, counts=counts, values=values, stats=stats, final=final,
                nerr=nerr)


def arena(envs, agent_seat, seed, sims, cpuct=1.5, mode=MODE_HASH, net=None, replay=None, max_moves=64,
          threads=1, agent="mcts", opponent="random"):
    """Arena.playGame (Arena.py:30-93): `agent` in seat agent_seat[i] vs `opponent`, each one of
    mcts (temp 0, fresh tree per game), random (RandomYachtPlayer), greedy (GreedyYachtPlayer).
    replay as in selfplay (MODE_REPLAY)."""
    e = np.ascontiguousarray(np.asarray(envs, dtype=np.uint32).reshape(-1))
    n = len(e)
    seat = np.ascontiguousarray(np.broadcast_to(np.asarray(agent_seat, dtype=np.int32), (n,)))
    result = np.zeros(n, dtype=np.float64)
    totals = np.zeros((n, 2), dtype=np.int32)
    actions = np.zeros((n, max_moves), dtype=np.int32)
    stats = np.zeros((n, 8), dtype=np.int64)
    final = np.zeros((n, 8), dtype=np.uint64)
    keep = []
    rpi = rv = rn = None
    if mode == MODE_REPLAY:
        rpi, rv, rn = _replay_ptrs(replay, keep)
    nerr = lib().or_arena(n, _p(e), _p(seat), PLAYERS[agent], PLAYERS[opponent], C.c_uint64(seed), sims,
                          C.c_double(cpuct), max_moves, mode,
                          C.c_void_p(net.h if net is not None else None), rpi, rv, rn, _p(result), _p(totals), _p(actions),
                          _p(stats), _p(final), threads)
    return dict(result=result, totals=totals, actions=actions, stats=stats, final=final, nerr=nerr)


def arena_dual(envs, agent_seat, seed, sims, cpuct=1.5, mode=MODE_HASH, net=None, net2=None, replay=None,
               shared=False, max_moves=64, threads=1):
    """The gating arena of Coach.learn (Coach.py:117-139): MCTS(net, temp 0) in seat agent_seat[i] vs
    MCTS(net2, temp 0), each seat with its own tree.  shared=True keeps both trees across the games,
    played in order, as the reference's pmcts / nmcts live across Arena.playGames; False: fresh trees
    per game.  replay: one (pi, v) log per game holding both seats' expansions in call order."""
    e = np.ascontiguousarray(np.asarray(envs, dtype=np.uint32).reshape(-1))
    n = len(e)
    seat = np.ascontiguousarray(np.broadcast_to(np.asarray(agent_seat, dtype=np.int32), (n,)))
    result = np.zeros(n, dtype=np.float64)
    totals = np.zeros((n, 2), dtype=np.int32)
    actions = np.zeros((n, max_moves), dtype=np.int32)
    stats = np.zeros((n, 8), dtype=np.int64)
    final = np.zeros((n, 8), dtype=np.uint64)
    rpi = rv = rn = None
    keep = []
    if mode == MODE_REPLAY:
        rpi, rv, rn = _replay_ptrs(replay, keep)
    nerr = lib().or_arena_dual(n, _p(e), _p(seat), C.c_uint64(seed), sims, C.c_double(cpuct), max_moves, mode,
                               C.c_void_p(net.h if net is not None else None),
                               C.c_void_p(net2.h if net2 is not None else None), rpi, rv, rn, int(bool(shared)),
                               _p(result), _p(totals), _p(actions), _p(stats), _p(final), threads)
    return dict(result=result, totals=totals, actions=actions, stats=stats, final=final, nerr=nerr)
