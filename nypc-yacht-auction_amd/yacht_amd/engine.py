"""SelfPlayEngine: batched Coach.executeEpisode on one GPU (yk_selfplay).

One ``run`` plays a complete episode for every one of ``n_envs`` games in lock-step:
48 real moves x ``sims`` MCTS simulations each, all on the device (include/yacht_hip.h).
Game i uses the RNG stream ``(seed, env_base + i)``; trees are fresh per episode
(Coach.py:93).  Records come back as numpy arrays or as one packed device buffer for the
multi-GPU all-gather (``yacht_amd.dist``).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from ._lib import YkEngineConfig, call, lib, stream_ptr

ACTION_SIZE = 3226


class SelfPlayEngine:
    def __init__(self, n_envs: int, sims: int, cpuct: float = 1.5, temp_threshold: int = 15, net=None,
                 prior: str = "net", max_moves: int = 64, record_predictions: bool = False,
                 max_expansions: int = 0, arena_entries: int = 0, record_stride: int = 1, groups: int = 0,
                 dual_trees: bool = False, opponent_net=None):
        if prior not in ("net", "hash"):
            raise ValueError("prior is 'net' (YachtNNet on MFMA) or 'hash' (deterministic test prior)")
        if prior == "net" and net is None:
            raise ValueError("prior='net' needs a YkNet")
        self.cfg = YkEngineConfig(n_envs=n_envs, sims=sims, cpuct=cpuct, temp_threshold=temp_threshold,
                                  max_moves=max_moves, prior=0 if prior == "net" else 1,
                                  record_predictions=int(record_predictions),
                                  max_expansions=max_expansions or (max_moves * sims + 8),
                                  arena_entries=arena_entries, record_stride=max(int(record_stride), 1),
                                  groups=int(groups), dual_trees=int(bool(dual_trees)))
        self.net = net  # keep the weights alive
        h = C.c_void_p()
        call("yk_engine_create", C.byref(h), C.byref(self.cfg), C.c_void_p(net.handle if net is not None else None))
        self.handle = h.value
        self.n_envs, self.sims, self.max_moves = n_envs, sims, max_moves
        self.opponent_net = opponent_net
        if opponent_net is not None:
            # MCTS vs MCTS with two nets, each seat its own tree (the gating arena, Coach.py:117-139)
            call("yk_engine_set_opponent_net", self.handle, C.c_void_p(opponent_net.handle))

    ERROR_BITS = {1: "node pool", 2: "edge pool", 4: "arena", 8: "search depth", 16: "transition status",
                  32: "root round went backwards", 64: "visit records", 128: "move cap", 256: "zero visit counts",
                  512: "root not in tree", 1024: "hash index full", 2048: "forward hand-off timed out"}

    def run(self, seed: int, env_base: int = 0, stream=None):
        from ._lib import YkError
        try:
            call("yk_selfplay", self.handle, seed & (2**64 - 1), env_base & (2**32 - 1), stream_ptr(stream))
        except YkError as e:
            st = self.stats()
            bits = [n for b, n in self.ERROR_BITS.items() if st["errors"] & b]
            raise YkError(f"yk_selfplay [{', '.join(bits)}; stats {st}]", e.code) from None

    PLAYERS = {"mcts": 0, "random": 1, "greedy": 2}  # YK_PLAYER_*

    def arena(self, agent_seat, seed: int, env_base: int = 0, stream=None, agent: str = "mcts",
              opponent: str = "random"):
        """Batched Arena.playGame (yk_arena): `agent` in seat agent_seat[i] against `opponent`,
        each "mcts" (temp 0, this engine's net / prior and sims), "random" or "greedy"; game i
        uses stream (seed, env_base + i)."""
        from ._lib import YkError
        seat = np.ascontiguousarray(np.broadcast_to(np.asarray(agent_seat, dtype=np.int32), (self.n_envs,)))
        try:
            call("yk_arena", self.handle, seed & (2**64 - 1), env_base & (2**32 - 1), seat.ctypes.data,
                 self.PLAYERS[agent], self.PLAYERS[opponent], stream_ptr(stream))
        except YkError as e:
            st = self.stats()
            bits = [n for b, n in self.ERROR_BITS.items() if st["errors"] & b]
            raise YkError(f"yk_arena [{', '.join(bits)}; stats {st}]", e.code) from None

    def arena_results(self) -> dict:
        E, M = self.n_envs, self.max_moves
        result = np.zeros(E, dtype=np.float64)
        totals = np.zeros((E, 2), dtype=np.int32)
        nm = np.zeros(E, dtype=np.int32)
        actions = np.zeros((E, M), dtype=np.int32)
        final = np.zeros((E, 8), dtype=np.uint64)
        ctr = np.zeros(E, dtype=np.uint64)
        call("yk_arena_results", self.handle, result.ctypes.data, totals.ctypes.data, nm.ctypes.data,
             actions.ctypes.data, final.ctypes.data, ctr.ctypes.data)
        return dict(result=result, totals=totals, n_moves=nm, actions=actions, final=final, ctr=ctr)

    # class 0: the first descent of each move; class 3: expand + backup + the next descent
    KERNEL_CLASSES = ("select", "forward", "root_sort_select", "expand_backup_select", "move_begin", "move_end")

    def profile(self, enable: bool = True, stride: int = 1):
        """Per-kernel HIP event timing; the forward / expand pair of every `stride`-th simulation."""
        call("yk_engine_profile", self.handle, int(stride) if enable else 0)

    def kernel_times(self) -> dict:
        ms = np.zeros(8, dtype=np.float64)
        n = np.zeros(8, dtype=np.int64)
        call("yk_engine_kernel_times", self.handle, ms.ctypes.data, n.ctypes.data)
        return {k: (float(ms[i]), int(n[i])) for i, k in enumerate(self.KERNEL_CLASSES) if k != "unused"}

    STAT_NAMES = ("expansions", "scanned", "moves", "errors", "max_nodes", "max_edges", "max_arena", "vnew",
                  "path_edges", "sims", "node_cap", "edge_cap", "arena_cap", "visit_cap", "groups",
                  "forward_parts")
    COUNTER_NAMES = ("scan_edges",)  # yk_engine_counters

    def stats(self) -> dict:
        out = np.zeros(16, dtype=np.int64)
        call("yk_engine_stats", self.handle, out.ctypes.data)
        st = {k: int(out[i]) for i, k in enumerate(self.STAT_NAMES)}
        more = np.zeros(len(self.COUNTER_NAMES), dtype=np.int64)
        if hasattr(lib(), "yk_engine_counters"):  # (absent only from older diagnostic baselines)
            call("yk_engine_counters", self.handle, more.ctypes.data, len(more))
        st.update({k: int(more[i]) for i, k in enumerate(self.COUNTER_NAMES)})
        return st

    def records(self) -> dict:
        E, M = self.n_envs, self.max_moves
        states = np.zeros((E, M, 8), dtype=np.uint64)
        info = np.zeros((E, M, 8), dtype=np.int32)
        ctr = np.zeros((E, M, 2), dtype=np.uint64)
        values = np.zeros((E, M), dtype=np.float64)
        final = np.zeros((E, 8), dtype=np.uint64)
        nm = np.zeros(E, dtype=np.int32)
        nv = np.zeros(1, dtype=np.int64)
        call("yk_engine_records", self.handle, None, None, None, None, None, None, None, None, nv.ctypes.data)
        voff = np.zeros(E * M + 1, dtype=np.int64)
        visits = np.zeros((max(int(nv[0]), 1), 2), dtype=np.int32)
        call("yk_engine_records", self.handle, states.ctypes.data, info.ctypes.data, ctr.ctypes.data,
             values.ctypes.data, final.ctypes.data, nm.ctypes.data, voff.ctypes.data, visits.ctypes.data,
             nv.ctypes.data)
        return dict(states=states, info=info, ctr=ctr, values=values, final=final, n_moves=nm,
                    visits_off=voff.reshape(-1)[:E * M + 1], visits=visits[:int(nv[0])])

    def predictions(self, leaves: bool = False):
        """(pi, v, count[, leaves]) of the recorded games (every record_stride-th): pi[r, k] is
        Ps * valids of game r * record_stride's k-th expansion (MCTS.py:86-88, before the
        renormalisation), exactly what the search used; count[r] its expansions."""
        R = (self.n_envs + self.cfg.record_stride - 1) // self.cfg.record_stride
        X = self.cfg.max_expansions
        pi = np.zeros((R, X, ACTION_SIZE), dtype=np.float32)
        v = np.zeros((R, X), dtype=np.float32)
        lv = np.zeros((R, X, 8), dtype=np.uint64) if leaves else None
        cnt = np.zeros(R, dtype=np.int32)
        call("yk_engine_predictions", self.handle, pi.ctypes.data, v.ctypes.data,
             lv.ctypes.data if leaves else None, cnt.ctypes.data)
        if (cnt > X).any():
            raise RuntimeError(f"prediction record truncated: {int(cnt.max())} expansions > max_expansions {X}")
        return (pi, v, cnt, lv) if leaves else (pi, v, cnt)

    def record_bytes(self) -> int:
        n = int(lib().yk_engine_record_bytes(self.handle))
        if n < 0:
            raise RuntimeError("yk_engine_record_bytes failed")
        return n

    def pack_records(self, out: torch.Tensor = None, stream=None) -> torch.Tensor:
        nb = self.record_bytes()
        if out is None:
            out = torch.empty(nb, dtype=torch.uint8, device="cuda")
        call("yk_engine_pack_records", self.handle, out.data_ptr(), out.numel(), stream_ptr(stream))
        return out

    def close(self):
        if getattr(self, "handle", None):
            lib().yk_engine_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def unpack_record_image(buf: np.ndarray, n_envs: int, max_moves: int, sims: int) -> dict:
    """Inverse of yk_engine_pack_records (host bytes of one rank's image)."""
    E, M = n_envs, max_moves
    vcap = 2 * M * max(sims, 32)
    parts = [("states", np.uint64, (E, M, 8)), ("info", np.int32, (E, M, 8)), ("ctr", np.uint64, (E, M, 2)),
             ("values", np.float64, (E, M)), ("visits_raw", np.uint32, (E, vcap)), ("voff", np.int32, (E, M + 1)),
             ("n_moves", np.int32, (E,)), ("final", np.uint64, (E, 8))]
    out, off = {}, 0
    raw = np.ascontiguousarray(buf).view(np.uint8)
    for name, dt, shape in parts:
        nb = int(np.prod(shape)) * np.dtype(dt).itemsize
        out[name] = raw[off:off + nb].view(dt).reshape(shape)
        off += (nb + 15) & ~15
    return out
