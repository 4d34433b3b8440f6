"""Test helper: a referee for two in-process protocol bots (INSTRUCTION.md:10-92).

Each bot is a ``yacht_amd.bot.main`` loop fed line by line through a queue-backed stdin on its
own thread; the referee rolls the bundles, resolves the bids, checks that every PUT uses held
dice and an unused category, and scores both sides independently of the bots' bookkeeping.
"""
from __future__ import annotations

import queue
import threading

import numpy as np


class _Pipe:
    def __init__(self):
        self.q = queue.Queue()

    def __iter__(self):
        while True:
            line = self.q.get()
            if line is None:
                return
            yield line + "\n"


class _Out:
    def __init__(self):
        self.q = queue.Queue()

    def write(self, s):
        for line in s.splitlines():
            self.q.put(line)

    def flush(self):
        pass


class BotProc:
    def __init__(self, ai_player):
        from yacht_amd import bot
        self.inp, self.out = _Pipe(), _Out()
        self.lines_in, self.lines_out = [], []
        self.rc = None

        def run():
            self.rc = bot.main(ai_player, stdin=self.inp, stdout=self.out)
        self.t = threading.Thread(target=run, daemon=True)
        self.t.start()

    def send(self, line, reply):
        self.lines_in.append(line)
        self.inp.q.put(line)
        if reply:
            r = self.out.q.get(timeout=120)
            self.lines_out.append(r)
            return r
        return None

    def close(self):
        self.send("FINISH", False)
        self.inp.q.put(None)
        self.t.join(timeout=60)
        assert self.rc == 0


def play_match(players, seed):
    """Play one match between two AIPlayer objects; returns (totals, bots)."""
    from yacht_amd.bot import rule_score
    from yacht_amd.state import CATEGORIES
    rng = np.random.default_rng(seed)
    bots = [BotProc(p) for p in players]
    for b in bots:
        assert b.send("READY", True) == "OK"
    carry, used, cat, bid = [[], []], [0, 0], [[0] * 12, [0] * 12], [0, 0]
    for rnd in range(1, 14):
        if rnd < 13:
            A, B = [int(x) for x in rng.integers(1, 7, 5)], [int(x) for x in rng.integers(1, 7, 5)]
            sa, sb = "".join(map(str, A)), "".join(map(str, B))
            bids = []
            for b in bots:
                cmd, g, x = b.send(f"ROLL {sa} {sb}", True).split()
                assert cmd == "BID" and g in ("A", "B") and 0 <= int(x) <= 100000
                bids.append((g, int(x)))
            (g0, x0), (g1, x1) = bids
            if g0 != g1:
                got = [g0, g1]
            else:
                win = 0 if x0 > x1 else 1 if x1 > x0 else int(rng.integers(2))
                other = "B" if g0 == "A" else "A"
                got = [g0, other] if win == 0 else [other, g1]
            for i, b in enumerate(bots):
                b.send(f"GET {got[i]} {bids[1 - i][0]} {bids[1 - i][1]}", False)
                carry[i] += A if got[i] == "A" else B
                bid[i] += -bids[i][1] if got[i] == bids[i][0] else bids[i][1]
        if rnd >= 2:
            puts = []
            for i, b in enumerate(bots):
                cmd, c, d = b.send("SCORE", True).split()
                assert cmd == "PUT" and len(d) == 5, (cmd, c, d)
                k = CATEGORIES.index(c)
                assert not (used[i] >> k) & 1, f"category {c} reused"
                dice = [int(v) for v in d]
                left = list(carry[i])
                for v in dice:
                    left.remove(v)  # ValueError if the die is not held
                carry[i] = left
                used[i] |= 1 << k
                cat[i][k] = rule_score(k, dice)
                puts.append((c, d))
            for i, b in enumerate(bots):
                b.send(f"SET {puts[1 - i][0]} {puts[1 - i][1]}", False)
    for b in bots:
        b.close()
    totals = []
    for i in range(2):
        basic = sum(cat[i][:6])
        totals.append(basic + (35000 if basic >= 63000 else 0) + sum(cat[i][6:]) + bid[i])
    assert used == [0xFFF, 0xFFF]
    return totals, bots
