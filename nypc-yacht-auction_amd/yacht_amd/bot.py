"""Competition bot: the stdin/stdout agent of yacht/submission/agent.py on the
MI355X, speaking the I/O protocol of INSTRUCTION.md:76-92.

    python -m yacht_amd.bot --model checkpoint.pth.tar [--sims N]

Commands (one per line):  READY -> ``OK``;  ``ROLL a1..a5 b1..b5`` -> ``BID g x``;
``GET g g0 x0`` (no output);  SCORE -> ``PUT c d1..d5``;  ``SET c d1..d5`` (no output);
FINISH -> exit.  The bookkeeping follows the reference agent exactly, including its quirks,
because they decide the network's input:

* the round counter advances after GET in round 1 and after SET in rounds 2-12
  (agent.py:602-625);
* ``use_dice`` removes the played dice from the carry *by value*, the first equal die each
  (agent.py:484-495) - the game removes by position, so the carry order (and with it the
  feature vector) can differ from self-play's;
* the network input is ``state_to_vec`` of the board with "me" as player 1
  (agent.py:108-147 == NNet.py:65-86), rolls shown only in a bidding phase.

The move (``AIPlayer.get_move``, agent.py:238-303) is the most probable decodable action of the
network's softmax, ties to the lowest index - computed on the GPU by ``yk_net_policy_action``
(featurize + forward + masked argmax in two launches).  With ``--sims N`` the bot instead plays
``argmax(getActionProb(board, temp=0))`` of an N-simulation MCTS on the engine (the Arena's
MCTS player, Coach.py:124-125) - an extension, not in the reference bot.

When the model file is missing the reference falls back to a fixed minimal move (``BID A 0``;
the first unused category with the first five carried dice, agent.py:370-397); this mirror does
the same.  A missing HIP library is an error, never a silent fallback.
"""
from __future__ import annotations

import argparse
import os
import sys
from dataclasses import dataclass
from enum import Enum
from typing import Callable, List, Optional

import numpy as np

from .state import (BID_STEP, COMB_5_OF_10, NUM_BID_ACTIONS, NUM_CATEGORIES, PlayerState, YachtState,
                    decode_bid_action, decode_score_action, pack)


class DiceRule(Enum):  # agent.py:306-319 (the game's category order)
    ONE = 0
    TWO = 1
    THREE = 2
    FOUR = 3
    FIVE = 4
    SIX = 5
    CHOICE = 6
    FOUR_OF_A_KIND = 7
    FULL_HOUSE = 8
    SMALL_STRAIGHT = 9
    LARGE_STRAIGHT = 10
    YACHT = 11


@dataclass
class Bid:  # agent.py:322-326
    group: str
    amount: int


@dataclass
class DicePut:  # agent.py:329-333
    rule: DiceRule
    dice: List[int]


def rule_score(cat: int, dice: List[int]) -> int:
    """Score of five dice in category `cat` (INSTRUCTION.md:44-70; score_category, YachtGame.py:57-104)."""
    cnt = [0] * 7
    for d in dice:
        cnt[d] += 1
    total = 1000 * sum(dice)
    if cat < 6:
        return 1000 * (cat + 1) * cnt[cat + 1]
    if cat == 6:
        return total
    if cat == 7:
        return total if max(cnt) >= 4 else 0
    if cat == 8:  # five of a kind counts as both the pair and the triple
        pair = any(c in (2, 5) for c in cnt)
        triple = any(c in (3, 5) for c in cnt)
        return total if pair and triple else 0
    has = [cnt[v] > 0 for v in range(7)]
    if cat == 9:
        return 15000 if any(all(has[v:v + 4]) for v in (1, 2, 3)) else 0
    if cat == 10:
        return 30000 if all(has[1:6]) or all(has[2:7]) else 0
    if cat == 11:
        return 50000 if max(cnt) == 5 else 0
    raise ValueError(f"invalid category {cat}")


class GameState:
    """One side's holdings (agent.py:446-561): carried dice, used categories, scores, bid total."""

    def __init__(self):
        self.carry: List[int] = []
        self.used_mask = 0
        self.cat_scores = [0] * NUM_CATEGORIES
        self.bid_score = 0

    @property
    def rule_score(self):
        return [self.cat_scores[i] if (self.used_mask >> i) & 1 else None for i in range(NUM_CATEGORIES)]

    def get_total_score(self) -> int:
        basic = sum(self.cat_scores[:6])
        return basic + (35000 if basic >= 63000 else 0) + sum(self.cat_scores[6:]) + self.bid_score

    def bid(self, is_successful: bool, amount: int):
        self.bid_score += -amount if is_successful else amount

    def add_dice(self, new_dice: List[int]):
        self.carry.extend(new_dice)

    def use_dice(self, put: DicePut):
        cat = put.rule.value
        if (self.used_mask >> cat) & 1:
            raise ValueError(f"rule {put.rule.name} already used")
        left = list(self.carry)
        for d in put.dice:  # by value: the first remaining equal die (agent.py:484-495)
            if d in left:
                left.remove(d)
        self.carry = left
        self.used_mask |= 1 << cat
        self.cat_scores[cat] = self.calculate_score(put)

    @staticmethod
    def calculate_score(put: DicePut) -> int:
        return rule_score(put.rule.value, list(put.dice))

    def player_state(self) -> PlayerState:
        return PlayerState(carry=list(self.carry), used_mask=self.used_mask, cat_scores=list(self.cat_scores),
                           bid_score=self.bid_score)


def board_of(game: "Game") -> YachtState:
    """The bot's view as a canonical board (me = p1).  Bids are not features; rolls are shown only
    while bidding (NNet.py:76-77), so they are kept only in phase 0."""
    rolls = game.phase == 0
    return YachtState(round_no=game.round_no, phase=game.phase, rollA=list(game.rollA) if rolls else [],
                      rollB=list(game.rollB) if rolls else [], p1=game.my_state.player_state(),
                      p2=game.opp_state.player_state())


def decode_action(a: int, game: "Game"):
    """Action index -> Bid / DicePut (agent.py:150-187); None when not decodable."""
    if a is None or a < 0:
        return None
    if game.phase == 0:
        if a >= NUM_BID_ACTIONS:
            return None
        g, amount = decode_bid_action(a)
        return Bid(g, amount)
    if a < NUM_BID_ACTIONS:
        return None
    cat, comb = decode_score_action(a)
    carry = game.my_state.carry
    if (game.my_state.used_mask >> cat) & 1 or len(carry) < 5 or max(comb) >= len(carry):
        return None
    return DicePut(DiceRule(cat), [carry[i] for i in comb])


class AIPlayer:
    """Network player (agent.py:190-303).  ``policy`` (packed board -> action index) replaces the
    network, for tests; otherwise the model file's network runs on the GPU."""

    def __init__(self, model_path: Optional[str] = None, sims: int = 0, cpuct: float = 1.5, seed: int = 0,
                 policy: Optional[Callable[[np.ndarray], int]] = None, log=None):
        self.policy = policy
        self.sims, self.cpuct, self.seed = sims, cpuct, seed
        self.log = log if log is not None else sys.stderr
        self.model = None
        self._mcts = None
        if policy is None and model_path is not None:
            self.load_model(model_path)

    def load_model(self, model_path: str):
        """Reference checkpoint dict ({"state_dict", "args"}, NNet.py:198-205), loaded without
        unpickling code (agent.py:198-221 reads the same dict)."""
        if not os.path.exists(model_path):
            print(f"Model file {model_path} not found, using fallback AI", file=self.log)
            return
        import torch
        from .nnet import YkNet
        ck = torch.load(model_path, map_location="cpu", weights_only=True)
        args = ck.get("args", {}) if isinstance(ck, dict) else {}
        sd = ck["state_dict"] if "state_dict" in ck else ck
        self.hidden, self.nblocks = int(args.get("hidden", 512)), int(args.get("nblocks", 8))
        self.state_dict = sd
        self.model = YkNet(sd, self.hidden, self.nblocks)
        print("AI model loaded successfully", file=self.log)

    def _mcts_action(self, board: YachtState) -> int:
        import torch
        if self._mcts is None:
            from .game import YachtGame
            from .mcts import MCTS
            from .nnet import NNetWrapper, DEFAULT_ARGS
            from .utils import dotdict
            args = dotdict(dict(DEFAULT_ARGS))
            args.update(hidden=self.hidden, nblocks=self.nblocks)
            nnet = NNetWrapper(YachtGame(self.seed), args)
            with torch.no_grad():
                nnet.nnet.load_state_dict(self.state_dict)
            self._mcts = MCTS(nnet.game, nnet, dotdict(dict(numMCTSSims=self.sims, cpuct=self.cpuct)))
        return int(np.argmax(self._mcts.getActionProb(board, temp=0)))

    def action(self, board: YachtState) -> int:
        if self.policy is not None:
            return int(self.policy(pack(board)))
        if self.model is None:
            return -1
        if self.sims > 0:
            return self._mcts_action(board)
        from . import kernels as K
        a, _ = self.model.policy_action(K.states_to_device(pack(board)))
        return int(a.item())

    def get_move(self, game: "Game", round_no, phase, rollA, rollB, p1_bid, p2_bid, current_player):
        if self.policy is None and self.model is None:
            return None
        return decode_action(self.action(board_of(game)), game)


class Game:
    """The agent's view of one match (agent.py:335-443)."""

    def __init__(self, ai_player: Optional[AIPlayer] = None):
        self.my_state = GameState()
        self.opp_state = GameState()
        self.ai_player = ai_player if ai_player is not None else AIPlayer()
        self.round_no = 1
        self.phase = 0
        self.rollA: List[int] = []
        self.rollB: List[int] = []
        self.p1_bid = ("", 0)
        self.p2_bid = ("", 0)

    def calculate_bid(self, dice_a: List[int], dice_b: List[int]) -> Bid:
        self.rollA, self.rollB, self.phase = list(dice_a), list(dice_b), 0
        move = self.ai_player.get_move(self, self.round_no, 0, self.rollA, self.rollB, self.p1_bid, self.p2_bid, 1)
        return move if isinstance(move, Bid) else Bid("A", 0)

    def calculate_put(self) -> DicePut:
        self.phase = 1
        move = self.ai_player.get_move(self, self.round_no, 1, self.rollA, self.rollB, self.p1_bid, self.p2_bid, 1)
        if isinstance(move, DicePut):
            return move
        rule = next((c for c in range(NUM_CATEGORIES) if not (self.my_state.used_mask >> c) & 1), 0)
        return DicePut(DiceRule(rule), self.my_state.carry[:5])

    def update_get(self, dice_a, dice_b, my_bid: Bid, opp_bid: Bid, my_group: str):
        self.p1_bid, self.p2_bid = (my_bid.group, my_bid.amount), (opp_bid.group, opp_bid.amount)
        mine, theirs = (dice_a, dice_b) if my_group == "A" else (dice_b, dice_a)
        self.my_state.add_dice(list(mine))
        self.opp_state.add_dice(list(theirs))
        opp_group = "B" if my_group == "A" else "A"
        self.my_state.bid(my_bid.group == my_group, my_bid.amount)
        self.opp_state.bid(opp_bid.group == opp_group, opp_bid.amount)

    def update_put(self, put: DicePut):
        self.my_state.use_dice(put)

    def update_set(self, put: DicePut):
        self.opp_state.use_dice(put)

    def advance_round(self):
        self.round_no += 1
        self.p1_bid = self.p2_bid = ("", 0)


def _dice(s: str) -> List[int]:
    return [int(c) for c in s]


def main(ai_player: Optional[AIPlayer] = None, stdin=None, stdout=None, log=None) -> int:
    """The protocol loop (agent.py:564-636); returns the exit status."""
    stdin = stdin if stdin is not None else sys.stdin
    stdout = stdout if stdout is not None else sys.stdout
    log = log if log is not None else sys.stderr
    game = Game(ai_player)
    dice_a, dice_b = [0] * 5, [0] * 5
    my_bid = Bid("", 0)

    def say(line: str):
        stdout.write(line + "\n")
        stdout.flush()

    for raw in stdin:
        line = raw.strip()
        if not line:
            continue
        cmd, *args = line.split()
        if cmd == "READY":
            say("OK")
        elif cmd == "ROLL":
            dice_a, dice_b = _dice(args[0]), _dice(args[1])
            my_bid = game.calculate_bid(dice_a, dice_b)
            say(f"BID {my_bid.group} {my_bid.amount}")
        elif cmd == "GET":
            get_group, opp_group, opp_score = args
            game.update_get(dice_a, dice_b, my_bid, Bid(opp_group, int(opp_score)), get_group)
            if game.round_no == 1:  # round 1 has no scoring
                game.advance_round()
        elif cmd == "SCORE":
            put = game.calculate_put()
            game.update_put(put)
            say(f"PUT {put.rule.name} {''.join(map(str, put.dice))}")
        elif cmd == "SET":
            rule, dice = args
            game.update_set(DicePut(DiceRule[rule], _dice(dice)))
            if 2 <= game.round_no <= 12:
                game.advance_round()
        elif cmd == "FINISH":
            break
        else:
            print(f"Invalid command: {cmd}", file=log)
            return 1
    return 0


def cli(argv=None) -> int:
    ap = argparse.ArgumentParser(description="Yacht Auction competition bot (MI355X)")
    ap.add_argument("--model", default="data.bin", help="reference-format checkpoint (state_dict + args)")
    ap.add_argument("--sims", type=int, default=0, help="MCTS simulations per move (0: policy argmax, as agent.py)")
    ap.add_argument("--cpuct", type=float, default=1.5)
    ap.add_argument("--seed", type=int, default=0, help="MCTS chance-node stream seed")
    a = ap.parse_args(argv)
    return main(AIPlayer(a.model, sims=a.sims, cpuct=a.cpuct, seed=a.seed))


if __name__ == "__main__":
    sys.exit(cli())

__all__ = ["DiceRule", "Bid", "DicePut", "GameState", "Game", "AIPlayer", "main", "cli", "rule_score", "board_of",
           "decode_action", "BID_STEP", "COMB_5_OF_10"]
