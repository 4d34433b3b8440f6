"""cProfile of bench.py's whole-iteration Coach leg (one Coach.learn iteration at config 5's
per-GPU shape): where the host time of the save / gate phases goes.

    python tools/coach_profile.py [games_per_gpu]
"""
import cProfile
import os
import pstats
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bench  # noqa: E402
from yacht_amd.nnet import YachtNNet  # noqa: E402

games = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
torch.manual_seed(0)
model = YachtNNet(hidden=bench.H, nblocks=bench.NB)
bench.coach_iter_leg(model, 1, games_per_gpu=512, warm=False)  # warm: library load, first allocations
pr = cProfile.Profile()
pr.enable()
out = bench.coach_iter_leg(model, 1, games_per_gpu=games, warm=False)
pr.disable()
print({k: v for k, v in out.items() if k.endswith("_s")})
pstats.Stats(pr).sort_stats("cumulative").print_stats(45)
