"""Diagnostic / regression fixture: the records of a small self-play batch with the YachtNNet
prior and no prediction recording (the engine's production path).  usage:
python tools/engine_records_dump.py OUT.npz   (YK_LIB_PATH selects the library)"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nypc-yacht-auction_amd"))
from oracle import spec  # noqa: E402
from yacht_amd.engine import SelfPlayEngine  # noqa: E402
from yacht_amd.nnet import YkNet  # noqa: E402


def run(n=64, sims=16, seed=5):
    eng = SelfPlayEngine(n, sims, 1.5, 15, net=YkNet(spec.closed_form_weights(256, 6), 256, 6), max_moves=64)
    eng.run(seed, 0)
    st = eng.stats()
    assert st["errors"] == 0, st
    r = eng.records()
    eng.close()
    return {k: r[k] for k in ("info", "values", "n_moves", "visits", "visits_off", "final")}


if __name__ == "__main__":
    np.savez_compressed(sys.argv[1], **run())
    print("wrote", sys.argv[1])
