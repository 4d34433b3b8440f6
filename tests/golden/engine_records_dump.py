"""Fixtures of the engine's production path (YachtNNet prior, no prediction recording).  usage:
python tests/golden/engine_records_dump.py records OUT.npz   the records of a small self-play batch
python tests/golden/engine_records_dump.py images OUT.npz    packed record images (yk_engine_pack_records)
    of games [0, 3) and [3, 6) ("rank 0" / "rank 1", env ids 0-5) and of all six in one batch:
    tests/golden/engine_images.npz, which the CPU all-gather test (tests/test_dist_cpu.py) pools
(YK_LIB_PATH selects the library)"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "nypc-yacht-auction_amd"))
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


def images(per_rank=3, sims=8, seed=17):
    net = YkNet(spec.closed_form_weights(64, 1), 64, 1)
    out = dict(per_rank=np.int64(per_rank), sims=np.int64(sims), seed=np.int64(seed), max_moves=np.int64(48))
    for name, n, base in (("rank0", per_rank, 0), ("rank1", per_rank, per_rank), ("all", 2 * per_rank, 0)):
        eng = SelfPlayEngine(n, sims, 1.5, 15, net=net, max_moves=48)
        eng.run(seed, base)
        assert eng.stats()["errors"] == 0
        out["img_" + name] = eng.pack_records().cpu().numpy()
        eng.close()
    return out


if __name__ == "__main__":
    what, path = sys.argv[1], sys.argv[2]
    np.savez_compressed(path, **(run() if what == "records" else images()))
    print("wrote", path)
