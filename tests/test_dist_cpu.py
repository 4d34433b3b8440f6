"""Multi-rank trajectory pooling on CPU: world_size 2 over gloo (no GPU).

The images are real engine output (tests/golden/engine_images.npz, written on an MI355X by
tests/golden/engine_records_dump.py images): games 0-2 as "rank 0", games 3-5 as "rank 1", and all six
in one batch.  Each rank all-gathers its image; the pooled examples (helpers.host_examples) must
equal those of the single six-game batch, and every field of every gathered image must come
back intact and in rank order."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    from conftest import GOLDEN, PKG, REPO
    for p in (REPO, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from yacht_amd import dist as D
    from yacht_amd.engine import unpack_record_image
    from helpers import host_examples
    r, w, _ = D.setup(backend="gloo")
    g = np.load(os.path.join(GOLDEN, "engine_images.npz"))
    E, M, sims = int(g["per_rank"]), int(g["max_moves"]), int(g["sims"])
    mine = g[f"img_rank{r}"]
    gathered = D.allgather_records(torch.from_numpy(mine.copy())).numpy()
    intact = []
    for k in range(w):
        a, b = unpack_record_image(gathered[k], E, M, sims), unpack_record_image(g[f"img_rank{k}"], E, M, sims)
        intact.append(all(np.array_equal(a[f], b[f]) for f in a))
    pooled = host_examples(gathered, E, M, sims)
    single = host_examples(g["img_all"], 2 * E, M, sims)
    same = all(np.array_equal(pooled[k], single[k]) for k in single)
    trimmed = host_examples(gathered, E, M, sims, n_games=4)
    _, lo, hi = D.shard(2 * E, r, w)
    q.put((r, intact, same, len(pooled["targets"]), len(trimmed["targets"]), (lo, hi),
           D.allreduce_counts([r + 1, 10])))
    dist.destroy_process_group()


def test_allgather_engine_images_two_ranks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r, intact, same, n, n4, span, tally in res:
        assert intact == [True, True]   # every field of both images, in rank order
        assert same                     # pooled examples == the single six-game batch
        assert n == 6 * 48 and n4 == 4 * 48
        assert span == (3 * r, 3 * r + 3)
        assert tally == [3, 20]


def test_host_examples_of_the_fixture():
    """The pooled examples' content: 48 per game, temp 1 for the first 14 moves (tempThreshold
    15, Coach.py:58), pi summing to 1, the target the argmax of pi."""
    from conftest import GOLDEN
    from helpers import host_examples
    g = np.load(os.path.join(GOLDEN, "engine_images.npz"))
    h = host_examples(g["img_all"], 2 * int(g["per_rank"]), int(g["max_moves"]), int(g["sims"]))
    n = len(h["targets"])
    assert n == 6 * 48
    sums = np.add.reduceat(h["pi_vals"], h["pi_indptr"][:-1])
    assert np.allclose(sums, 1.0, rtol=0, atol=1e-12)
    lens = np.diff(h["pi_indptr"])
    move = np.arange(n) % 48
    assert (lens[move >= 14] == 1).all() and (lens[move < 14] >= 1).all() and (lens[move < 14] > 1).any()
    for k in range(n):
        a0, a1 = h["pi_indptr"][k], h["pi_indptr"][k + 1]
        cols, vals = h["pi_cols"][a0:a1], h["pi_vals"][a0:a1]
        assert h["targets"][k] == cols[np.argmax(vals)]
    assert set(np.unique(np.abs(h["values"]))) <= {1.0, 1e-4}
