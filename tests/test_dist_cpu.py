"""Multi-rank trajectory pooling on CPU: world_size 2 over gloo (no GPU)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_envs, max_moves, sims, q):
    import sys
    from conftest import PKG, REPO
    for p in (REPO, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from yacht_amd import dist as D
    from yacht_amd.engine import unpack_record_image
    r, w, _ = D.setup(backend="gloo")
    # a synthetic record image laid out like yk_engine_pack_records, tagged by rank
    E, M = n_envs, max_moves
    vcap = 2 * M * max(sims, 32)
    parts = [(np.uint64, (E, M, 8)), (np.int32, (E, M, 8)), (np.uint64, (E, M, 2)), (np.float64, (E, M)),
             (np.uint32, (E, vcap)), (np.int32, (E, M + 1)), (np.int32, (E,)), (np.uint64, (E, 8))]
    chunks = []
    for dt, shape in parts:
        a = np.full(shape, r + 1, dtype=dt).view(np.uint8).reshape(-1)
        pad = (-a.size) % 16
        chunks.append(np.concatenate([a, np.zeros(pad, dtype=np.uint8)]))
    buf = torch.from_numpy(np.concatenate(chunks))
    g = D.allgather_records(buf)
    rb = D.ReplayBuffer()
    rb.add_gathered(g, E, M, sims)
    imgs = rb.batches[0]
    q.put((r, [int(img["n_moves"][0]) for img in imgs], rb.num_examples(), D.env_base(r, E)))
    dist.destroy_process_group()


def test_allgather_records_two_ranks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, 3, 4, 8, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r, nm, nex, base in res:
        assert nm == [1, 2]           # rank order preserved, each rank's image intact
        assert nex == 3 * 1 + 3 * 2   # n_moves summed over both ranks' games
        assert base == r * 3          # global env ids: rank-independent streams
