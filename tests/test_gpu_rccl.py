"""The RCCL branches of yacht_amd/dist.py, executed on the one GPU of the box: a process group
of world size 1 over backend "nccl" (RCCL on ROCm).  The collectives short-circuit only when no
group exists, so every device-side call the 8-GPU run issues is made here once:

* allgather_records - `all_gather_into_tensor` of a real engine record image (uint8), which
  must come back byte for byte, and the Coach's sharded self-play through it
  (Coach.selfPlayExamples, Coach.py:88-101's pooling) equal to the same call without a group;
* allreduce_grads - the in-place `all_reduce` of the native trainer's flat f32 gradient buffer
  (DDP, NNet.py:118-174's step), unweighted and share-weighted, bit for bit;
* allreduce_counts - the int64 device tally of the gating arena (Coach.py:123-139), including
  values past 2^32, and the sharded GatingArena through it equal to the run without a group.

World size 1 makes each expected value exact (a sum over one rank), so the checks are equality,
not tolerance."""
import os
import socket

import numpy as np
import pytest

from oracle import spec

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


ARGS = dict(numIters=1, numEps=6, tempThreshold=15, updateThreshold=0.55, maxlenOfQueue=200000, numMCTSSims=4,
            arenaCompare=4, cpuct=1.5, numItersForTrainExamplesHistory=5, lr=2e-3, weight_decay=1e-4, epochs=1,
            batch_size=64, vloss_weight=1.5, cuda=True, hidden=64, nblocks=1, dropout=0.0, seed=3)


def _worker(_index, port, out):  # (start_processes passes the process index first)
    import sys
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (here, os.path.join(here, "nypc-yacht-auction_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    torch.cuda.set_device(0)
    from yacht_amd import dist as D
    from yacht_amd import kernels as K
    from yacht_amd.arena import GatingArena
    from yacht_amd.coach import Coach
    from yacht_amd.engine import SelfPlayEngine
    from yacht_amd.game import YachtGame
    from yacht_amd.nnet import NNetWrapper, YkNet
    from yacht_amd.train import Trainer
    from yacht_amd.utils import dotdict

    # ---- references, computed before any process group exists (the short-circuit paths)
    eng = SelfPlayEngine(5, 6, 1.5, 15, net=YkNet(spec.closed_form_weights(64, 1), 64, 1), max_moves=48)
    eng.run(17, 40)
    img = eng.pack_records()
    eng.close()
    args = dotdict(ARGS, checkpoint="/tmp/yk_rccl_ck", load_folder_file=("/tmp/yk_rccl_ck", "x"))
    torch.manual_seed(5)
    game = YachtGame(seed=21, env_id=500)
    coach = Coach(game, NNetWrapper(game, args), args)
    ref_ex = coach.selfPlayExamples(args.numEps)
    ref_ex = [t.cpu().clone() for t in (ref_ex.states, ref_ex.targets, ref_ex.values)]
    other = NNetWrapper(game, args)
    ref_pit = GatingArena(game, coach.nnet, other, args).playGames(args.arenaCompare, env_base=900)
    sd = {k: torch.tensor(np.asarray(v, dtype=np.float32)) for k, v in spec.closed_form_weights(64, 1).items()}
    states = np.load(os.path.join(here, "tests", "golden", "states.npz"))["states"][:48]
    rng = np.random.RandomState(3)
    tg = torch.tensor(rng.randint(0, 3226, 48).astype(np.int32), device="cuda")
    vv = torch.tensor((rng.rand(48) * 2 - 1).astype(np.float32), device="cuda")

    # ---- the RCCL group: world size 1 on cuda:0
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        out["backend"] = str(dist.get_backend())
        g = D.allgather_records(img)
        out["gather"] = (tuple(g.shape), g.dtype == torch.uint8, g.is_cuda,
                         bool(torch.equal(g.reshape(-1), img.reshape(-1))), int(img.numel()))
        tr = Trainer(sd, 64, 1, max_batch=48, dropout=0.0, seed=5)
        tr.backward(K.states_to_device(states), tg, vv)
        g0 = tr.grads().clone()
        D.allreduce_grads(tr)
        same_mean = torch.equal(tr.grads().view(torch.int32), g0.view(torch.int32))
        D.allreduce_grads(tr, weight=0.25)
        same_weighted = torch.equal(tr.grads().view(torch.int32), (g0 * 0.25).view(torch.int32))
        out["grads"] = (same_mean, same_weighted, int(g0.numel()), bool(g0.abs().sum() > 0))
        out["counts"] = D.allreduce_counts([3, 2 ** 40 + 7, -5], device="cuda")
        torch.manual_seed(5)
        coach2 = Coach(game, NNetWrapper(game, args), args)
        ex = coach2.selfPlayExamples(args.numEps)
        out["examples"] = all(torch.equal(a, b.cpu()) for a, b in zip(ref_ex, (ex.states, ex.targets, ex.values)))
        out["n_examples"] = len(ex)
        out["pit"] = (tuple(ref_pit), tuple(GatingArena(game, coach2.nnet, other, args).playGames(args.arenaCompare,
                                                                                               env_base=900)))
    finally:
        dist.destroy_process_group()


def test_rccl_world1_collectives_on_device():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.multiprocessing as mp
    mgr = mp.get_context("spawn").Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(_free_port(), out), nprocs=1, start_method="spawn")
    assert out["backend"] == "nccl"
    shape, u8, cuda, same, n = out["gather"]
    assert shape == (1, n) and u8 and cuda and same
    same_mean, same_weighted, ng, nonzero = out["grads"]
    assert nonzero and ng > 100_000 and same_mean and same_weighted
    assert out["counts"] == [3, 2 ** 40 + 7, -5]
    assert out["examples"] and out["n_examples"] == 6 * 48
    assert out["pit"][0] == out["pit"][1] and sum(out["pit"][0]) == 4
