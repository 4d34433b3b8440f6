#!/usr/bin/env python3
"""Benchmark: batched Yacht Auction self-play on MI355X.

One step = one complete self-play episode batch: ``--envs`` games (default 4096) per GPU,
each running ``--sims`` (default 100) MCTS simulations per real move over all 48 moves
(Coach.executeEpisode -> MCTS.getActionProb -> MCTS.search, all on the GPU), followed by
the RCCL all-gather of the trajectory records when N > 1.

Metric (BASELINE.json): MCTS node-expansions/sec (one expansion = one NNetWrapper.predict
of the reference = one new MCTS.Ps entry), whole job, plus episodes/s.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

`python bench.py --gpus N` (N > 1) with no launcher environment starts the N ranks itself
(spawn_ranks: one fresh process per GPU, torchrun's environment contract) and relays rank 0's
line; under torch.distributed.run each rank runs main() directly.

Prints ONE JSON line on rank 0.  Data: synthetic (games from seeded streams), random-init
YachtNNet (kaiming-uniform per YachtNNet._init, seed 0, hidden 256, 6 blocks).
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "nypc-yacht-auction_amd"))
sys.path.insert(0, REPO)

METRIC = "MCTS node-expansions/sec/GPU @4096 envs x100 sims; episodes/sec 1-8 GPU"
F16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense f16 matrix peak (~2.5 PF)
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E spec peak
H, NB, A = 256, 6, 3226
# k_forward runs each f32 product as fp16 MFMA products on hi / lo planes: four in the input layer,
# the trunk and the value head (hi.hi, hi.lo, lo.hi, (lo 2^-11).lo), three in the policy head (no
# lo.lo: yk_fwd.h pi_chunk).  The f32-equivalent peak the forward's algorithmic FLOPs are priced
# against is the f16 dense peak over the FLOP-weighted product count (the full 3226-wide head).
_TRUNK_MAC, _HEAD_MAC = 59 * H + 2 * NB * H * H + H * 128 + 128, H * A
SPLIT_PRODUCTS = (4 * _TRUNK_MAC + 3 * _HEAD_MAC) / (_TRUNK_MAC + _HEAD_MAC)  # = 3.50
SPLIT_PEAK_TFLOPS = F16_MFMA_PEAK_TFLOPS / SPLIT_PRODUCTS
GAME_MOVES = 48  # every Yacht Auction game has exactly 48 real moves: the record image's size
# algorithmic FLOPs per expansion (one predicted row), YachtNNet.py:24-70 at hidden 256, 6 blocks
PREDICT_FLOP = 2 * (59 * H + 2 * NB * H * H + H * 128 + 128 + H * A)  # = 3,320,576


def _cgroup_cpus():
    """CPUs this process's cgroup may use: cgroup v2 cpu.max (quota / period), else v1's
    cpu.cfs_quota_us / cpu.cfs_period_us; None when unlimited or unreadable."""
    try:
        with open("/proc/self/cgroup") as fh:
            lines = [ln.strip().split(":", 2) for ln in fh if ln.strip()]
    except OSError:
        lines = []
    cands = []
    for _, ctrl, path in lines:
        if ctrl == "":  # v2 unified hierarchy
            cands.append(("v2", os.path.join("/sys/fs/cgroup", path.lstrip("/"))))
            cands.append(("v2", "/sys/fs/cgroup"))
        elif "cpu" in ctrl.split(","):
            for root in ("/sys/fs/cgroup/cpu,cpuacct", "/sys/fs/cgroup/cpu"):
                cands.append(("v1", os.path.join(root, path.lstrip("/"))))
                cands.append(("v1", root))
    for kind, d in cands:
        try:
            if kind == "v2":
                with open(os.path.join(d, "cpu.max")) as fh:
                    q, per = fh.read().split()[:2]
                if q == "max":
                    return None
                return max(1, int(int(q) // int(per)))
            with open(os.path.join(d, "cpu.cfs_quota_us")) as fh:
                q = int(fh.read())
            with open(os.path.join(d, "cpu.cfs_period_us")) as fh:
                per = int(fh.read())
            return None if q <= 0 else max(1, q // per)
        except (OSError, ValueError):
            continue
    return None


def host_cores():
    """The host cores this process may use: the minimum of the CPUs in its affinity mask and its
    cgroup's CPU quota (unlimited quota: the mask).  -> (cores, {affinity_cpus, cgroup_cpus,
    omp_num_threads_env, host_cpus})."""
    aff = len(os.sched_getaffinity(0))
    cg = _cgroup_cpus()
    cores = min(aff, cg) if cg else aff
    return cores, {"affinity_cpus": aff, "cgroup_cpus": cg,
                   "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"), "host_cpus": os.cpu_count()}


def cpu_baseline(state_dict, sims, seconds_target=15.0, threads=None):
    """The oracle restatement (C, OpenMP over games) on every host core this process may use:
    a bounded sample of the same workload."""
    from oracle import oracle as O
    src = {"source": "argument"}
    if not threads:
        threads, src = host_cores()
    os.environ["OMP_NUM_THREADS"] = str(threads)  # (the oracle's OpenMP pool reads it when it loads)
    net = O.Net(state_dict, H, NB)
    # calibrate: one game per thread, then scale the sample to ~seconds_target
    t0 = time.time()
    r = O.selfplay(list(range(threads)), 1, sims, mode=O.MODE_MLP, net=net, want_counts=False, threads=threads)
    dt = time.time() - t0
    exps = int(r["stats"][:, 1].sum())
    games = threads
    if dt < seconds_target / 2:
        k = max(1, int(seconds_target / max(dt, 1e-3)) - 1)
        t1 = time.time()
        r = O.selfplay(list(range(threads, threads * (k + 1))), 1, sims, mode=O.MODE_MLP, net=net,
                       want_counts=False, threads=threads)
        dt += time.time() - t1
        exps += int(r["stats"][:, 1].sum())
        games += threads * k
    return {"value": exps / dt, "unit": "expansions/s", "cores": threads, "kind": "port",
            "affinity_cpus": src.get("affinity_cpus"), "cgroup_cpus": src.get("cgroup_cpus"),
            "omp_num_threads_env": src.get("omp_num_threads_env"), "host_cpus": src.get("host_cpus"),
            "cores_basis": "cores = min(affinity_cpus, cgroup_cpus) (cgroup_cpus null: no quota); one OpenMP "
                           "thread per core",
            "sample": f"{games} full self-play games x {sims} sims (C restatement, oracle/yk_oracle.c, "
                      f"same net, one OpenMP thread per game), {exps} expansions in {dt:.1f}s",
            "reference_python": "the reference's own Coach/MCTS (Python, 1 core) ran 236 expansions/s in the "
                                "survey container (SURVEY.md section 6); it is not on the GPU box"}


def kernel_sources_sha16():
    """The search / predict kernels' identity: sha256 over the sources k_forward and
    k_expand_backup are built from (every csrc file but the trainers' and the replay buffer's,
    the C-ABI header, the Makefile), 16 hex digits.  tools/profile_bench.sh records it with every
    rocprofv3 summary, so the bench line cites counters of the kernels it runs, or says they are stale."""
    import hashlib
    h = hashlib.sha256()
    pkg = os.path.join(REPO, "nypc-yacht-auction_amd")
    files = sorted(os.path.join(pkg, "csrc", f) for f in os.listdir(os.path.join(pkg, "csrc"))
                   if f.endswith((".hip", ".h")) and not f.startswith(("yk_train", "yk_replay")))
    for f in files + [os.path.join(REPO, "include", "yacht_hip.h"), os.path.join(pkg, "Makefile")]:
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def _measured(args, pattern):
    """The committed rocprofv3 summary (profiles/<pattern>) of this configuration measured on these
    kernel sources; without one, the last of another tree's, marked stale.  -> (json, relpath, stale)."""
    import glob
    cur = kernel_sources_sha16()
    match = other = None
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", pattern))):
        with open(f) as fh:
            t = json.load(fh)
        c = t.get("config", {})
        if (c.get("envs"), c.get("sims"), c.get("hidden"), c.get("nblocks")) != (args.envs, args.sims, H, NB):
            continue
        if t.get("kernel_src_sha16") == cur:
            match = (t, os.path.relpath(f, REPO))
        else:
            other = (t, os.path.relpath(f, REPO))
    if match:
        return match[0], match[1], False
    return (other[0], other[1], True) if other else None


def measured_traffic(args, kind="forward"):
    """HBM bytes per k_forward (kind "forward") / k_expand_backup ("expand") launch from the
    committed rocprofv3 PMC passes of this configuration (profiles/*_{kind}_traffic.json,
    tools/profile_bench.sh): (bytes, source, stale) or None."""
    m = _measured(args, f"*_{kind}_traffic.json")
    return (m[0]["hbm_bytes_per_launch"], m[1], m[2]) if m else None


def measured_mfma(args):
    """k_forward's MFMA busy fraction from the committed rocprofv3 SQ/GRBM pass of this
    configuration (profiles/*_forward_mfma.json, tools/profile_bench.sh); None otherwise."""
    m = _measured(args, "*_forward_mfma.json")
    return dict(m[0], source=m[1], stale=m[2]) if m else None


def arena_leg(net, games=1000, sims=25, seed=0, reps=3):
    """Config 4: Arena.playGames(1000) in one lock-step device batch (agent seat 1 for the first
    half, -1 for the second): MCTS(temp 0, 25 sims) vs the uniform-random legal player, and the
    reference's GreedyYachtPlayer vs random (9.9 games/s on the reference)."""
    import numpy as np
    import torch

    from yacht_amd.engine import SelfPlayEngine
    seats = np.array([1] * (games // 2) + [-1] * (games - games // 2), dtype=np.int32)
    out = {}
    for name, agent, s in (("mcts_vs_random", "mcts", sims), ("greedy_vs_random", "greedy", 1)):
        eng = SelfPlayEngine(games, s, 1.5, 0, net=net, max_moves=64)
        eng.arena(seats, seed + 1000, 0, agent=agent)  # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(reps):
            eng.arena(seats, seed + 1001 + i, 0, agent=agent)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        r = eng.arena_results()
        st = eng.stats()
        eng.close()
        won = r["result"] * seats
        out[name] = {"config": f"Arena.playGames({games}), {agent}" + (f" (temp 0, {s} sims, random-init YachtNNet)"
                                                                      if agent == "mcts" else "") +
                               " vs uniform-random legal player",
                     "games_per_s": games / dt, "ms_per_batch": 1000.0 * dt,
                     "agent_won": int((won == 1).sum()), "random_won": int((won == -1).sum()),
                     "draws": int(((won != 1) & (won != -1)).sum()), "moves": int(r["n_moves"].sum())}
        if agent == "mcts":
            out[name]["expansions_per_s"] = st["expansions"] / dt
    return out


def train_leg(model_sd, eng, steps=40, batch=512, seed=0):
    """Config 5's train step on one GPU (NNetWrapper.train semantics, NNet.py:118-174): minibatches
    of 512 replay entries drawn from the self-play records just produced - the device replay
    buffer yk_examples_from_records builds (packed boards, argmax(pi) targets as
    NNet.py:145-146 takes them, values) - forward + backward + clip + AdamW, dropout 0.3, in both
    modes: f32 and the amp trainer (the reference's GPU path)."""
    import torch

    from yacht_amd.replay import examples_from_images
    from yacht_amd.train import Trainer
    shard = examples_from_images(eng.pack_records(), eng.n_envs, eng.max_moves, eng.sims)
    S, T, V = shard.states, shard.targets, shard.values
    n = S.shape[0]
    out = {}
    for amp in (False, True):
        tr = Trainer(model_sd, H, NB, max_batch=batch, dropout=0.3, seed=seed, amp=amp)
        g = torch.Generator(device="cuda")
        g.manual_seed(seed)
        perm = torch.randperm(n, generator=g, device="cuda").to(torch.int32)
        for i in range(3):  # warm-up
            tr.step(S, T, V, idx=perm[i * batch:(i + 1) * batch])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            j = (i * batch) % (n - batch)
            tr.step(S, T, V, idx=perm[j:j + batch])
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        ce, se, _ = tr.losses()
        st = tr.amp_state() if amp else None
        tr.close()
        flop = 3 * PREDICT_FLOP * batch  # forward + backward (2x) per example
        key = "amp" if amp else "f32"
        out[key] = {"config": f"minibatch {batch} of {n} self-play examples, YachtNNet hidden {H} x {NB}, " +
                              ("autocast('cuda') + GradScaler arithmetic on hand-written fp16 MFMA kernels (6 launches)"
                               if amp else "f32 (hand-written f32 MFMA GEMMs + fused HIP row kernels)") +
                              ", AdamW + clip 5.0, dropout 0.3",
                    "ms_per_step": 1000.0 * dt, "examples_per_s": batch / dt, "achieved_tflops": flop / dt / 1e12,
                    "last_loss": ce / batch + 1.5 * se / batch}
        if st:
            out[key]["grad_scaler"] = st
    out["ms_per_step"] = out["amp"]["ms_per_step"]
    out["basis"] = "ms_per_step is the amp mode's (the reference's GPU train path, NNet.py:113-116, 141-155)"
    return out


def shape_leg(net, envs=2048, sims=200, seed=0):
    """Config 3's per-GPU shape (16384 games x 200 sims over 8 GPUs = 2048 games/GPU x 200 sims):
    one full episode batch on this GPU after one warm-up batch, with the node-pool capacity use
    (NCAP is sized from sims)."""
    import torch

    from yacht_amd.engine import SelfPlayEngine
    eng = SelfPlayEngine(envs, sims, 1.5, 15, net=net, max_moves=64)
    eng.run(seed + 500, 0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.run(seed + 501, 0)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = eng.stats()
    eng.close()
    if st["errors"]:
        raise SystemExit(f"config-3 leg: engine error flags {st['errors']}")
    return {"config": f"{envs} games x {sims} sims on one GPU (config 3's per-GPU shape), full episodes",
            "expansions_per_s": st["expansions"] / dt, "episodes_per_s": envs / dt, "s_per_batch": dt,
            "forward_parts": st["forward_parts"],
            "capacity_use": {k: int(st[k]) for k in ("max_nodes", "node_cap", "max_edges", "edge_cap", "max_arena",
                                                     "arena_cap")}}


def f16_leg(sd, envs=4096, sims=100, seed=0):
    """The opt-in fp16 predict mode (YK_PREDICT_F16: fp16 weights and GEMM inputs, f32
    accumulation - the arithmetic of the reference's own GPU predict under autocast('cuda'),
    NNet.py:186-189) at the headline shape: one warm-up batch, one timed batch, the forward's
    roofline against the f16 dense MFMA peak (one MFMA per product).  Not the headline: the
    headline keeps the f32-equivalent products the north star's 1e-5 tolerance needs."""
    import torch

    from yacht_amd.engine import SelfPlayEngine
    from yacht_amd.nnet import YkNet
    net16 = YkNet(sd, H, NB, precision="f16")
    eng = SelfPlayEngine(envs, sims, 1.5, 15, net=net16, max_moves=64)
    eng.run(seed + 600, 0)
    torch.cuda.synchronize()
    eng.profile(True, stride=20)
    t0 = time.perf_counter()
    eng.run(seed + 601, 0)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st, kt = eng.stats(), eng.kernel_times()
    eng.close()
    if st["errors"]:
        raise SystemExit(f"fp16 leg: engine error flags {st['errors']}")
    out = {"config": f"{envs} games x {sims} sims, full episodes, YachtNNet {H} x {NB}, predict in fp16 "
                     f"(one fp16 MFMA per product, f32 accumulation; LayerNorm / SiLU / softmax f32)",
           "expansions_per_s": st["expansions"] / dt, "episodes_per_s": envs / dt, "s_per_batch": dt}
    if kt.get("forward", (0, 0))[1]:
        f_ms = kt["forward"][0] / kt["forward"][1]
        x_ms = kt["expand_backup_select"][0] / kt["expand_backup_select"][1]
        exp_per_launch = st["expansions"] / max(st["sims"] * st["groups"], 1)
        ach = PREDICT_FLOP * exp_per_launch / (f_ms * 1e-3) / 1e12
        out["kernel_avg_ms"] = {"forward": round(f_ms, 5), "expand_backup_select": round(x_ms, 5)}
        out["roofline"] = {"kernel": "k_forward<256, 1>", "bound": "mfma", "achieved": ach,
                           "peak": F16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": ach / F16_MFMA_PEAK_TFLOPS,
                           "work_per_launch": f"{exp_per_launch:.0f} expansions x {PREDICT_FLOP} FLOP"}
    return out


def coach_iter_leg(model, world, games_per_gpu=8192, seed=0, amp=True, warm=True, history=1):
    """Config 5 at its per-GPU shape: ONE whole Coach.learn iteration (Coach.py:74-139) with
    main.py's args (main.py:17-43: 25 sims, tempThreshold 15, maxlenOfQueue 200,000, 15 epochs of
    batch 512, dropout 0.3, arenaCompare 10, updateThreshold 0.55) over numEps = games_per_gpu x
    N games sharded over the N ranks (65,536 on 8 GPUs = config 5), the reference's GPU train
    path (autocast + GradScaler: the amp trainer) unless amp=False.  Per-phase wall times of a
    steady-state iteration: warm=True first runs a 512-game iteration untimed (the first torch.save
    / zipfile / allocator use of the process cost about 1.5 s once, profiles/r03c_coach_profile.log).
    history > 1: the steady state of Coach.learn (numItersForTrainExamplesHistory 5, main.py:30):
    the replay history already holds history - 1 earlier iterations' worth of examples (copies of
    one untimed self-play iteration's 200,000-example shard), so the timed iteration trains on
    history x 200,000 examples as every iteration after the fourth does (Coach.py:99-111)."""
    if warm:
        coach_iter_leg(model, world, games_per_gpu=min(512, games_per_gpu), seed=seed + 1, amp=amp, warm=False)
    import shutil
    import tempfile

    from yacht_amd.coach import Coach
    from yacht_amd import dist as D
    from yacht_amd.game import YachtGame
    from yacht_amd.nnet import NNetWrapper
    from yacht_amd.utils import dotdict
    rank, _ = D.rank_world()
    tmp = tempfile.mkdtemp(prefix="yk_coach_") if rank == 0 else None
    if world > 1:
        import torch.distributed as dist
        box = [tmp]
        dist.broadcast_object_list(box, src=0)
        tmp = box[0]
    args = dotdict(numIters=1, numEps=games_per_gpu * world, tempThreshold=15, updateThreshold=0.55,
                   maxlenOfQueue=200000, numMCTSSims=25, arenaCompare=10, cpuct=1.5, checkpoint=tmp,
                   load_folder_file=(tmp, "best.pth.tar"), numItersForTrainExamplesHistory=5, lr=2e-3,
                   weight_decay=1e-4, epochs=15, batch_size=512, vloss_weight=1.5, cuda=True, hidden=H,
                   nblocks=NB, dropout=0.3, amp=amp, examples_format="npz", seed=seed)
    game = YachtGame(seed=seed + 99, env_id=2 * 10**6)
    nn = NNetWrapper(game, args)
    nn.nnet.load_state_dict(model.state_dict())
    c = Coach(game, nn, args)
    if history > 1:
        earlier = c.selfPlayExamples(args.numEps, maxlen=args.maxlenOfQueue)  # untimed
        c.trainExamplesHistory = [earlier] * (history - 1)
    c.learn()
    n = sum(len(x) for x in c.trainExamplesHistory)
    steps = 15 * -(-n // 512)
    out = {"config": f"one Coach.learn iteration, main.py args: numEps {args.numEps} ({games_per_gpu}/GPU x {world}), "
                     f"25 sims, maxlenOfQueue 200000, 15 epochs x batch 512 "
                     f"({'autocast + GradScaler on fp16 MFMA' if amp else 'f32'}; every rank the whole minibatch), "
                     f"dropout 0.3, arenaCompare 10",
           "history_iterations": len(c.trainExamplesHistory), "examples_trained": n, "train_steps": steps,
           "gate_tally_prev_new_draws": list(c.last_pit)}
    out.update({k: round(v, 4) for k, v in c.phase_times.items()})
    out["train_ms_per_step"] = 1000.0 * c.phase_times["train_s"] / max(steps, 1)
    if rank == 0:
        shutil.rmtree(tmp, ignore_errors=True)
    return out


def coach_leg(model, image, n_envs, max_moves, sims, world, train_steps=60, arena_games=256, arena_sims=25,
              seed=0):
    """Config 5's Coach iteration after the self-play the timed steps just did (Coach.py:74-139),
    on every rank: the pooled replay buffer from the (all-gathered) record images
    (yk_examples_from_records), `train_steps` train steps of the reference minibatch (512
    examples, clip, AdamW; NNetWrapper.train: every rank the whole minibatch, the default
    ddp_batch "replicated" - and at N > 1 also timed "split": the minibatch split over the
    ranks with a gradient all-reduce per step), and
    the gating arena (previous vs new net, MCTS temp 0 each, one dual-tree batch sharded over
    the ranks).  Returns this rank's phase times; rank 0 reports them."""
    import numpy as np
    import torch

    from yacht_amd import dist as D
    from yacht_amd.arena import GatingArena
    from yacht_amd.game import YachtGame
    from yacht_amd.nnet import DEFAULT_ARGS, NNetWrapper
    from yacht_amd.replay import examples_from_images
    from yacht_amd.utils import dotdict
    rank, _ = D.rank_world()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    shard = examples_from_images(image, n_envs, max_moves, sims)
    torch.cuda.synchronize()
    t_ex = time.perf_counter() - t0
    args = dotdict(DEFAULT_ARGS, epochs=1, numMCTSSims=arena_sims, cpuct=1.5, seed=seed)
    game = YachtGame(seed=seed + 77, env_id=10**6)
    prev, new = NNetWrapper(game, args), NNetWrapper(game, args)
    prev.nnet.load_state_dict(model.state_dict())
    new.nnet.load_state_dict(model.state_dict())
    bs = args.batch_size
    n = len(shard)
    sub = torch.randperm(n, generator=torch.Generator().manual_seed(seed))[:bs * (train_steps + 3)]
    few = (shard.states[sub.to("cuda")], shard.targets[sub.to("cuda")], shard.values[sub.to("cuda")])
    from yacht_amd.replay import ExampleShard
    warm = ExampleShard(*(x[:3 * bs] for x in few))
    new.train(warm, verbose=False)  # warm-up: 3 steps
    timed = ExampleShard(*(x[3 * bs:] for x in few))
    D.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    new.train(timed, verbose=False)
    torch.cuda.synchronize()
    train_steps = -(-len(timed) // bs)
    t_tr = (time.perf_counter() - t1) / max(train_steps, 1)
    t_split = None
    if world > 1:  # the DDP alternative: each rank a 1/N share, one RCCL all-reduce per step
        spl = NNetWrapper(game, dotdict(args, ddp_batch="split"))
        spl.nnet.load_state_dict(model.state_dict())
        spl.train(warm, verbose=False)
        D.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        spl.train(timed, verbose=False)
        torch.cuda.synchronize()
        t_split = (time.perf_counter() - t1) / max(train_steps, 1)
    D.barrier()
    t2 = time.perf_counter()
    pw, nw, dr = GatingArena(game, prev, new, args).playGames(arena_games, env_base=10**6)
    torch.cuda.synchronize()
    t_ar = time.perf_counter() - t2
    return {"config": f"pooled examples of the timed batch ({n} examples from {world} rank(s)); "
                      f"{train_steps} train steps of minibatch {bs} (every rank the whole minibatch: "
                      f"ddp_batch replicated; clip 5.0, AdamW, dropout {args.dropout}); gating arena {arena_games} games, "
                      f"{arena_sims} sims, previous vs new net on dual trees, sharded",
            "train_mode": "amp (autocast + GradScaler on fp16 MFMA, NNet.py:113-116: args.cuda)" if new.uses_amp()
                          else "f32",
            "examples": n, "examples_ms": 1000.0 * t_ex, "train_ms_per_step": 1000.0 * t_tr,
            "train_examples_per_s": bs / t_tr,
            "train_ms_per_step_split": None if t_split is None else 1000.0 * t_split,
            "train_split_basis": "ddp_batch split: the minibatch split over the ranks, one gradient all-reduce per "
                                 "step (N > 1 only)",
            "arena_s": t_ar, "arena_games_per_s": arena_games / t_ar,
            "arena_tally_prev_new_draws": [pw, nw, dr]}


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def spawn_ranks(nprocs, argv, timeout_s, script=None, out=None, err=None, poll_s=0.2):
    """Run `nprocs` ranks of this job on one node without an external launcher: fresh child
    interpreters (`python -u script argv`), each with torchrun's environment contract (RANK,
    LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR 127.0.0.1, a free MASTER_PORT), started
    before this process makes any GPU call (it makes none).  Rank 0's stdout lines that parse as
    a JSON object are relayed to `out` (the bench line); everything else any rank prints goes to
    `err` (stderr is inherited when `err` is sys.stderr).  The first child to fail (or the
    timeout) ends the job: the other ranks' process groups are terminated (then killed) and the
    return code is non-zero (the failing rank's code, 124 on timeout, 1 when rank 0 printed no
    JSON line or more than one, 128 + the signal when this process is told to stop: the ranks then
    stop too; a child also gets SIGTERM if this process dies, PR_SET_PDEATHSIG).  -> exit code."""
    import signal
    import subprocess
    import threading
    out = out or sys.stdout
    err = err or sys.stderr
    script = script or os.path.abspath(__file__)
    port = _free_port()
    procs, lines = [], []

    def pump(stream, rank):
        for raw in iter(stream.readline, b""):
            line = raw.decode(errors="replace")
            obj = None
            if rank == 0 and line.lstrip().startswith("{"):
                try:
                    obj = json.loads(line)
                except ValueError:
                    obj = None
            if isinstance(obj, dict):
                lines.append(line.rstrip("\n"))
            else:
                err.write(f"[rank {rank if rank >= 0 else -1 - rank}] {line}")
                err.flush()
        stream.close()

    def die_with_parent():  # (in the child, before exec: no GPU state exists yet)
        try:
            import ctypes
            ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGTERM)  # PR_SET_PDEATHSIG
        except OSError:
            pass

    for r in range(nprocs):  # every child first: preexec_fn runs while this process has no threads
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nprocs),
                   LOCAL_WORLD_SIZE=str(nprocs), GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   YK_SELF_SPAWNED="1")
        procs.append(subprocess.Popen([sys.executable, "-u", script] + list(argv), env=env, stdout=subprocess.PIPE,
                                      stderr=None if err is sys.stderr else subprocess.PIPE, start_new_session=True,
                                      preexec_fn=die_with_parent))
    pumps = []
    for r, p in enumerate(procs):
        for stream, kind in ((p.stdout, "out"), (p.stderr, "err")):
            if stream is not None:  # (stderr: inherited unless `err` is not this process's stderr)
                t = threading.Thread(target=pump, args=(stream, r if kind == "out" else -1 - r), daemon=True)
                t.start()
                pumps.append(t)

    def stop_all():
        for sig, wait in ((signal.SIGTERM, 10.0), (signal.SIGKILL, 5.0)):
            live = [p for p in procs if p.poll() is None]
            for p in live:
                try:
                    os.killpg(p.pid, sig)  # the child's own process group (start_new_session)
                except ProcessLookupError:
                    pass
            t_end = time.time() + wait
            while any(p.poll() is None for p in live) and time.time() < t_end:
                time.sleep(0.1)

    # a launcher that is itself terminated (a driver's time limit) takes its ranks down with it
    stopped = []

    def on_signal(signum, frame):
        stopped.append(signum)

    old_handlers = {sg: signal.signal(sg, on_signal) for sg in (signal.SIGTERM, signal.SIGINT, signal.SIGHUP)}
    t0 = time.time()
    rc = 0
    while True:
        if stopped:
            err.write(f"spawn_ranks: signal {stopped[0]}; stopping every rank\n")
            stop_all()
            rc = 128 + stopped[0]
            break
        codes = [p.poll() for p in procs]
        bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
        if bad:
            r, c = bad[0]
            err.write(f"spawn_ranks: rank {r} exited with {c}; stopping the other ranks\n")
            stop_all()
            rc = c if c > 0 else 128 - c  # (a signal: 128 + signal number)
            break
        if all(c == 0 for c in codes):
            break
        if time.time() - t0 > timeout_s:
            err.write(f"spawn_ranks: timeout after {timeout_s:.0f} s; stopping every rank\n")
            stop_all()
            rc = 124
            break
        time.sleep(poll_s)
    for sg, h in old_handlers.items():
        signal.signal(sg, h)
    for t in pumps:
        t.join(timeout=5.0)
    if rc == 0 and len(lines) != 1:
        err.write(f"spawn_ranks: rank 0 printed {len(lines)} JSON lines (expected one)\n")
        rc = 1
    if rc == 0:
        out.write(lines[0] + "\n")
        out.flush()
    err.flush()
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--envs", type=int, default=4096, help="games per GPU")
    ap.add_argument("--sims", type=int, default=100)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="skip the per-kernel event timing")
    ap.add_argument("--profile-stride", type=int, default=20,
                    help="time the forward / expand pair of every k-th simulation (1 = all; each event "
                         "record between dependent launches costs GPU time: ~5 %% of the batch at 1)")
    ap.add_argument("--no-arena", action="store_true", help="skip the config-4 Arena leg")
    ap.add_argument("--no-train", action="store_true", help="skip the config-5 train-step leg")
    ap.add_argument("--no-coach", action="store_true", help="skip the config-5 Coach-iteration legs")
    ap.add_argument("--no-shape", action="store_true", help="skip the config-3 shape leg (2048 x 200)")
    ap.add_argument("--no-f16", action="store_true", help="skip the fp16 predict-mode leg")
    ap.add_argument("--no-steady", action="store_true",
                    help="skip the steady-state Coach iteration (a 5-iteration replay history)")
    ap.add_argument("--coach-games", type=int, default=8192,
                    help="games per GPU of the whole-iteration config-5 leg (config 5: 65,536 / 8 = 8192)")
    ap.add_argument("--dist-backend", default=None, help="nccl (RCCL, default on GPUs) or gloo (rehearsal)")
    ap.add_argument("--groups", type=int, default=0,
                    help="game groups on their own streams (0: the engine's auto choice)")
    ap.add_argument("--root-scan", type=int, default=1,
                    help="0: every descent scans the root's whole compact set (YK_ROOT_SCAN=0; A/B only)")
    ap.add_argument("--root-k", type=int, default=0,
                    help="entries of the root's P order kept (YK_ROOT_K; 0: the engine's 512; A/B only)")
    ap.add_argument("--arena-entries", type=int, default=0,
                    help="P-arena entries per game (0: the engine's overflow-free default)")
    ap.add_argument("--spawn-timeout", type=float, default=3000.0,
                    help="--gpus N > 1 without a launcher's WORLD_SIZE: seconds the self-spawned ranks may take")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: this process starts the N ranks itself (before touching the GPU) and relays
        # rank 0's line; under torchrun (WORLD_SIZE set) each rank runs the code below
        raise SystemExit(spawn_ranks(args.gpus, sys.argv[1:], args.spawn_timeout))
    if not args.root_scan:
        os.environ["YK_ROOT_SCAN"] = "0"
    if args.root_k:
        os.environ["YK_ROOT_K"] = str(args.root_k)

    import torch
    import torch.distributed as dist

    from yacht_amd import dist as D
    from yacht_amd.engine import SelfPlayEngine
    from yacht_amd.nnet import YachtNNet, YkNet

    rank, world, local = D.setup(args.dist_backend)
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(D.device_index(local))
    torch.manual_seed(args.seed)
    model = YachtNNet(hidden=H, nblocks=NB)  # random init of the reference architecture
    sd = model.state_dict()
    net = YkNet(sd, H, NB)
    eng = SelfPlayEngine(args.envs, args.sims, 1.5, 15, net=net, max_moves=GAME_MOVES, arena_entries=args.arena_entries,
                         groups=args.groups)
    stream = torch.cuda.current_stream()
    env_base = D.env_base(rank, args.envs)
    gathered_bytes = 0
    image_bytes = 0

    last_gather = [None]

    def step(i):
        nonlocal gathered_bytes
        eng.run(args.seed + i, env_base, stream)
        if world > 1:
            buf = eng.pack_records(stream=stream)
            g = D.allgather_records(buf)
            gathered_bytes = g.numel()
            last_gather[0] = g

    for i in range(args.warmup):
        step(i)
    image_bytes = int(eng.pack_records(stream=stream).numel())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    exp0 = 0
    if not args.no_profile:
        eng.profile(True, stride=args.profile_stride)
    t0 = time.perf_counter()
    exps = 0
    games = 0
    for i in range(args.steps):
        step(args.warmup + i)
        st = eng.stats()
        exps += st["expansions"]
        games += args.envs
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kt = eng.kernel_times() if not args.no_profile else {}
    st = eng.stats()
    if st["errors"]:
        raise SystemExit(f"engine error flags {st['errors']}")

    tot = torch.tensor([elapsed, float(exps), float(games)], dtype=torch.float64,
                       device="cuda" if world > 1 and dist.get_backend() == "nccl" else "cpu")
    gather_ok = None
    if world > 1:
        # the all-gather delivered every rank's image byte for byte: each rank compares its slot of
        # the pooled buffer with its own freshly packed image, and every rank's checksum of every slot
        # must agree across ranks
        own = eng.pack_records(stream=stream)
        g = last_gather[0]
        mine = bool(torch.equal(g[rank].to(own.device), own))
        w = torch.arange(1, g.shape[1] + 1, dtype=torch.int64, device=g.device) % 1000003
        sums = (g.to(torch.int64) * w).sum(dim=1)  # one position-weighted checksum per slot
        if dist.get_backend() != "nccl":
            sums = sums.cpu()
        allsums = [torch.zeros_like(sums) for _ in range(world)]
        dist.all_gather(allsums, sums)
        agree = all(torch.equal(a.cpu(), allsums[0].cpu()) for a in allsums)
        flag = torch.tensor([1 if (mine and agree) else 0], dtype=torch.int32,
                            device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        gather_ok = bool(flag.item())
        del own
    if world > 1:
        t_max = tot[:1].clone()
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        sums = tot[1:].clone()
        dist.all_reduce(sums, op=dist.ReduceOp.SUM)
        elapsed, exps, games = float(t_max[0]), float(sums[0]), float(sums[1])
    coach = None
    if not args.no_coach:
        img = last_gather[0] if world > 1 else eng.pack_records(stream=stream)
        coach = coach_leg(model, img, args.envs, GAME_MOVES, args.sims, world, seed=args.seed)
        del img
        with contextlib.redirect_stdout(sys.stderr):  # Coach.learn's progress lines: stdout is the JSON line
            coach["iteration"] = coach_iter_leg(model, world, games_per_gpu=args.coach_games, seed=args.seed)
            if not args.no_steady:
                coach["iteration_steady"] = coach_iter_leg(model, world, games_per_gpu=args.coach_games,
                                                           seed=args.seed + 3, warm=False, history=5)
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    value = exps / elapsed
    out = {
        "metric": METRIC, "value": value, "unit": "expansions/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": 1000.0 * elapsed / args.steps, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "precision": "predict: f32-equivalent fp16 hi/lo split on MFMA (f32 accumulate), within 1e-5 of torch fp32; "
                     "search arithmetic f32/f64 as the reference",
        "config": {"workload": f"{args.envs} games/GPU x {args.sims} sims, full 48-move self-play episodes, "
                               f"YachtNNet hidden {H} x {NB} blocks (random init)",
                   "envs_per_gpu": args.envs, "sims": args.sims, "cpuct": 1.5, "temp_threshold": 15,
                   "parallelism": f"games sharded over {world} GPU(s), RCCL all-gather of trajectories"},
        "episodes_per_s": games / elapsed,
        "value_basis": "whole job, as the bench contract defines `value` (the driver derives scaling "
                       "efficiency from it): expansions of all GPUs / the slowest rank's time; the metric's "
                       "per-GPU rate is value_per_gpu (= value at N=1)",
        "value_total": value,
        "value_per_gpu": value / world,
        "expansions_per_s_per_gpu": value / world,
        "expansions_per_episode_batch": exps / args.steps,
        "game_groups": st["groups"],
        "forward_parts": st["forward_parts"],
        "kernel_src_sha16": kernel_sources_sha16(),
        "capacity_use": {k: int(st[k]) for k in ("max_nodes", "node_cap", "max_edges", "edge_cap", "max_arena",
                                                 "arena_cap")},
    }
    if world > 1:
        # the pooled replay buffer holds every rank's complete games (48 moves each), and
        # the ranks played different games (global env ids)
        from yacht_amd.engine import unpack_record_image
        imgs = [unpack_record_image(last_gather[0][r].cpu().numpy(), args.envs, GAME_MOVES, args.sims)
                for r in range(world)]
        ok = all(bool((im["n_moves"] == 48).all()) for im in imgs)
        ok = ok and len({im["final"].tobytes() for im in imgs}) == world
        out["allgather_check"] = "ok" if ok and gather_ok else "FAILED"
        out["allgather_check_basis"] = ("every rank's slot of the pooled buffer equals that rank's own packed image "
                                        "byte for byte, the per-slot checksums agree on all ranks, every game has "
                                        "48 moves and the ranks' final boards differ")
        out["dist_backend"] = dist.get_backend()
    # the trajectory all-gather's payload: one fixed-size record image per rank (48 moves), gathered
    # into every rank's buffer (at N = 1 there is no collective; the figure is the image it would send)
    out["record_image_bytes_per_rank"] = image_bytes
    out["allgather_bytes"] = gathered_bytes if world > 1 else image_bytes
    out["allgather_bytes_basis"] = ("bytes of the pooled buffer every rank receives per episode batch (N x the "
                                    "per-rank image); N = 1: the one image, no collective runs")
    if kt:
        # dominant kernel and its roofline (algorithmic work per launch / average launch time)
        per = {k: (ms / n if n else 0.0, n, ms) for k, (ms, n) in kt.items()}
        out["kernel_ms"] = {k: {"avg_ms": round(a, 5), "launches": n, "total_ms": round(t, 2)}
                            for k, (a, n, t) in per.items()}
        out["kernel_ms_basis"] = (f"HIP event intervals on the engine's stream inside the timed region; forward and "
                                  f"expand_backup_select timed in every {args.profile_stride}th simulation of "
                                  f"each move (launches = the timed ones), the per-move kernels every time")
        dom = max(per, key=lambda k: per[k][2])
        fwd = env = None
        if "forward" in per and per["forward"][1]:
            # k_forward (MFMA): algorithmic FLOP per launch = expansions predicted per launch x 3,320,576
            # (one forward launch per simulation and game group; st["sims"] = simulations per batch)
            exp_per_launch = exps / world / args.steps / max(st["sims"] * st["groups"], 1)
            flop = PREDICT_FLOP * exp_per_launch
            ach = flop / (per["forward"][0] * 1e-3) / 1e12
            tr = measured_traffic(args)  # per-GPU configuration, so per-launch bytes hold at any N
            fwd = {"kernel": "k_forward", "bound": "mfma", "achieved": ach,
                   "peak": SPLIT_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": ach / SPLIT_PEAK_TFLOPS,
                   "traffic": tr[0] if tr else None,
                   "traffic_source": tr[1] if tr else None,
                   "traffic_stale": tr[2] if tr else None,
                   "work_per_launch": f"{exp_per_launch:.0f} expansions x {PREDICT_FLOP} FLOP (f32)",
                   "peak_basis": f"f16 dense MFMA peak / {SPLIT_PRODUCTS:.2f}: every f32 product runs as hi*hi + "
                                 "hi*lo + lo*hi (+ (lo 2^-11)*lo outside the policy head) on fp16 planes with f32 "
                                 "accumulation; the product count FLOP-weighted over the layers",
                   "limiter": "per-CU weight stream: each 16-row tile streams all 6.7 MB of weight "
                              "planes through its CU, and one CU streams a weight set shared by all CUs "
                              "at 110-123 GB/s at any CU count; the fp16 MFMAs overlap the stream "
                              "(tools/stream_bench.hip, profiles/r02_stream_sweep.txt, DESIGN.md section 6)"}
            mf = measured_mfma(args)
            if mf:
                fwd["mfma_busy"] = {k: mf[k] for k in ("busy_frac", "formula", "source", "stale") if k in mf}
        if "expand_backup_select" in per and per["expand_backup_select"][1]:
            # k_expand_backup (HBM): algorithmic bytes from the engine's own counters of the last batch,
            # per launch.  SURVEY 8d's formula (4 S_scan + 16 D + 4 V_new + 364 per expansion) counts 4 B
            # per UCB entry; what the kernel must read and write is 6 B per scanned entry (P f32 + the
            # u16 edge slot), 16 B per visited entry's edge, 32 B per backed-up path edge (read +
            # write), 10 B per new valid entry (its logit read, P and slot written), 364 B per expansion
            launches = max(st["sims"] * st["groups"], 1)
            survey_b = (4 * st["scanned"] + 16 * st["path_edges"] + 4 * st["vnew"] + 364 * st["expansions"]) / launches
            b = (6 * st["scanned"] + 16 * st.get("scan_edges", 0) + 32 * st["path_edges"] + 10 * st["vnew"]
                 + 364 * st["expansions"]) / launches
            ach = b / (per["expand_backup_select"][0] * 1e-3) / 1e9
            tr = measured_traffic(args, "expand")
            env = {"kernel": "k_expand_backup", "bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS,
                   "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "traffic": tr[0] if tr else None,
                   "traffic_source": tr[1] if tr else None, "traffic_stale": tr[2] if tr else None,
                   "work_per_launch": f"{b:.0f} algorithmic bytes = (6 x {st['scanned']} UCB entries scanned + "
                                      f"16 x {st.get('scan_edges', 0)} edges gathered + 32 x {st['path_edges']} path "
                                      f"edges + 10 x {st['vnew']} new valid entries + 364 x {st['expansions']} "
                                      f"expansions) / {launches} launches",
                   "survey_formula_bytes_per_launch": survey_b,
                   # SURVEY 8d's byte basis (4 / 16 / 4 / 364 B; rounds 1-4 priced the kernel on it): the
                   # like-for-like fraction across rounds
                   "frac_survey_formula": survey_b / (per["expand_backup_select"][0] * 1e-3) / 1e9 / HBM_PEAK_GBS,
                   "frac_basis": "frac: the kernel's own bytes (6 B per scanned entry, 16 B per gathered edge, 32 B "
                                 "per path edge, 10 B per new valid entry, 364 B per expansion; since round 5); "
                                 "frac_survey_formula: SURVEY 8d's formula"}
        if dom == "forward":
            out["roofline"], out["roofline_env"] = fwd, env
        else:
            out["roofline"], out["roofline_mfma"] = env, fwd
    if coach is not None:
        out["coach"] = coach
    if world == 1 and not args.no_shape:
        out["config3_shape"] = shape_leg(net, seed=args.seed)
    if world == 1 and not args.no_f16:
        out["predict_f16"] = f16_leg(sd, args.envs, args.sims, seed=args.seed)
    if world == 1 and not args.no_arena:
        out["arena"] = arena_leg(net, seed=args.seed)
    if world == 1 and not args.no_train:
        out["train"] = train_leg(sd, eng, seed=args.seed)
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(sd, args.sims)
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
