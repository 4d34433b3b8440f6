"""Opt-in statistic (not a parity gate): how often the engine's self-play at the bench configuration
(4096 games x 100 sims, YachtNNet 256 x 6, closed-form weights) takes a different search outcome
from an independent float32 predict (the oracle's C restatement of YachtNNet.forward, MODE_MLP),
on a larger sample than test_selfplay_net_prior_at_bench_size's 64 games, so that two engine
builds can be compared (64 games give a standard error of about 4 points).

    YK_DIVERGENCE_STRIDE=16 YK_DIVERGENCE_TAG=head python -m pytest tests/test_gpu_divergence.py -s

Each run writes its per-game first diverging move to gpurun_out/div_<tag>_<stride>.npz and also
reports its divergence from every other tag's engine plays found there (build vs build).  The
oracle's plays (and its reverse-summation twin, the rate float32 rounding alone gives) take minutes
of CPU: they are cached as move lists + per-move visit-count digests in
tools/_div_oracle_<stride>.npz (git-ignored), which `python tests/test_gpu_divergence.py STRIDE`
writes on any host beforehand."""
import hashlib
import os

import numpy as np
import pytest

from oracle import oracle as O
from oracle import spec

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

STRIDE = int(os.environ.get("YK_DIVERGENCE_STRIDE", "0"))
TAG = os.environ.get("YK_DIVERGENCE_TAG", "head")
OUT = "gpurun_out"
N_GAMES, SIMS, SEED, BASE = 4096, 100, 2024, 0


def _digest(c):
    return int.from_bytes(hashlib.blake2b(np.ascontiguousarray(c, dtype=np.int32).tobytes(), digest_size=8).digest(), "little")


def _plays_oracle(run, n):
    mv = np.full((n, 48), -1, np.int64)
    dg = np.zeros((n, 48), np.uint64)
    for r in range(n):
        M = int(run["stats"][r, 0])
        mv[r, :M] = run["mv"][r, :M, 2]
        for m in range(M):
            dg[r, m] = _digest(run["counts"][r, m])
    return mv, dg


def _plays_engine(rec, pick):
    M = rec["states"].shape[1]
    mv = np.full((len(pick), 48), -1, np.int64)
    dg = np.zeros((len(pick), 48), np.uint64)
    for r, e in enumerate(pick):
        n = int(rec["n_moves"][e])
        mv[r, :n] = rec["info"][e, :n, 2]
        for m in range(n):
            a0, a1 = rec["visits_off"][e * M + m], rec["visits_off"][e * M + m + 1]
            c = np.zeros(3226, dtype=np.int32)
            v = rec["visits"][a0:a1]
            c[v[:, 0]] = v[:, 1]
            dg[r, m] = _digest(c)
    return mv, dg


def _first(a, b):
    diff = (a[0] != b[0]) | (a[1] != b[1])
    return np.where(diff.any(1), diff.argmax(1), -1)


def oracle_plays(stride):
    here = os.path.dirname(os.path.abspath(__file__))
    cache = os.path.join(here, "..", "tools", f"_div_oracle_{stride}.npz")
    if not os.path.exists(cache):
        pick = np.arange(0, N_GAMES, stride)
        sd = spec.closed_form_weights(256, 6)
        kw = dict(max_moves=48, threads=min(16, os.cpu_count() or 1))
        orc = _plays_oracle(O.selfplay(BASE + pick, SEED, SIMS, 1.5, 15, O.MODE_MLP, net=O.Net(sd, 256, 6), **kw), len(pick))
        rev = _plays_oracle(O.selfplay(BASE + pick, SEED, SIMS, 1.5, 15, O.MODE_MLP,
                                       net=O.Net(sd, 256, 6, reverse_sums=True), **kw), len(pick))
        np.savez(cache, omv=orc[0], odg=orc[1], rmv=rev[0], rdg=rev[1])
    z = np.load(cache)
    return (z["omv"], z["odg"]), (z["rmv"], z["rdg"])


@pytest.mark.skipif(STRIDE <= 0, reason="opt-in: set YK_DIVERGENCE_STRIDE")
def test_divergence_statistic():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from yacht_amd import engine as E, nnet as N
    n, sims, seed, base = N_GAMES, SIMS, SEED, BASE
    pick = np.arange(0, n, STRIDE)
    sd = spec.closed_form_weights(256, 6)
    eng = E.SelfPlayEngine(n, sims, 1.5, 15, net=N.YkNet(sd, 256, 6), max_moves=48)
    eng.run(seed, base)
    assert eng.stats()["errors"] == 0
    mine = _plays_engine(eng.records(), pick)
    eng.close()
    os.makedirs(OUT, exist_ok=True)
    orc, rev = oracle_plays(STRIDE)
    f = _first(mine, orc)
    ff = _first(rev, orc)
    se = np.sqrt((f >= 0).mean() * (1 - (f >= 0).mean()) / len(pick))
    print(f"\n[{TAG}] {len(pick)} games x {sims} sims: engine vs independent f32 {(f >= 0).mean():.3f} "
          f"(+- {se:.3f}) of the games diverge; f32 vs f32 (reverse sums) {(ff >= 0).mean():.3f}")
    np.savez(f"{OUT}/div_{TAG}_{STRIDE}.npz", mv=mine[0], dg=mine[1], first=f)
    for fn in sorted(os.listdir(OUT)):
        if fn.startswith("div_") and fn.endswith(f"_{STRIDE}.npz") and not fn.startswith(("div_oracle", f"div_{TAG}_")):
            z = np.load(f"{OUT}/{fn}")
            g = _first(mine, (z["mv"], z["dg"]))
            print(f"[{TAG}] vs engine {fn[4:-len(f'_{STRIDE}.npz')]}: {(g >= 0).mean():.3f} of the games diverge; "
                  f"both diverge from the oracle: {((f >= 0) & (z['first'] >= 0)).mean():.3f}")


if __name__ == "__main__":
    import sys
    oracle_plays(int(sys.argv[1]))
