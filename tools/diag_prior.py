"""diagnostic (GPU box): where do the engine's recorded priors and the oracle net's predict part?
Runs a small recorded self-play batch, then compares, per renormalised prior P (MCTS.py:86-91):
engine (valid-only forward), GPU full predict, oracle C net, torch fp32 CPU - each against a
torch float64 CPU forward of the same weights.  usage: python tools/diag_prior.py"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "nypc-yacht-auction_amd")]
from oracle import oracle as O  # noqa: E402
from oracle import spec  # noqa: E402
from yacht_amd import kernels as K  # noqa: E402
from yacht_amd.engine import SelfPlayEngine  # noqa: E402
from yacht_amd.nnet import YachtNNet, YkNet  # noqa: E402


def renorm64(pi, ok):
    p = np.where(ok, pi.astype(np.float64), 0.0)
    s = p.sum(1, keepdims=True)
    return np.divide(p, s, out=np.zeros_like(p), where=s > 0)


def main():
    sd = spec.closed_form_weights(256, 6)
    net = YkNet(sd, 256, 6)
    n, sims = 6, 12
    eng = SelfPlayEngine(n, sims, 1.5, 15, net=net, max_moves=64, record_predictions=True, max_expansions=64 * sims)
    eng.run(77, 10)
    pi, v, cnt, leaves = eng.predictions(leaves=True)
    S = np.concatenate([leaves[e, :cnt[e]] for e in range(n)])
    P = np.concatenate([pi[e, :cnt[e]] for e in range(n)])
    ok = O.valid(S, 1)[0].astype(bool)
    V = np.concatenate([v[e, :cnt[e]] for e in range(n)])
    full, vfull = (t.cpu().numpy() for t in net.predict_states(K.states_to_device(S)))
    opi, ov = O.Net(sd, 256, 6).predict_states(S)
    x = torch.from_numpy(O.featurize(S))
    m32 = YachtNNet(hidden=256, nblocks=6)
    m32.load_state_dict({k: torch.as_tensor(np.asarray(t, dtype=np.float32)) for k, t in sd.items()})
    m32.eval()
    m64 = YachtNNet(hidden=256, nblocks=6).double()
    m64.load_state_dict({k: torch.as_tensor(np.asarray(t, dtype=np.float64)) for k, t in sd.items()})
    m64.eval()
    with torch.no_grad():
        l32, v32 = m32(x)
        l64, v64 = m64(x.double())
    v32, v64 = v32.numpy().reshape(-1), v64.numpy().reshape(-1)
    t32 = torch.exp(torch.log_softmax(l32, 1)).numpy()
    t64 = torch.exp(torch.log_softmax(l64, 1)).numpy()
    truth = renorm64(t64, ok)
    print(f"rows {len(S)}; |logit| max {float(l64.abs().max()):.2f}, mean {float(l64.abs().mean()):.2f}")
    for name, arr in (("engine", P), ("gpu_full", full), ("oracle", opi), ("torch32", t32)):
        r = renorm64(arr, ok)
        rel = np.abs(r - truth) / np.maximum(truth, 1e-30)
        big = truth > 1e-3
        print(f"{name:9s} max rel err (P > 1e-3) {rel[big].max():.3e}  p99.99 {np.quantile(rel[big], 0.9999):.3e}  "
              f"max abs {np.abs(r - truth).max():.3e}")
    for name, arr in (("engine", V), ("gpu_full", vfull), ("oracle", ov), ("torch32", v32)):
        print(f"{name:9s} v max abs err vs f64 {np.abs(arr - v64).max():.3e}")
    print(f"engine v vs oracle v: max abs {np.abs(V - ov).max():.3e}")
    # worst rows for the engine-vs-oracle comparison of the test
    d = np.abs(renorm64(P, ok) - renorm64(opi, ok))
    tol = 1e-7 + 3e-5 * np.abs(renorm64(opi, ok))
    bad = np.argwhere(d > tol)
    rows = np.unique(bad[:, 0])
    print(f"test-tolerance violations: {len(bad)} elements in {len(rows)} rows; valid counts {ok[rows].sum(1)[:20]}")
    for i in rows[:5]:
        print(f"  row {i}: nvalid {ok[i].sum()} logit range [{float(l64[i][ok[i]].min()):.2f}, "
              f"{float(l64[i][ok[i]].max()):.2f}] valid mass (t64) {float(t64[i][ok[i]].sum()):.3e}")


if __name__ == "__main__":
    main()
