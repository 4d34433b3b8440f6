"""Shared parity checks for the GPU tests (test infrastructure: uses the oracle as the checker)."""
import numpy as np

from oracle import oracle as O

# The north star's tolerance is on predict's policy tensor (pi within 1e-5, as test_gpu_net; x3 here
# for the prior and its renormalising sum, as test_gpu_net's leaf-prior test) and value (1e-5).  The
# checker is a float64 forward of the same weights (torch on the CPU): the engine's f32-equivalent
# products and the reference's own f32 CPU path each sit a few 1e-6 off it, so two f32 paths can
# differ by twice that (measured: v 1.1e-5 engine vs oracle; tools/diag_prior.py,
# profiles/r02_diag_prior.log).  After MCTS.py:88-91's renormalisation over a few valid actions of
# small total mass, P inherits the logits' absolute error as a RELATIVE error (measured vs float64:
# engine 6.3e-5, the reference's torch fp32 4.8e-5, the oracle 5.9e-5), so P is checked in predict
# space (P x the valid mass, i.e. the pi that renormalises to it) at the north-star tolerance, and
# directly against the reference's own f32 forward: P's worst relative error (entries > 1e-3) may be
# at most REF_FACTOR times that of torch fp32 on the CPU over the same rows.  The engine's products
# carry 22-bit operands (fp16 hi + lo planes, all four products incl. lo*lo) and the policy softmax
# uses the accurate expf / logf, so its tails sit at torch fp32's (round 4: 3.73e-5 vs 4.49e-5 at
# the bench size, 6.10e-6 vs 4.53e-6 for the config-5 kaiming net); the check prints both.
RTOL_PI, ATOL_PI, ATOL_V = 3e-5, 1e-7, 1e-5
REF_FACTOR = 1.5
_NETS = {}


def torch_predict(sd, hidden, nblocks, states, dtype, chunk=4096):
    """YachtNNet.forward (yacht/pytorch/YachtNNet.py) on the CPU in `dtype`, eval mode, over
    state_to_vec of the states (the oracle's featurize, pinned to the reference): (pi, v) as
    NNetWrapper.predict returns them (exp(log_softmax), NNet.py:193)."""
    import torch
    from yacht_amd.nnet import YachtNNet
    key = (id(sd), hidden, nblocks, dtype)
    if key not in _NETS:
        m = YachtNNet(hidden=hidden, nblocks=nblocks).to(dtype)
        m.load_state_dict({k: torch.as_tensor(np.asarray(t)).to(dtype) for k, t in sd.items()})
        _NETS[key] = m.eval()
    m = _NETS[key]
    x = torch.from_numpy(O.featurize(states)).to(dtype)
    pis, vs = [], []
    with torch.no_grad():
        for i in range(0, len(x), chunk):
            lg, v = m(x[i:i + chunk])
            pis.append(torch.exp(torch.log_softmax(lg, 1)).double().numpy())
            vs.append(v.double().numpy().reshape(-1))
    return np.concatenate(pis), np.concatenate(vs)


def renorm64(pi, ok):
    p = np.where(ok, np.asarray(pi, dtype=np.float64), 0.0)
    s = p.sum(1, keepdims=True)
    return np.divide(p, s, out=np.zeros_like(p), where=s > 0), s


def check_recorded_priors(pi, v, cnt, leaves, sd, hidden=256, nblocks=6, every=1, net=None):
    """The recorded priors (the production valid-only forward inside the engine, Ps * valids)
    renormalised as MCTS.py:88-91 does vs a float64 forward put through the same lines: zero
    outside the valid set; within the north-star tolerance in predict space; P and v no further
    from exact than REF_FACTOR x the reference's own f32 forward (v: or within 1e-5).
    net (a f32-mode YkNet of the same weights, GPU runs): the priors are also held at the north
    star's 1e-5 itself (rtol, predict space) against yk_net_predict's pi of the same leaves put
    through the same renormalisation - the predict test_gpu_net holds to 1e-5 of torch fp32 - so
    the engine's own ops (valid-only softmax statistics, exp_acc, the renormalising sum) add no
    more than that; v equal to predict's within 1e-6."""
    rs = np.concatenate([np.full(len(range(0, int(c), every)), r) for r, c in enumerate(cnt)])
    ks = np.concatenate([np.arange(0, int(c), every) for c in cnt])
    S = leaves[rs, ks]
    P = pi[rs, ks]
    ok, _ = O.valid(S, 1)
    ok = ok.astype(bool)
    assert not P[~ok].any()
    import torch
    tpi, tv = torch_predict(sd, hidden, nblocks, S, torch.float64)
    Pt, mass = renorm64(tpi, ok)
    none = ~ok.any(1)
    Pt[none, 0] = 1.0  # no valid action: P is one-hot on action 0 (MCTS.py:108-111)
    Pe = O.mcts_prior(P, S).astype(np.float64)  # exactly as the reference renormalises (f32, pairwise)
    np.testing.assert_allclose(Pe * mass, Pt * mass, rtol=RTOL_PI, atol=ATOL_PI)
    if net is not None and getattr(net, "precision", "f32") == "f32":
        from yacht_amd import kernels as K
        gp, gv = [], []
        for i in range(0, len(S), 4096):
            p_, v_ = net.predict_states(K.states_to_device(np.ascontiguousarray(S[i:i + 4096])))
            gp.append(p_.cpu().numpy())
            gv.append(v_.cpu().numpy())
        Pg, _ = renorm64(np.concatenate(gp), ok)
        Pg[none, 0] = 1.0
        d = np.abs(Pe - Pg) * mass
        tol = 1e-5 * np.abs(Pg) * mass + ATOL_PI
        print(f"engine priors vs yk_net_predict, predict space: max |d| / (1e-5 |pi| + 1e-7) = {float((d / tol).max()):.3f}")
        np.testing.assert_allclose(Pe * mass, Pg * mass, rtol=1e-5, atol=ATOL_PI)
        np.testing.assert_allclose(v[rs, ks], np.concatenate(gv), rtol=0, atol=1e-6)
    # v within 1e-5 of exact, or no worse than the reference's own f32 CPU forward (x REF_FACTOR);
    # P no worse than that forward, relative to exact arithmetic
    rpi, rv = torch_predict(sd, hidden, nblocks, S, torch.float32)
    verr_e, verr_r = float(np.abs(v[rs, ks] - tv).max()), float(np.abs(rv - tv).max())
    assert verr_e <= max(ATOL_V, REF_FACTOR * verr_r), (verr_e, verr_r)
    Pr, _ = renorm64(rpi, ok)
    Pr[none, 0] = 1.0
    big = Pt > 1e-3
    err_e = float((np.abs(Pe - Pt)[big] / Pt[big]).max())
    err_r = float((np.abs(Pr - Pt)[big] / Pt[big]).max())
    print(f"priors of {len(rs)} leaves: max rel err of P vs float64 {err_e:.2e} (torch fp32 {err_r:.2e}), "
          f"max |v err| {verr_e:.2e} (torch fp32 {verr_r:.2e})")
    assert err_e <= REF_FACTOR * err_r, (err_e, err_r)
    return len(rs)


# ---- the trainers' dropout keep masks on the host (yk_common.h dropout_bits), for torch references
_M32 = np.uint64(0xFFFFFFFF)


def philox_draw64_np(seed, env, ctr):
    """Philox4x32-10 of (ctr lo, ctr hi, env, 0) under key (seed lo, seed hi), the first two words:
    yk_common.h philox_draw / oracle/spec.py draw64, vectorised over ctr (uint64 array)."""
    ctr = np.asarray(ctr, dtype=np.uint64)
    c0, c1 = ctr & _M32, ctr >> np.uint64(32)
    c2 = np.full_like(ctr, np.uint64(int(env) & 0xFFFFFFFF))
    c3 = np.zeros_like(ctr)
    k0, k1 = np.uint64(int(seed) & 0xFFFFFFFF), np.uint64((int(seed) >> 32) & 0xFFFFFFFF)
    for _ in range(10):
        p0, p1 = np.uint64(0xD2511F53) * c0, np.uint64(0xCD9E8D57) * c2
        c0, c1, c2, c3 = (p1 >> np.uint64(32)) ^ c1 ^ k0, p1 & _M32, (p0 >> np.uint64(32)) ^ c3 ^ k1, p0 & _M32
        k0, k1 = (k0 + np.uint64(0x9E3779B9)) & _M32, (k1 + np.uint64(0xBB67AE85)) & _M32
    return c0 | (c1 << np.uint64(32))


def dropout_keep_np(seed, layer, step, rows, H, p, row_base=0):
    """The keep mask [rows, H] of dropout layer `layer` (0: inp, 1 + b: block b) at dropout step
    `step`: element e = (row_base + row) H + col is kept iff the 16-bit uniform (bits 16 (e % 4) ..)
    of the draw of its group e // 4 is >= p (yk_common.h dropout_bits / dropout_keep)."""
    g = (np.arange(rows, dtype=np.uint64)[:, None] + np.uint64(row_base)) * np.uint64(H // 4) + \
        np.arange(H // 4, dtype=np.uint64)[None, :]
    d = philox_draw64_np(seed, 0x44524F50 + layer, (np.uint64(step) << np.uint64(32)) ^ g)
    u = (d[:, :, None] >> (np.uint64(16) * np.arange(4, dtype=np.uint64))) & np.uint64(0xFFFF)
    keep = u.astype(np.float32) * np.float32(1.0 / 65536.0) >= np.float32(p)
    return keep.reshape(rows, H)


# ---- the replay examples from host copies of record images (numpy; yk_examples_from_records restated)
def host_examples(images: np.ndarray, n_envs: int, max_moves: int, sims: int, n_games: int = -1) -> dict:
    """The same examples from host copies of the record images, with the full policies
    (Coach.py:57-61: MCTS.getActionProb's pi per move - one-hot at the played action at temp 0,
    N / sum(N) at temp 1, MCTS.py:44-54) as a sparse CSR.  An
    independent restatement of yk_examples_from_records / yk_examples_policies (tests, the 2-rank
    CPU rehearsal).  Test infrastructure (moved here from yacht_amd/replay.py in round 6)."""
    from yacht_amd.engine import unpack_record_image
    from yacht_amd.replay import _vcap
    imgs = np.ascontiguousarray(images).reshape(images.shape[0] if images.ndim > 1 else 1, -1)
    total_games = imgs.shape[0] * n_envs
    n_games = total_games if n_games is None or n_games < 0 else min(n_games, total_games)
    parts = {k: [] for k in ("states", "values", "targets", "cols", "vals", "lens")}
    for r in range(imgs.shape[0]):
        g = min(max(n_games - r * n_envs, 0), n_envs)
        if g == 0:
            continue
        img = unpack_record_image(imgs[r], n_envs, max_moves, sims)
        nm = np.clip(img["n_moves"][:g], 0, max_moves)
        mask = np.arange(max_moves)[None, :] < nm[:, None]
        e_idx, m_idx = np.nonzero(mask)
        info = img["info"][:g][mask]
        temp, action = info[:, 0], info[:, 2]
        voff = img["voff"]
        a0, a1 = voff[e_idx, m_idx].astype(np.int64), voff[e_idx, m_idx + 1].astype(np.int64)
        hot = temp != 0
        lens = np.where(hot, a1 - a0, 1)
        n = len(temp)
        starts = np.concatenate([[0], np.cumsum(lens)])
        within = np.arange(starts[-1]) - np.repeat(starts[:-1], lens)
        row = np.repeat(np.arange(n), lens)
        vcap = _vcap(max_moves, sims)
        raw = img["visits_raw"].reshape(-1)[(e_idx[row].astype(np.int64) * vcap + a0[row] + within)
                                           .clip(0, n_envs * vcap - 1)]
        cols = np.where(hot[row], (raw >> 16).astype(np.int64), action[row].astype(np.int64))
        cnt = np.where(hot[row], (raw & 0xFFFF).astype(np.float64), 1.0)
        sums = np.bincount(row, weights=cnt, minlength=n)
        vals = cnt / np.where(sums[row] > 0, sums[row], 1.0)
        # argmax(pi): the most visited action, the lowest on ties (ascending action order)
        mx = np.zeros(n)
        np.maximum.at(mx, row, cnt)
        big = np.iinfo(np.int64).max
        first = np.full(n, big, dtype=np.int64)
        np.minimum.at(first, row, np.where(cnt == mx[row], cols, big))
        targets = np.where((first == big) | (mx == 0), action, first).astype(np.int32)
        keep = cnt > 0  # the examples file stores the nonzero entries of pi
        kl = np.bincount(row[keep], minlength=n)
        parts["states"].append(img["states"][:g][mask])
        parts["values"].append(img["values"][:g][mask])
        parts["targets"].append(targets)
        parts["cols"].append(cols[keep].astype(np.int32))
        parts["vals"].append(vals[keep])
        parts["lens"].append(kl)
    cat = {k: (np.concatenate(v) if v else None) for k, v in parts.items()}
    n = 0 if cat["targets"] is None else len(cat["targets"])
    lens = cat["lens"] if cat["lens"] is not None else np.zeros(0, np.int64)
    return dict(states=cat["states"] if n else np.zeros((0, 8), np.uint64),
                values=cat["values"] if n else np.zeros(0),
                targets=cat["targets"] if n else np.zeros(0, np.int32),
                pi_indptr=np.concatenate([[0], np.cumsum(lens)]).astype(np.int64),
                pi_cols=cat["cols"] if n else np.zeros(0, np.int32),
                pi_vals=cat["vals"] if n else np.zeros(0))
