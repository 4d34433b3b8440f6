"""diagnostic (CPU): where does the engine prior's error beyond torch fp32's come from?

A numpy emulation of k_forward's arithmetic (csrc/yk_net.hip) at hidden 256 x 6 blocks over the
reference's own fixture states (tests/golden/states.npz) with switches for each candidate error
source the round-3 verdict names:
  * the GEMM operands: hi/lo fp16 planes (22-bit operands, yk_net.hip put_planes / ld_w2) or exact
    f32 operands, per side (activations A, weights W), and the dropped lo x lo product;
  * MFMA accumulation: exact products, summed per 32-deep slice and added to an f32 accumulator
    (one rounding per v_mfma_f32_16x16x32_f16), the hi.hi and the cross-term accumulators combined
    once (combine());
  * SiLU: the kernel's exp2(-u log2 e) + 1 and reciprocal (silu2) or IEEE exp and division;
  * LayerNorm: one-pass shifted statistics + reciprocal square root (ln_stats2) or two-pass + 1/sqrt;
  * the leaf prior: exp(x - m - log sum) over the valid tiles, renormalised as MCTS.py:88-91.
Hardware exp2 / rcp / rsq / log are modelled as correctly rounded f32 results (their own <= 1 ulp
errors are not emulated; --ulp-noise adds +-1 ulp random perturbations to each).

Reported, per variant: P's max and rms relative error (entries with P > 1e-3) against a float64
forward, and the same for torch's float32 CPU forward (the reference's arithmetic).
usage: python tools/prior_error_emulation.py [--rows 2000] [--weights closed|kaiming]
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "nypc-yacht-auction_amd"), os.path.join(REPO, "tests")]
from oracle import oracle as O  # noqa: E402
from oracle import spec  # noqa: E402

F32, F64 = np.float32, np.float64
SPLIT = F32(2048.0)
LOG2E = F32(1.4426950408889634)
RNG = np.random.RandomState(1)
NOISE = [False]


def r32(x):
    """round to f32 (from f64); with --ulp-noise, a random +-1 ulp on top (hardware transcendental)"""
    y = np.asarray(x, dtype=F64).astype(F32)
    if NOISE[0]:
        k = RNG.randint(-1, 2, size=y.shape).astype(np.int32) * (np.isfinite(y) & (np.abs(y) > 1e-30))
        y = (y.view(np.int32) + k).view(F32)
    return y


def planes(x):
    h = x.astype(np.float16)
    lo = ((x - h.astype(F32)) * SPLIT).astype(np.float16)
    return h.astype(F64), lo.astype(F64)


def gemm(A, W, cfg):
    """A [n, K] f32 x W [N, K]^T -> f32 [n, N], the kernel's MFMA arithmetic"""
    n, K = A.shape
    Kp = (K + 31) // 32 * 32
    if Kp != K:
        A = np.pad(A, ((0, 0), (0, Kp - K)))
        W = np.pad(W, ((0, 0), (0, Kp - K)))
    if cfg["exact_a"]:
        ah, al = A.astype(F64), np.zeros_like(A, dtype=F64)
    else:
        ah, al = planes(A)
    if cfg["exact_w"]:
        wh, wl = W.astype(F64), np.zeros_like(W, dtype=F64)
    else:
        wh, wl = planes(W)
    m = np.zeros((n, W.shape[0]), F32)
    c = np.zeros_like(m)
    d = np.zeros_like(m)
    for ks in range(Kp // 32):
        s = slice(32 * ks, 32 * ks + 32)
        m = (m.astype(F64) + ah[:, s] @ wh[:, s].T).astype(F32)
        c = (c.astype(F64) + ah[:, s] @ wl[:, s].T).astype(F32)
        c = (c.astype(F64) + al[:, s] @ wh[:, s].T).astype(F32)
        if cfg["lolo"] == "scaled":  # the kernel's form: lo * 2^-11 as an fp16 operand into the cross terms
            als = (al[:, s].astype(np.float16) * np.float16(1.0 / 2048.0)).astype(F64)
            c = (c.astype(F64) + als @ wl[:, s].T).astype(F32)
        elif cfg["lolo"]:
            d = (d.astype(F64) + al[:, s] @ wl[:, s].T).astype(F32)
    out = (m + c * F32(1.0 / 2048.0)).astype(F32)
    if cfg["lolo"] is True:
        out = (out + d * F32(1.0 / 2048.0 / 2048.0)).astype(F32)
    return out


def silu(u, cfg):
    u = u.astype(F32)
    if cfg["ieee_silu"]:
        e = np.exp(-u.astype(F64)).astype(F32)
        return (u / (F32(1) + e)).astype(F32)
    a = (u * -LOG2E).astype(F32)
    d = (r32(np.exp2(a.astype(F64))) + F32(1)).astype(F32)
    return (u * r32(1.0 / d.astype(F64))).astype(F32)


def layernorm(x, g, b, cfg, H):
    x = x.astype(F32)
    if cfg["twopass_ln"]:
        mean = (x.sum(1, dtype=F32) / F32(H)).astype(F32)[:, None]
        dv = (x - mean).astype(F32)
        var = ((dv * dv).sum(1, dtype=F32) / F32(H)).astype(F32)[:, None]
        rstd = (1.0 / np.sqrt((var + F32(1e-5)).astype(F64))).astype(F32)
    else:
        sh = x[:, :1]
        dv = (x - sh).astype(F32)
        s = dv.sum(1, dtype=F32)[:, None]
        q = (dv * dv).sum(1, dtype=F32)[:, None]
        m = (s / F32(H)).astype(F32)
        var = np.maximum((q / F32(H) - m * m).astype(F32), F32(0))
        rstd = r32(1.0 / np.sqrt((var + F32(1e-5)).astype(F64)))
        mean = (sh + m).astype(F32)
    return ((((x - mean) * rstd).astype(F32) * g).astype(F32) + b).astype(F32)


def forward(sd, X, cfg, H=256, NB=6):
    L = lambda name: (np.asarray(sd[name + ".weight"], F32), np.asarray(sd[name + ".bias"], F32))
    only = cfg.get("lolo_only")  # the lo*lo product in these layers only ("inp", "trunk", "head")

    def G(A, W, where):
        return gemm(A, W, cfg if only is None else dict(cfg, lolo=cfg["lolo"] if where in only else False))
    blocks = cfg.get("lolo_blocks")  # with "trunk" in lolo_only: the blocks (0 .. NB-1) that get it
    w, b = L("inp.0")
    g, be = L("inp.1")
    h = silu(layernorm(G(X, w, "inp") + b, g, be, cfg, H), cfg)
    for k in range(NB):
        w1, b1 = L(f"blocks.{k}.fc1")
        g1, e1 = L(f"blocks.{k}.ln1")
        w2, b2 = L(f"blocks.{k}.fc2")
        g2, e2 = L(f"blocks.{k}.ln2")
        tw = "trunk" if blocks is None or k in blocks else "-"
        t = layernorm(silu(G(h, w1, tw) + b1, cfg), g1, e1, cfg, H)
        t = layernorm(silu(G(t, w2, tw) + b2, cfg), g2, e2, cfg, H)
        h = (h + t).astype(F32)
    gp, bp = L("pi_head.0")
    wp, bpi = L("pi_head.2")
    a = silu(layernorm(h, gp, bp, cfg, H), cfg)
    return (G(a, wp, "head") + bpi).astype(F32)


def leaf_prior(logits, ok):
    """the engine's P before renormalisation: exp(x - m - log sum exp) over the tiles holding a
    valid action (yk_net.hip pi_chunk statistics, k_leaf_prior / the expand's prior pass)"""
    n, A = ok.shape
    tiles = np.zeros((n, (A + 15) // 16 * 16), bool)
    okp = np.pad(ok, ((0, 0), (0, tiles.shape[1] - A)))
    tiles[:] = np.repeat(okp.reshape(n, -1, 16).any(2), 16, axis=1)
    keep = tiles[:, :A]
    x = np.where(keep, logits, -np.inf).astype(F32)
    m = x.max(1, keepdims=True)
    e = r32(np.exp((x - m).astype(F64)))
    s = e.sum(1, dtype=F32, keepdims=True)
    lse = r32(np.log(s.astype(F64)))
    return np.where(ok, r32(np.exp(((logits - m).astype(F32) - lse).astype(F64))), F32(0))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2000)
    ap.add_argument("--weights", default="closed", choices=["closed", "kaiming"])
    ap.add_argument("--ulp-noise", action="store_true")
    args = ap.parse_args()
    NOISE[0] = args.ulp_noise
    import torch
    from helpers import renorm64, torch_predict
    if args.weights == "closed":
        sd = spec.closed_form_weights(256, 6)
    else:
        from yacht_amd.nnet import YachtNNet
        torch.manual_seed(0)
        sd = {k: v.numpy() for k, v in YachtNNet(hidden=256, nblocks=6).state_dict().items()}
    S = np.load(os.path.join(REPO, "tests/golden/states.npz"))["states"]
    ok = O.valid(S, 1)[0].astype(bool)
    keep = ok.any(1)
    S, ok = S[keep][:args.rows], ok[keep][:args.rows]
    X = O.featurize(S).astype(F32)
    tpi, _ = torch_predict(sd, 256, 6, S, torch.float64)
    Pt, _ = renorm64(tpi, ok)
    big = Pt > 1e-3
    rpi, _ = torch_predict(sd, 256, 6, S, torch.float32)
    Pr, _ = renorm64(rpi, ok)

    def err(P):
        r = np.abs(P - Pt)[big] / Pt[big]
        return float(r.max()), float(np.sqrt((r * r).mean()))

    base = dict(exact_a=False, exact_w=False, lolo=False, ieee_silu=False, twopass_ln=False)
    only = os.environ.get("YK_EMU_ONLY")  # a substring: run the matching variants only
    variants = [
        ("kernel (r03: hi/lo planes, no lo*lo, hw SiLU, one-pass LN + rsq)", {}),
        ("+ lo*lo product (own accumulator)", dict(lolo=True)),
        ("+ lo*lo as (lo 2^-11 in fp16) x lo into the cross terms", dict(lolo="scaled")),
        ("exact activations (A operand f32)", dict(exact_a=True)),
        ("exact weights (W operand f32)", dict(exact_w=True)),
        ("exact operands (both f32; MFMA accumulation kept)", dict(exact_a=True, exact_w=True)),
        ("IEEE SiLU (exp + division)", dict(ieee_silu=True)),
        ("two-pass LayerNorm + exact 1/sqrt", dict(twopass_ln=True)),
        ("IEEE SiLU + two-pass LN", dict(ieee_silu=True, twopass_ln=True)),
        ("lo*lo + IEEE SiLU + two-pass LN", dict(lolo=True, ieee_silu=True, twopass_ln=True)),
        ("lo*lo (scaled) + exact activations", dict(lolo="scaled", exact_a=True)),
        ("lo*lo (scaled) in the policy head only", dict(lolo="scaled", lolo_only=("head",))),
        ("lo*lo (scaled) in the input layer + policy head", dict(lolo="scaled", lolo_only=("inp", "head"))),
        ("lo*lo (scaled) in the trunk only", dict(lolo="scaled", lolo_only=("inp", "trunk"))),
        ("lo*lo (scaled) in the input layer only", dict(lolo="scaled", lolo_only=("inp",))),
        ("lo*lo (scaled) in the input layer + blocks 0-2", dict(lolo="scaled", lolo_only=("inp", "trunk"), lolo_blocks=(0, 1, 2))),
        ("lo*lo (scaled) in the input layer + blocks 3-5", dict(lolo="scaled", lolo_only=("inp", "trunk"), lolo_blocks=(3, 4, 5))),
        ("lo*lo (scaled) in blocks 0-5, not the input layer", dict(lolo="scaled", lolo_only=("trunk",))),
        ("lo*lo (scaled) in block 0 only", dict(lolo="scaled", lolo_only=("trunk",), lolo_blocks=(0,))),
        ("lo*lo (scaled) in blocks 0-1 only", dict(lolo="scaled", lolo_only=("trunk",), lolo_blocks=(0, 1))),
        ("lo*lo (scaled) in block 1 only", dict(lolo="scaled", lolo_only=("trunk",), lolo_blocks=(1,))),
        ("lo*lo (scaled) in block 2 only", dict(lolo="scaled", lolo_only=("trunk",), lolo_blocks=(2,))),
    ]
    e_r = err(Pr)
    print(f"{len(S)} fixture states with a valid action, weights {args.weights}, ulp noise {args.ulp_noise}; "
          f"{int(big.sum())} priors > 1e-3")
    print(f"{'torch float32 (CPU, the reference arithmetic)':62s} max {e_r[0]:.3e}  rms {e_r[1]:.3e}")
    for name, over in variants:
        if only and only not in name:
            continue
        cfg = dict(base, **over)
        lg = forward(sd, X, cfg)
        P = O.mcts_prior(leaf_prior(lg, ok), S).astype(F64)
        e = err(P)
        print(f"{name:62s} max {e[0]:.3e}  rms {e[1]:.3e}   (x{e[0] / e_r[0]:.2f} / x{e[1] / e_r[1]:.2f} torch f32)",
              flush=True)


if __name__ == "__main__":
    main()
