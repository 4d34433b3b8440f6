// yk_fwd.h - the batched YachtNNet forward of one 16-row tile (forward_tile) behind k_forward
// (yk_net.hip: one workgroup of 8 waves per tile), which the predict entry points and the engine's
// simulations launch.  Device code only; see yk_net.hip for the design notes.
#pragma once
#include "yk_common.h"
#include "yk_net.h"

#include <type_traits>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));

namespace ykf {
using namespace yk;
namespace {


constexpr int ROWS = 16;     // rows per workgroup (the MFMA M)
constexpr int WAVES = 8;     // waves per workgroup
constexpr int NTHR = 64 * WAVES;
constexpr int RPW = ROWS / WAVES;  // rows per wave in the row passes
constexpr int PCH = 4;       // policy-head tiles per chunk
constexpr int YK_PW = 2;    // policy-head ring depth, two fp16 planes
// policy-head ring depth (32-deep slices): a single fp16 plane (PL = 1, the fp16 predict mode)
// takes half the registers per slice, so its ring is twice as deep
constexpr int pw_of(int PL) { return PL == 1 ? 2 * YK_PW : YK_PW; }
constexpr float SPLIT = 2048.f, UNSPLIT = 1.f / 2048.f;  // lo plane scale (keeps it out of fp16 subnormals)
constexpr int REAL_TILES = (ASIZE + 15) / 16;  // policy tiles holding an action column (202 of 204)
constexpr float FULL_SPREAD = 80.f;  // logit spread bound above which a workgroup takes the full pass

// SiLU with the hardware exp / reciprocal (<= 2 ulp each; well inside the 1e-5 contract)
__device__ __forceinline__ float silu(float x) { return x * __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }

template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp_f(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROW_MASK, 0xF, false));
}
// full-wave sum with DPP (quad perms, half-row / row mirrors, row broadcasts) -> lane 63
__device__ __forceinline__ float wave_sum(float v) {
    v += dpp_f<0xB1, 0xF>(v);   // quad_perm [1,0,3,2]
    v += dpp_f<0x4E, 0xF>(v);   // quad_perm [2,3,0,1]
    v += dpp_f<0x141, 0xF>(v);  // row_half_mirror
    v += dpp_f<0x140, 0xF>(v);  // row_mirror: every lane holds its 16-lane row sum
    v += dpp_f<0x142, 0xA>(v);  // row_bcast15 into rows 1, 3
    v += dpp_f<0x143, 0xC>(v);  // row_bcast31 into rows 2, 3
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops, NOT for its
// outstanding global loads (a __syncthreads() would drain vmcnt and the weight stream).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// One 16-column x 32-deep weight slice of a packed [N][K] matrix (yk_net.h): the hi and the lo
// plane, 1 KB each per wave (raw fp16 bits, 8 per lane).
struct W2 {
    float4 h, l;
};
// PL = 1 (fp16 predict mode) loads the hi plane only: half the weight bytes of the stream
template <int PL>
__device__ __forceinline__ W2 ld_w2(const float* __restrict__ P, int KS, int nt, int ks, int lane) {
    const float* p = P + ((long)(nt * KS + ks) * 2 * 64 + lane) * 4;
    if constexpr (PL == 1) return W2{*reinterpret_cast<const float4*>(p), make_float4(0.f, 0.f, 0.f, 0.f)};
    return W2{*reinterpret_cast<const float4*>(p), *reinterpret_cast<const float4*>(p + 256)};
}

__device__ __forceinline__ floatx4 mfma16(float4 a, float4 b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, a), __builtin_bit_cast(half8, b), c, 0, 0, 0);
}

// f32-equivalent product of one A slice (hi, lo planes) and one weight slice: four fp16 MFMAs
// (exact products, f32 accumulation): hi x hi into m; hi x lo, lo x hi and (lo 2^-11) x lo into
// c, which carries the 2^11 scale of the lo planes until combine().  lo 2^-11 is an exact power-of-
// two scaling in fp16 (v_pk_mul_f16) down to the fp16 subnormals (kept: denorm mode 16/64 = 3),
// whose 2^-25 absolute rounding is 2^-36 |w| of a product - below an f32 rounding of any product
// the lo*lo term matters to.
struct Acc3 {
    floatx4 m, c;
};
__device__ __forceinline__ void acc_zero(Acc3& a) { a.m = a.c = floatx4{0.f, 0.f, 0.f, 0.f}; }
template <int PL>
__device__ __forceinline__ floatx4 combine(const Acc3& a) {
    if constexpr (PL == 1) return a.m;
    return a.m + a.c * UNSPLIT;
}
__device__ __forceinline__ float4 lo_scaled(float4 al) {  // the lo plane x 2^-11, fp16
    return __builtin_bit_cast(float4, __builtin_bit_cast(half8, al) * (_Float16)(1.0f / 2048.0f));
}
// one 16x16x32 product into the accumulators: hi*hi (+ the three lo terms when PL = 2)
template <int PL>
__device__ __forceinline__ void mma3(Acc3& c, float4 ah, float4 al, const W2& w) {
    c.m = mfma16(ah, w.h, c.m);
    if constexpr (PL == 2) {
        c.c = mfma16(ah, w.l, c.c);
        c.c = mfma16(al, w.h, c.c);
        c.c = mfma16(lo_scaled(al), w.l, c.c);
    }
}

// A fragment of a plane pair in LDS (row stride SA halves): lane l reads row l & 15,
// k = 32 ks + 8 (l >> 4) .. + 7 of each plane.
struct APtr {
    const _Float16* h;
    const _Float16* l;
};
__device__ __forceinline__ APtr a_ptr(const _Float16* planes, int sa) {
    const int lane = threadIdx.x & 63;
    const int off = (lane & 15) * sa + 8 * (lane >> 4);
    return APtr{planes + off, planes + ROWS * sa + off};
}
__device__ __forceinline__ float4 ld_a(const _Float16* p, int ks) { return *reinterpret_cast<const float4*>(p + 32 * ks); }

// x -> (hi, lo * 2^11) into row r, column c of a plane pair (row stride sa halves), VPL values
template <int PL, int VPL>
__device__ __forceinline__ void put_planes(_Float16* planes, int sa, int r, int c, const float (&x)[VPL]) {
    _Float16 h[VPL], l[VPL];
#pragma unroll
    for (int i = 0; i < VPL; i++) {
        h[i] = (_Float16)x[i];
        l[i] = (_Float16)((x[i] - (float)h[i]) * SPLIT);
    }
    _Float16* ph = planes + r * sa + c;
    _Float16* pl = planes + ROWS * sa + r * sa + c;
    if constexpr (VPL == 4) {
        *reinterpret_cast<half4*>(ph) = half4{h[0], h[1], h[2], h[3]};
        if constexpr (PL == 2) *reinterpret_cast<half4*>(pl) = half4{l[0], l[1], l[2], l[3]};
    } else {
#pragma unroll
        for (int i = 0; i < VPL; i++) {
            ph[i] = h[i];
            if constexpr (PL == 2) pl[i] = l[i];
        }
    }
}

// acc[t] = A[16 x K] (plane pair in LDS) x W^T over this wave's NT tiles (nt0 ...), with the
// weight slices taken from the ring; slice ks lives in slot ks % RW.  After use, the slot is
// refilled with slice ks + RW of this layer (cur) or, past its end, of the next layer (nxt,
// same shape).
// DEF > 0: the last DEF slots' next-layer refills are left to the caller (ring_fill_part during the
// row pass that follows, where the CU's vector-memory path is otherwise idle).
// VH (the last trunk GEMM, RW == KS): each consumed slot's first tile is refilled with slice ks of
// tile `vt` of nxt (v_head.2's weights, read from the ring by the head).
template <int PL, int K, int NT, int RW, bool NEXT = true, int DEF = 0, bool VH = false>
__device__ __forceinline__ void mma_ring(const _Float16* A, int sa, W2 (&ring)[RW][NT], floatx4 (&acc)[NT],
                                         const float* __restrict__ cur, const float* __restrict__ nxt, int nt0,
                                         int vt = 0) {
    static_assert(!VH || (RW == K / 32 && !NEXT), "the v_head.2 refill replaces a one-layer ring's last refills");
    constexpr int KS = K / 32;
    const int lane = threadIdx.x & 63;
    const APtr ap = a_ptr(A, sa);
    Acc3 c[NT];
#pragma unroll
    for (int t = 0; t < NT; t++) acc_zero(c[t]);
    float4 ah = ld_a(ap.h, 0), al = ld_a(ap.l, 0);
#pragma unroll
    for (int ks = 0; ks < KS; ks++) {
        const float4 ahn = ld_a(ap.h, (ks + 1) % KS);
        const float4 aln = PL == 2 ? ld_a(ap.l, (ks + 1) % KS) : ahn;
        W2(&w)[NT] = ring[ks % RW];
#pragma unroll
        for (int t = 0; t < NT; t++) c[t].m = mfma16(ah, w[t].h, c[t].m);
        if constexpr (PL == 2) {
#pragma unroll
            for (int t = 0; t < NT; t++) c[t].c = mfma16(ah, w[t].l, c[t].c);
#pragma unroll
            for (int t = 0; t < NT; t++) c[t].c = mfma16(al, w[t].h, c[t].c);
            const float4 als = lo_scaled(al);
#pragma unroll
            for (int t = 0; t < NT; t++) c[t].c = mfma16(als, w[t].l, c[t].c);
        }
        const int g = ks + RW;
        if (g < KS || (NEXT && ks < KS - DEF)) {
#pragma unroll
            for (int t = 0; t < NT; t++)
                w[t] = g < KS ? ld_w2<PL>(cur, KS, nt0 + t, g, lane) : ld_w2<PL>(nxt, KS, nt0 + t, g - KS, lane);
        } else if constexpr (VH) {
            w[0] = ld_w2<PL>(nxt, KS, vt, ks, lane);
        }
        __builtin_amdgcn_sched_barrier(0);  // keep the refill here, a ring's depth ahead of its use
        ah = ahn;
        al = aln;
    }
#pragma unroll
    for (int t = 0; t < NT; t++) acc[t] = combine<PL>(c[t]);
}

// slices S0 .. S1-1 of the ring's first fill (the prologue issues the fill in parts)
template <int PL, int KS, int NT, int RW, int S0, int S1>
__device__ __forceinline__ void ring_fill_part(W2 (&ring)[RW][NT], const float* __restrict__ W, int nt0) {
    static_assert(0 <= S0 && S0 <= S1 && S1 <= RW, "slots within the ring");
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int ks = S0; ks < S1; ks++)
#pragma unroll
        for (int t = 0; t < NT; t++) ring[ks][t] = ld_w2<PL>(W, KS, nt0 + t, ks, lane);
}

// D[16 x 16] tile t of the wave: lane holds rows 4(l>>4)+j, column 16(nt0 + t) + (l&15).
// bias == nullptr: raw accumulators (the row pass adds the bias).
template <int NT>
__device__ __forceinline__ void store_acc(float* D, int ldd, int nt0, const floatx4 (&acc)[NT], const float* bias) {
    const int lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
#pragma unroll
    for (int t = 0; t < NT; t++) {
        const int c = 16 * (nt0 + t) + r;
        const float b = bias ? bias[c] : 0.f;
#pragma unroll
        for (int j = 0; j < 4; j++) D[(4 * q + j) * ldd + c] = bias ? acc[t][j] + b : acc[t][j];
    }
}

// nn.LayerNorm over H values held VPL per lane (two-pass, biased variance, eps 1e-5);
// g / b point into LDS
template <int VPL>
__device__ __forceinline__ void layernorm(float (&x)[VPL], const float* g, const float* b, int c0, int H) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; i++) s += x[i];
    const float mean = wave_sum(s) / (float)H;
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; i++) {
        const float d = x[i] - mean;
        v += d * d;
    }
    const float rstd = 1.0f / sqrtf(wave_sum(v) / (float)H + 1e-5f);
#pragma unroll
    for (int i = 0; i < VPL; i++) x[i] = (x[i] - mean) * rstd * g[c0 + i] + b[c0 + i];
}

// Packed forms of the row passes (two floats per VALU instruction: v_pk_add/mul_f32,
// v_cvt_pk_f16_f32) for even VPL: the same operations per element as silu / layernorm /
// put_planes, except that each lane's partial sums pair its values ((x0 + x2) + (x1 + x3)).
// The trunk's LayerNorm phases are VALU-bound and on the forward's critical path.
// The library builds with -ffp-contract=off (the search's f32 arithmetic rounds after every
// operation, as numpy does); the forward's LayerNorm row passes - VALU-bound and on every layer's
// critical path - contract their multiply-adds into v_pk_fma_f32 (one rounding instead of two: no
// less accurate than torch's own LayerNorm kernels, which fuse them too).  Scoped per function.
#ifndef FWD_SYNC_MODE
// (A/B) how a timed-out value-head wait is reported: 0 not at all, 1 LDS flag from a re-read of the
// count + the net's error word at the end, 2 NaN v for the tile, 3 LDS flag from the loop count + error word,
// 4 the error word written right after the wait (loop count)
#define FWD_SYNC_MODE 1
#endif
#define YK_ROW_CONTRACT _Pragma("clang fp contract(fast)")
typedef float f2v __attribute__((ext_vector_type(2)));
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v ld2(const float* p) { return *reinterpret_cast<const f2v*>(p); }
__device__ __forceinline__ f2v silu2(f2v u) {
    const f2v a = u * -1.4426950408889634f;  // exp(-u) = exp2(-u log2 e)
    f2v d, rc;
    d.x = __builtin_amdgcn_exp2f(a.x);
    d.y = __builtin_amdgcn_exp2f(a.y);
    d = d + 1.0f;
    rc.x = __builtin_amdgcn_rcpf(d.x);
    rc.y = __builtin_amdgcn_rcpf(d.y);
    return u * rc;
}
// LayerNorm of a wave's R rows at once, NP value pairs per lane: one pass of shifted sums
// (shift = the row's first value, so the variance E[(x-k)^2] - E[x-k]^2 does not cancel), the 2R
// wave reductions independent of each other (their DPP latencies overlap), rstd by v_rsq_f32.
// Four full-wave sums at once by a halving butterfly: the two quad steps trade halves of the
// 4-vector (3 DPP adds instead of 8), two row rotations and two cross-row shuffles then carry ONE
// value per lane, and the sums are read from lanes 0 (v0), 2 (v1), 1 (v2), 3 (v3).
__device__ __forceinline__ void wave_sum4(float (&v)[4]) {
    const int lane = threadIdx.x & 63;
    const bool b0 = (lane & 1) != 0, b1 = (lane & 2) != 0;
    float k0 = b0 ? v[2] : v[0], k1 = b0 ? v[3] : v[1];
    const float s0 = b0 ? v[0] : v[2], s1 = b0 ? v[1] : v[3];
    k0 += dpp_f<0xB1, 0xF>(s0);  // quad_perm [1,0,3,2]: even lanes now hold v0 / v1, odd v2 / v3
    k1 += dpp_f<0xB1, 0xF>(s1);
    float k = b1 ? k1 : k0;
    const float sd = b1 ? k0 : k1;
    k += dpp_f<0x4E, 0xF>(sd);  // quad_perm [2,3,0,1]: lane & 3 = 0 -> v0, 2 -> v1, 1 -> v2, 3 -> v3
    k += dpp_f<0x124, 0xF>(k);  // row_ror:4 and row_ror:8: the row's four quads (lane & 3 kept)
    k += dpp_f<0x128, 0xF>(k);
    k += xlane<16>(k);  // the wave's four rows (permlane swaps: no LDS round trip)
    k += xlane<32>(k);
    const int ki = __builtin_bit_cast(int, k);
    v[0] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(ki, 0));
    v[1] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(ki, 2));
    v[2] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(ki, 1));
    v[3] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(ki, 3));
}

template <int NP, int R>
__device__ __forceinline__ void ln_stats2(const f2v (&x)[R][NP], float (&mean)[R], float (&rstd)[R], int H) {
    YK_ROW_CONTRACT
    float sh[R], s[R], q[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
        sh[r] = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, x[r][0].x)));
        f2v a = {0.f, 0.f}, a2 = {0.f, 0.f};
#pragma unroll
        for (int i = 0; i < NP; i++) {
            const f2v d = x[r][i] - sh[r];
            a = a + d;
            a2 = a2 + d * d;
        }
        s[r] = a.x + a.y;
        q[r] = a2.x + a2.y;
    }
    if constexpr (R == 2) {
        float v4[4] = {s[0], q[0], s[1], q[1]};
        wave_sum4(v4);
        s[0] = v4[0];
        q[0] = v4[1];
        s[1] = v4[2];
        q[1] = v4[3];
    } else {
#pragma unroll
        for (int r = 0; r < R; r++) {
            s[r] = wave_sum(s[r]);
            q[r] = wave_sum(q[r]);
        }
    }
#pragma unroll
    for (int r = 0; r < R; r++) {
        const float m = s[r] / (float)H;
        const float var = fmaxf(q[r] / (float)H - m * m, 0.f);
        rstd[r] = __builtin_amdgcn_rsqf(var + 1e-5f);
        mean[r] = sh[r] + m;
    }
}
template <int NP, int R>
__device__ __forceinline__ void ln_apply2(f2v (&x)[R][NP], const float (&mean)[R], const float (&rstd)[R],
                                          const float* g, const float* b, int c0) {
    YK_ROW_CONTRACT
#pragma unroll
    for (int r = 0; r < R; r++)
#pragma unroll
        for (int i = 0; i < NP; i++) x[r][i] = (x[r][i] - mean[r]) * rstd[r] * ld2(g + c0 + 2 * i) + ld2(b + c0 + 2 * i);
}
template <int NP, int R>
__device__ __forceinline__ void layernorm2(f2v (&x)[R][NP], const float* g, const float* b, int c0, int H) {
    float mean[R], rstd[R];
    ln_stats2<NP, R>(x, mean, rstd, H);
    ln_apply2<NP, R>(x, mean, rstd, g, b, c0);
}
template <int PL, int NP>
__device__ __forceinline__ void put_planes2(_Float16* planes, int sa, int r, int c, const f2v (&x)[NP]) {
#pragma unroll
    for (int i = 0; i < NP; i++) {
        const h2v h = __builtin_convertvector(x[i], h2v);
        *reinterpret_cast<h2v*>(planes + r * sa + c + 2 * i) = h;
        if constexpr (PL == 2) {
            const f2v back = __builtin_convertvector(h, f2v);
            const h2v l = __builtin_convertvector((x[i] - back) * SPLIT, h2v);
            *reinterpret_cast<h2v*>(planes + ROWS * sa + r * sa + c + 2 * i) = l;
        }
    }
}

// Policy head chunks.  The workgroup computes the tiles of a list (every real tile, or the union
// of its rows' valid columns, TL in LDS); wave w owns list entries w + WAVES k, PCH of them per
// chunk, NTL <= PCH in a wave's last chunk.  The ring (RD slices of PCH tiles) streams across
// chunk boundaries: past the last slice it refills with the next chunk's first slices (NXT tiles).
// Chunk shapes are template parameters, so the loop body has no branches.
template <int PL, int KS, int NTL, int NXT, int PC = PCH, int RD = (pw_of(PL) < KS ? pw_of(PL) : KS), bool LL = true>
__device__ __forceinline__ void ring_chunk(const _Float16* A, int sa, W2 (&ring)[RD][PC], floatx4 (&pa)[NTL],
                                           const float* __restrict__ W, const int (&tile)[PC],
                                           const float* __restrict__ Wn, const int (&ntile)[PC]) {
    const int lane = threadIdx.x & 63;
    const APtr ap = a_ptr(A, sa);
    Acc3 c[NTL];
#pragma unroll
    for (int t = 0; t < NTL; t++) acc_zero(c[t]);
    float4 ah = ld_a(ap.h, 0), al = ld_a(ap.l, 0);
#pragma unroll
    for (int ks = 0; ks < KS; ks++) {
        const float4 ahn = ld_a(ap.h, (ks + 1) % KS);
        const float4 aln = PL == 2 ? ld_a(ap.l, (ks + 1) % KS) : ahn;
        W2(&w)[PC] = ring[ks % RD];
#pragma unroll
        for (int t = 0; t < NTL; t++) c[t].m = mfma16(ah, w[t].h, c[t].m);
        if constexpr (PL == 2) {
#pragma unroll
            for (int t = 0; t < NTL; t++) c[t].c = mfma16(ah, w[t].l, c[t].c);
#pragma unroll
            for (int t = 0; t < NTL; t++) c[t].c = mfma16(al, w[t].h, c[t].c);
            if constexpr (LL) {
                const float4 als = lo_scaled(al);
#pragma unroll
                for (int t = 0; t < NTL; t++) c[t].c = mfma16(als, w[t].l, c[t].c);
            }
        }
        const int g = ks + RD;
        if (g < KS) {
#pragma unroll
            for (int t = 0; t < NTL; t++) w[t] = ld_w2<PL>(W, KS, tile[t], g, lane);
        } else {
#pragma unroll
            for (int t = 0; t < NXT; t++) w[t] = ld_w2<PL>(Wn, KS, ntile[t], g - KS, lane);
        }
        __builtin_amdgcn_sched_barrier(0);
        ah = ahn;
        al = aln;
    }
#pragma unroll
    for (int t = 0; t < NTL; t++) pa[t] = combine<PL>(c[t]);
}
// Which logits of a row are stored (valid_only launches: the engine reads a leaf's logits only
// at its valid actions, MCTS.py:87-88, so the rest never leave the CU): per row a mode nibble -
// 0 none (no valid move, or no leaf), 1 the bids (YachtGame.py:379-383), 2 the score actions of
// unused categories at 10 dice (every combo), 3 the same at 5 dice (combo 0 only; :395-396),
// 4 every column (any other carry, or a full launch) - and the used-category mask << 4.
constexpr uint32_t LM_NONE = 0, LM_BID = 1, LM_SCORE10 = 2, LM_SCORE5 = 3, LM_ALL = 4;
__device__ __forceinline__ uint32_t logit_mode(const YkS& s) {
    const int round = s_round(s), phase = s_phase(s);
    if (phase == 0 && round != 13) return LM_BID;
    if (phase != 1) return LM_NONE;
    const uint64_t wa = s_pw(s, 0, 0);
    const int n = wa_n(wa);
    if (n < 5) return LM_NONE;
    const uint32_t used = (uint32_t)wa_used(wa) << 4;
    return n >= 10 ? (LM_SCORE10 | used) : n == 5 ? (LM_SCORE5 | used) : LM_ALL;
}
// Tile masks (204 bits = 7 words) of the columns a row keeps: the bids, every real column, each
// category's 252 combos, each category's combo 0.
constexpr int TMW = (PI_TILES + 31) / 32;
struct TileMasks {
    uint32_t bid[TMW], all[TMW], cat[NCAT][TMW], first[NCAT][TMW];
};
constexpr void tm_set(uint32_t (&m)[TMW], int c0, int c1) {  // columns c0 .. c1
    for (int t = c0 / 16; t <= c1 / 16; t++) m[t / 32] |= 1u << (t % 32);
}
constexpr TileMasks make_tile_masks() {
    TileMasks m{};
    tm_set(m.bid, 0, NBID - 1);
    tm_set(m.all, 0, ASIZE - 1);
    for (int c = 0; c < NCAT; c++) {
        tm_set(m.cat[c], NBID + NCOMB * c, NBID + NCOMB * c + NCOMB - 1);
        tm_set(m.first[c], NBID + NCOMB * c, NBID + NCOMB * c);
    }
    return m;
}
// word w of the mask of tiles t0 .. t1 (arithmetic: a per-lane constant-table load would be a
// vector load retiring behind the weight ring's first fill)
constexpr __host__ __device__ uint32_t tile_range_word(int t0, int t1, int w) {
    const int lo = t0 > 32 * w ? t0 : 32 * w, hi = t1 < 32 * w + 31 ? t1 : 32 * w + 31;
    return lo > hi ? 0u : (uint32_t)(((2ull << (hi - lo)) - 1ull) << (lo - 32 * w));
}
constexpr bool tile_words_match_tables() {
    const TileMasks m = make_tile_masks();
    for (int w = 0; w < TMW; w++) {
        bool ok = m.all[w] == tile_range_word(0, (ASIZE - 1) / 16, w) && m.bid[w] == tile_range_word(0, (NBID - 1) / 16, w);
        for (int c = 0; c < NCAT; c++) {
            const int a0 = NBID + NCOMB * c;
            ok = ok && m.cat[c][w] == tile_range_word(a0 / 16, (a0 + NCOMB - 1) / 16, w) &&
                 m.first[c][w] == tile_range_word(a0 / 16, a0 / 16, w);
        }
        if (!ok) return false;
    }
    return true;
}
static_assert(tile_words_match_tables(), "arithmetic tile words == the range tables");
// word w of the tile mask of a row with descriptor vd
__device__ __forceinline__ uint32_t tile_word(uint32_t vd, int w) {
    const uint32_t m = vd & 0xF;
    if (m == LM_NONE) return 0u;
    if (m == LM_ALL) return tile_range_word(0, (ASIZE - 1) / 16, w);
    if (m == LM_BID) return tile_range_word(0, (NBID - 1) / 16, w);
    uint32_t x = 0;
#pragma unroll
    for (int c = 0; c < NCAT; c++) {
        const int a0 = NBID + NCOMB * c;
        if (!((vd >> (4 + c)) & 1u)) x |= tile_range_word(a0 / 16, (m == LM_SCORE10 ? a0 + NCOMB - 1 : a0) / 16, w);
    }
    return x;
}

// Running softmax statistics (online form: max and sum exp(x - max)), merged over lanes and waves
// at the end of the head (the max of the parts first, then one rescale per part).  The native
// __expf suffices here: its relative error |y| 2^-24 on a term exp(y) is largest where the term is
// small, so the log-sum-exp moves by < 1e-7 (the expand's final exp(x - m - lse) is the accurate
// exp_acc, yk_common.h); the log is the library logf
// one chunk of policy tiles: a row's logits (+ bias) in the tiles it keeps a column in (`allc`:
// every real column) - a set that depends on the row alone - stored and folded into its running
// (max, sum exp): one rescale per row and chunk.  Lane (q, c) holds rows 4 q + j, column c.
// Three products, not four: the lo*lo term pays in the trunk, where its error compounds over 13
// layers, and not in this one layer (tools/prior_error_emulation.py: P's max relative error
// 3.59e-5 with lo*lo in the trunk only, 3.59e-5 everywhere, 7.47e-5 in the head only; torch f32
// 4.79e-5), while the head holds most of the forward's MFMAs.
template <int PL, int KS, int NTL, int NXT, int PC = PCH, int RD = (pw_of(PL) < KS ? pw_of(PL) : KS)>
__device__ __forceinline__ void pi_chunk(const _Float16* A, int sa, W2 (&ring)[RD][PC], const float* __restrict__ W,
                                         const int (&tile)[PC], const int (&ntile)[PC], const float* bias,
                                         float* __restrict__ logits, int row0, int n, float (&sm)[4], float (&ss)[4],
                                         const uint16_t* trb, const bool (&allc)[4]) {
    const int lane = threadIdx.x & 63;
    floatx4 pa[NTL];
    ring_chunk<PL, KS, NTL, NXT, PC, RD, false>(A, sa, ring, pa, W, tile, W, ntile);  // no lo*lo (below)
    const int rr = lane & 15, q = lane >> 4;
#pragma unroll
    for (int t = 0; t < NTL; t++) {
        const int col = 16 * tile[t] + rr;
        const float b = bias[col];
        const uint32_t rows = (uint32_t)trb[tile[t]] >> (4 * q);  // this lane's four rows
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int row = row0 + 4 * q + j;
            const bool mine = col < ASIZE && (allc[j] || ((rows >> j) & 1u));
            pa[t][j] += b;
            if (row < n && mine) logits[(long)row * PI_LD + col] = pa[t][j];
            if (!mine) pa[t][j] = -INFINITY;  // outside the row's softmax
        }
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
        float mn = sm[j];
#pragma unroll
        for (int t = 0; t < NTL; t++) mn = fmaxf(mn, pa[t][j]);
        if (mn != -INFINITY) {
            float acc = ss[j] > 0.f ? ss[j] * __expf(sm[j] - mn) : 0.f;
#pragma unroll
            for (int t = 0; t < NTL; t++) acc += __expf(pa[t][j] - mn);
            sm[j] = mn;
            ss[j] = acc;
        }
    }
}

// Row passes (LayerNorm / SiLU / residual): wave w owns rows RPW w ... RPW w + RPW - 1.
// PL = 2: f32-equivalent hi/lo planes (the parity mode); PL = 1: one fp16 plane of weights and
// GEMM inputs with f32 accumulation (the fp16 predict mode, as the reference's autocast('cuda')
// predict, NNet.py:186-189; LayerNorm, SiLU, softmax and the value head stay f32)
template <int H, int PL, int NW, bool NB0 = false>
__device__ __forceinline__ void forward_tile(NetDev net, const yk_state_t* __restrict__ states,
                                             const float* __restrict__ xin, const int32_t* __restrict__ rows,
                                             const int32_t* __restrict__ count, int n,
                                             float* __restrict__ logits, float* __restrict__ vout,
                                             const uint8_t* __restrict__ active, float2* __restrict__ mlse,
                                             int valid_only, uint32_t want, int parts, int mstride, int row0, int part) {
    constexpr int LD = (H > 128 ? H : 128) + 4;      // X also holds the 128-wide v_head hidden
    constexpr int SA = H + 8;                        // plane row stride (halves): conflict-free b128 reads
    constexpr int NT = H >= 16 * NW ? H / (16 * NW) : 1;  // 16-col tiles per wave, H-wide layers
    constexpr int NACT = H / (16 * NT);              // waves owning columns of the H-wide layers
    constexpr int VPL = H / 64;                      // values per lane in row passes
    constexpr int KS = H / 32;                       // 32-deep slices of an H-deep layer
    constexpr int YK_RCAP = 16;
    constexpr int RCAP = H >= 512 ? 8 : YK_RCAP;      // ring slices x tiles held per wave (VGPR budget)
    constexpr int RW = KS * NT <= RCAP ? KS : RCAP / NT;  // trunk ring depth (slices)
    constexpr int NVS = vstat_size(H), NVB = 6 * H;
    constexpr int TSZ = ROWS * LD > ROWS * SA ? ROWS * LD : ROWS * SA;  // T, or a_v's plane pair
    constexpr int NTH = 64 * NW, RPWN = ROWS / NW;
    static_assert(NW == 8 || NW == 16, "v_head.2's 8 column tiles map to waves 0-7 (16 waves: 8-15 repeat them)");
    __shared__ __attribute__((aligned(16))) float X[ROWS * LD];
    __shared__ __attribute__((aligned(16))) float T[TSZ];
    __shared__ __attribute__((aligned(16))) _Float16 P[2 * ROWS * SA];  // the next GEMM's input planes
    constexpr int NV4 = NVS / 4, PER = (NV4 + NTH - 1) / NTH;
    __shared__ __attribute__((aligned(16))) float VS[4 * NTH * PER];  // static vectors (yk_net.h VS_*; padded)
    constexpr int NB4 = NVB / 4, PB = (NB4 + NTH - 1) / NTH;
    __shared__ __attribute__((aligned(16))) float VB[4 * NTH * PB];  // this block's b1 g1 be1 b2 g2 be2 (padded)
    __shared__ uint32_t VD[ROWS];                            // per row: which logits are stored
    __shared__ float HN[ROWS];                               // per row: |a_pi|^2 (policy-head input)
    __shared__ uint8_t TL[PI_TILES];                         // policy tiles a valid-only pass computes
    __shared__ int TC;                                       // ... and their count
    __shared__ uint32_t UM[TMW];                             // the union of the rows' tile masks
    __shared__ uint32_t RM[ROWS][TMW];                       // each row's tile mask
    __shared__ uint16_t TRB[PI_TILES];                       // per tile: the rows that keep a column in it
    __shared__ uint32_t VHC;                                 // waves whose v_head.2 columns are in X
    __shared__ uint32_t SYNC_LOST;                           // a value-head wait timed out (FWD_ERR_SYNC)

    if (count) n = min(n, *count);
    if (row0 >= n) return;
    uint32_t amask = 0xFFFFu;  // rows with a leaf (bit r: row row0 + r)
    if (active) {  // uniform: every wave reads the same 16 flags (one scalar load when whole)
        amask = 0;
        if (row0 + ROWS <= n && (reinterpret_cast<uintptr_t>(active) & 15) == 0) {
            const uint4 a4 = *reinterpret_cast<const uint4*>(active + row0);
            const uint32_t w4[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
            for (int i = 0; i < ROWS; i++) amask |= (((w4[i >> 2] >> (8 * (i & 3))) & want) != 0 ? 1u : 0u) << i;
        } else {
#pragma unroll
            for (int i = 0; i < ROWS; i++) amask |= (row0 + i < n && (active[row0 + i] & want) ? 1u : 0u) << i;
        }
        if (!amask) return;
    }
    const float bv2 = net.b_v2[0];  // (v_head.4's bias, read at the end: loaded now, off that path)
    const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    // owns columns of the H-wide layers: every wave when NACT == NW (hidden >= 128), as a
    // compile-time true - a branch around the weight ring would make the wait counters merge at its
    // join, and the resulting vmcnt(0) drains the ring's in-flight refills of the next layer
    const bool gw = NACT == NW || wave < NACT;
    const int nt0 = wave * NT;
    const int c0 = lane * VPL;

    // loads in the order they are needed: the static vectors first (their LDS writes must not
    // wait behind the weight stream: vmcnt retires in order), then each wave's two state rows by
    // scalar loads (wave-uniform addresses: SMEM, lgkmcnt), then the weight stream - the input
    // layer and the first part of fc1's ring fill (the rest between the phases below) - and only
    // then the features
    constexpr int FPT = ROWS * 64 / NTH;  // feature rows per wave (row = wave + NW k)
    static_assert(FPT * NW == ROWS, "one feature row per wave and k");
    // the wave's state rows first: their scalar loads (both rows at once; the row map, when given,
    // read before them) fly beside the static vectors' round trip below instead of after it
    YkS fs[FPT];
    if (!xin) {
        int src[FPT];
#pragma unroll
        for (int k = 0; k < FPT; k++) {
            const int row = row0 + wave + NW * k;
            src[k] = row < n ? row : 0;
        }
        if (rows) {
#pragma unroll
            for (int k = 0; k < FPT; k++) src[k] = row0 + wave + NW * k < n ? rows[row0 + wave + NW * k] : 0;
        }
#pragma unroll
        for (int k = 0; k < FPT; k++) {
            const uint64_t* p = reinterpret_cast<const uint64_t*>(states + __builtin_amdgcn_readfirstlane(src[k]));
#pragma unroll
            for (int q = 0; q < 8; q++) fs[k].w[q] = p[q];
        }
    }
    float4 vsv[PER];
#pragma unroll
    for (int k = 0; k < PER; k++) vsv[k] = reinterpret_cast<const float4*>(net.vstat)[min(tid + NTH * k, NV4 - 1)];
#pragma unroll
    for (int k = 0; k < PER; k++)
        reinterpret_cast<float4*>(VS)[tid + NTH * k] = vsv[k];  // unconditional: the PER loads are waited for once
    // explicit features (predict on given rows) are loaded here, ahead of the weight stream: a
    // vector load issued after it would retire behind it (vmcnt is in order)
    float xv[FPT];
#pragma unroll
    for (int k = 0; k < FPT; k++) {
        const int row = row0 + wave + NW * k;
        xv[k] = 0.f;
        if (xin && row < n && lane < FEAT) xv[k] = xin[(long)(rows ? rows[row] : row) * FEAT + lane];
    }
    W2 w0[2][NT];
    W2 ring[RW][NT];
    // DUAL (the fp16 mode, one plane: a layer's slices take half the registers): a second ring, so
    // fc1 and fc2 each have their own - fc1's refills fetch the next block's fc1 and stream through
    // the row passes of fc1 and fc2, where a one-layer ring is full and the CU's stream stands idle
    constexpr bool DUAL = PL == 1 && NW == 8 && RW == KS;
    // DEF: each trunk GEMM's last DEF ring slots are refilled during the row pass that follows instead
    // of right after their MFMAs (mma_ring).  A wave's refills stall it while the CU's vector-memory
    // path is busy with every wave's loads, and that path is otherwise idle during the row passes;
    // the slices refilled late are the ones the next GEMM reads last.  Measured at 4096 x 100
    // (profiles/r05l_defer_ab.log): f32-equivalent forward 74.8 -> 72.4 us at 2 (1: 73.5, 3: 72.6),
    // the fp16 mode 52.4 -> 49.5 us at 4 (6: 50.6, 8: 53.0).
    constexpr int DEF = (RW == KS && VPL % 2 == 0) ? (PL == 2 ? 2 : 4) : 0;
    // VHP: v_head.2's weights (one 16-column tile per wave) stream into the trunk ring's slots during
    // the last trunk GEMM, whose slots otherwise go unrefilled, so the head computes that layer from
    // registers while its ring fetches the first policy chunk (streamed behind the heads' LayerNorm,
    // v_head.2 took ~11.6K of a workgroup's ~158K cycles: profiles/r05n_forward_phases.txt)
    constexpr bool VHP = RW == KS && NW == 8 && NACT == NW;  // (every wave runs the trunk GEMMs)
    const int vwave = wave & 7;  // v_head.2's tile: 8 of them (16 waves: waves 8-15 redo 0-7, unstored)
    // where in the row pass the two halves go: after the SiLU and after the statistics (f32-equivalent),
    // after the statistics and after the affine map (fp16 mode; profiles/r05l_defer_pos_ab.log)
    constexpr bool LATE = PL == 1;
    W2 ring2[DUAL ? RW : 1][NT];
    const float* w_first = net.NB > 0 ? net.w1 : net.w_in;  // (a valid address either way: see below)
    const float* w_second = net.NB > 0 ? net.w2 : net.w_in;
    if (gw) {
#pragma unroll
        for (int ks = 0; ks < 2; ks++)
#pragma unroll
            for (int t = 0; t < NT; t++) w0[ks][t] = ld_w2<PL>(net.w_in, 2, nt0 + t, ks, lane);
    }
    __builtin_amdgcn_sched_barrier(0);  // the input layer's slices ahead of the ring's (in-order vmcnt)
    // The ring's first fill in four parts, one between each of the prologue's phases: a wave issuing
    // its 32 loads at once stalls ~4.5K cycles on the CU's vector-memory path (which every wave's
    // loads share), where issued in parts its featurize / tile-mask / input-layer work runs while the
    // other waves' loads move; each part still lands long before the fc1 GEMM reads it.
    constexpr int RQ = RW / 4 > 0 ? RW / 4 : 1;
    constexpr int RQ2 = 2 * RQ < RW ? 2 * RQ : RW, RQ3 = 3 * RQ < RW ? 3 * RQ : RW;
    // (unconditional - no NB > 0 branch: a join there would make every later wait count the ring as
    // absent and over-wait; the slices are unused when NB = 0)
    if (gw) ring_fill_part<PL, KS, NT, RW, 0, RQ>(ring, w_first, nt0);
    __builtin_amdgcn_sched_barrier(0);  // the first layer streams in under the featurize / input phase
    // featurize (state_to_vec, NNet.py:65-86) straight into the input layer's planes, K = 64
    uint32_t vdk[FPT];
#pragma unroll
    for (int k = 0; k < FPT; k++) {
        const int rr = wave + NW * k, f = lane;
        const int row = row0 + rr;
        float val = 0.f;
        if (row < n && f < FEAT) val = xin ? xv[k] : feature(fs[k], f);
        const float one[1] = {val};
        put_planes<PL, 1>(P, SA, rr, f, one);
        const uint32_t vdr = row >= n || !((amask >> rr) & 1u) ? LM_NONE
                             : (valid_only && !xin) ? logit_mode(fs[k]) : LM_ALL;
        if (lane == 0) VD[rr] = vdr;
        vdk[k] = vdr;
    }
    if (gw) ring_fill_part<PL, KS, NT, RW, RQ, RQ2>(ring, w_first, nt0);  // part 2 of the first fill
    __builtin_amdgcn_sched_barrier(0);
    if (tid < TMW) UM[tid] = 0u;
    if (tid == 0) {
        VHC = 0u;
        SYNC_LOST = 0u;
    }
    lds_barrier();
    if (lane < TMW) {  // this wave's rows' tile masks, and into the union (read after the input barrier)
        uint32_t w = 0;
#pragma unroll
        for (int k = 0; k < FPT; k++) {
            const uint32_t x = tile_word(vdk[k], lane);
            RM[wave + NW * k][lane] = x;
            w |= x;
        }
        if (w) atomicOr(&UM[lane], w);
    }

    if (gw) ring_fill_part<PL, KS, NT, RW, RQ2, RQ3>(ring, w_first, nt0);  // part 3
    __builtin_amdgcn_sched_barrier(0);
    floatx4 acc[NT];
    // inp: Linear -> LayerNorm -> SiLU (-> Dropout, identity in eval)  YachtNNet.py:30-35
    if (gw) {
        const APtr ap = a_ptr(P, SA);
        Acc3 c[NT];
#pragma unroll
        for (int t = 0; t < NT; t++) acc_zero(c[t]);
#pragma unroll
        for (int ks = 0; ks < 2; ks++) {
            const float4 ah = ld_a(ap.h, ks);
            const float4 al = PL == 2 ? ld_a(ap.l, ks) : ah;
#pragma unroll
            for (int t = 0; t < NT; t++) mma3<PL>(c[t], ah, al, w0[ks][t]);
        }
#pragma unroll
        for (int t = 0; t < NT; t++) acc[t] = combine<PL>(c[t]);
        store_acc<NT>(T, LD, nt0, acc, nullptr);
    }
    lds_barrier();  // T complete; every wave is done reading the feature planes
    if (gw) {  // part 4 (and the fp16 mode's second ring)
        ring_fill_part<PL, KS, NT, RW, RQ3, RW>(ring, w_first, nt0);
        if constexpr (DUAL) ring_fill_part<PL, KS, NT, RW, 0, RW>(ring2, w_second, nt0);
    }
    __builtin_amdgcn_sched_barrier(0);
    // the union as an ascending list, and each tile's rows (read by the policy head): chunk c (tiles
    // 64 c .. 64 c + 63) built by wave c of 0-3, its list offset the union's bits below the chunk.  Built
    // in block 0, where waves 0-3 wait for the younger waves' fc2 weights, not here on the input
    // layer's path (one wave building all four chunks there held every wave ~3K cycles).
    auto build_tiles = [&](int c) __attribute__((always_inline)) {
        static_assert((PI_TILES + 63) / 64 == 4, "four 64-tile chunks");
        const int t = lane + 64 * c;
        if (t < PI_TILES) {
            uint32_t rb = 0;
#pragma unroll
            for (int r = 0; r < ROWS; r++) rb |= ((RM[r][t >> 5] >> (t & 31)) & 1u) << r;
            TRB[t] = (uint16_t)rb;
        }
        int base = 0, tot = 0;
#pragma unroll
        for (int j = 0; j < TMW; j++) {
            const int pc = __popc(UM[j]);
            base += j < 2 * c ? pc : 0;
            tot += pc;
        }
        const bool need = t < PI_TILES && ((UM[t >> 5] >> (t & 31)) & 1u);
        const uint64_t bal = __ballot(need);
        if (need) TL[base + __popcll(bal & ((1ull << lane) - 1))] = (uint8_t)t;
        if (c == 0 && lane == 0) TC = tot;
    };
    if constexpr (VPL % 2 == 0) {
        f2v x[RPWN][VPL / 2];
#pragma unroll
        for (int rr = 0; rr < RPWN; rr++)
#pragma unroll
            for (int i = 0; i < VPL / 2; i++)
                x[rr][i] = ld2(T + (wave * RPWN + rr) * LD + c0 + 2 * i) + ld2(VS + VS_BIN * H + c0 + 2 * i);
        layernorm2<VPL / 2, RPWN>(x, VS + VS_GIN * H, VS + VS_BEIN * H, c0, H);
#pragma unroll
        for (int rr = 0; rr < RPWN; rr++) {
            const int r = wave * RPWN + rr;
#pragma unroll
            for (int i = 0; i < VPL / 2; i++) {
                x[rr][i] = silu2(x[rr][i]);
                *reinterpret_cast<f2v*>(X + r * LD + c0 + 2 * i) = x[rr][i];
            }
            put_planes2<PL, VPL / 2>(P, SA, r, c0, x[rr]);
        }
    } else {
#pragma unroll
        for (int rr = 0; rr < RPWN; rr++) {
            const int r = wave * RPWN + rr;
            float x[VPL];
#pragma unroll
            for (int i = 0; i < VPL; i++) x[i] = T[r * LD + c0 + i] + VS[VS_BIN * H + c0 + i];
            layernorm<VPL>(x, VS + VS_GIN * H, VS + VS_BEIN * H, c0, H);
#pragma unroll
            for (int i = 0; i < VPL; i++) {
                x[i] = silu(x[i]);
                X[r * LD + c0 + i] = x[i];
            }
            put_planes<PL, VPL>(P, SA, r, c0, x);
        }
    }
    lds_barrier();

    // ResidualBlock x NB: h = LN1(SiLU(fc1 x)); h = LN2(SiLU(fc2 h)); x + h  YachtNNet.py:17-21
    // The last block is peeled (LAST: its refills stop) so that no branch joins streams of different
    // lengths inside the loop: at such a join the wait counters merge and the next GEMM's first wait
    // would drain the refills in flight.
    auto block = [&](int b, auto last_tag) __attribute__((always_inline)) {
        constexpr bool LAST = decltype(last_tag)::value;
        const long wo = (long)b * H * H;
        const float* after = net.w1 + wo + (long)H * H;  // the stream after fc2: the next block's fc1
        // where each GEMM's ring refills from (DUAL: fc1 -> the next block's fc1, fc2 -> its fc2)
        constexpr bool N1 = DUAL ? !LAST : true, N2 = !LAST;
        const float* nxt1 = DUAL ? after : net.w2 + wo;
        const float* nxt2 = DUAL ? net.w2 + wo + (long)H * H : after;
        // the GEMMs' deferred refills (DEF slots), issued in two parts inside the row pass that follows
        auto refill = [&](auto& rg, const float* nx, auto part) __attribute__((always_inline)) {
            constexpr int P0 = decltype(part)::value ? KS - DEF / 2 : KS - DEF;
            constexpr int P1 = decltype(part)::value ? KS : KS - DEF / 2;
            if (gw) ring_fill_part<PL, KS, NT, RW, P0, P1>(rg, nx, nt0);
            __builtin_amdgcn_sched_barrier(0);
        };
        float4 vb[PB];
#pragma unroll
        for (int k = 0; k < PB; k++) vb[k] = reinterpret_cast<const float4*>(net.vblk + (long)b * NVB)[min(tid + NTH * k, NB4 - 1)];
        if (gw) mma_ring<PL, H, NT, RW, N1, DEF>(P, SA, ring, acc, net.w1 + wo, nxt1, nt0);
#pragma unroll
        for (int k = 0; k < PB; k++)  // the previous block's readers passed a barrier; unconditional
            reinterpret_cast<float4*>(VB)[tid + NTH * k] = vb[k];  // (no branch join after the ring)
        if (gw) store_acc<NT>(T, LD, nt0, acc, nullptr);
        lds_barrier();  // T complete; every wave is done reading x's planes
        if constexpr (VPL % 2 == 0) {
            f2v x[RPWN][VPL / 2];
#pragma unroll
            for (int rr = 0; rr < RPWN; rr++)
#pragma unroll
                for (int i = 0; i < VPL / 2; i++)
                    x[rr][i] = silu2(ld2(T + (wave * RPWN + rr) * LD + c0 + 2 * i) + ld2(VB + c0 + 2 * i));
            if constexpr (DEF > 0 && N1 && !LATE) refill(ring, nxt1, std::false_type{});
            float mean[RPWN], rstd[RPWN];
            ln_stats2<VPL / 2, RPWN>(x, mean, rstd, H);
            if constexpr (DEF > 0 && N1) refill(ring, nxt1, std::integral_constant<bool, !LATE>{});
            ln_apply2<VPL / 2, RPWN>(x, mean, rstd, VB + H, VB + 2 * H, c0);
            if constexpr (DEF > 0 && N1 && LATE) refill(ring, nxt1, std::true_type{});
#pragma unroll
            for (int rr = 0; rr < RPWN; rr++) put_planes2<PL, VPL / 2>(P, SA, wave * RPWN + rr, c0, x[rr]);  // fc2's input
        } else {
#pragma unroll
            for (int rr = 0; rr < RPWN; rr++) {
                const int r = wave * RPWN + rr;
                float x[VPL];
#pragma unroll
                for (int i = 0; i < VPL; i++) x[i] = silu(T[r * LD + c0 + i] + VB[c0 + i]);
                layernorm<VPL>(x, VB + H, VB + 2 * H, c0, H);
                put_planes<PL, VPL>(P, SA, r, c0, x);  // fc2's input
            }
        }
        lds_barrier();
        if (gw) {
            // (the last block: v_head.2's tile into the consumed slots, VHP)
            constexpr bool V = LAST && VHP;
            const float* n2 = V ? net.w_v1 : nxt2;
            if constexpr (DUAL) mma_ring<PL, H, NT, RW, N2, DEF, V>(P, SA, ring2, acc, net.w2 + wo, n2, nt0, vwave);
            else mma_ring<PL, H, NT, RW, N2, DEF, V>(P, SA, ring, acc, net.w2 + wo, n2, nt0, vwave);
        }
        if (gw) store_acc<NT>(T, LD, nt0, acc, nullptr);
        if (b == 0 && wave < 4) build_tiles(wave);  // (waves 0-3: the tile list, above)
        auto refill2 = [&](auto part) __attribute__((always_inline)) {
            if constexpr (DUAL) refill(ring2, nxt2, part);
            else refill(ring, nxt2, part);
        };
        lds_barrier();  // T complete; every wave is done reading h's planes
        if constexpr (VPL % 2 == 0) {
            f2v x[RPWN][VPL / 2];
#pragma unroll
            for (int rr = 0; rr < RPWN; rr++)
#pragma unroll
                for (int i = 0; i < VPL / 2; i++)
                    x[rr][i] = silu2(ld2(T + (wave * RPWN + rr) * LD + c0 + 2 * i) + ld2(VB + 3 * H + c0 + 2 * i));
            if constexpr (DEF > 0 && N2 && !LATE) refill2(std::false_type{});
            float mean[RPWN], rstd[RPWN];
            ln_stats2<VPL / 2, RPWN>(x, mean, rstd, H);
            if constexpr (DEF > 0 && N2) refill2(std::integral_constant<bool, !LATE>{});
            ln_apply2<VPL / 2, RPWN>(x, mean, rstd, VB + 4 * H, VB + 5 * H, c0);
            if constexpr (DEF > 0 && N2 && LATE) refill2(std::true_type{});
#pragma unroll
            for (int rr = 0; rr < RPWN; rr++) {
                const int r = wave * RPWN + rr;
#pragma unroll
                for (int i = 0; i < VPL / 2; i++) {
                    x[rr][i] = x[rr][i] + ld2(X + r * LD + c0 + 2 * i);
                    *reinterpret_cast<f2v*>(X + r * LD + c0 + 2 * i) = x[rr][i];
                }
                if constexpr (!LAST) put_planes2<PL, VPL / 2>(P, SA, r, c0, x[rr]);  // the next fc1's input
            }
        } else {
#pragma unroll
            for (int rr = 0; rr < RPWN; rr++) {
                const int r = wave * RPWN + rr;
                float x[VPL];
#pragma unroll
                for (int i = 0; i < VPL; i++) x[i] = silu(T[r * LD + c0 + i] + VB[3 * H + c0 + i]);
                layernorm<VPL>(x, VB + 4 * H, VB + 5 * H, c0, H);
#pragma unroll
                for (int i = 0; i < VPL; i++) {
                    x[i] += X[r * LD + c0 + i];
                    X[r * LD + c0 + i] = x[i];
                }
                if constexpr (!LAST) put_planes<PL, VPL>(P, SA, r, c0, x);  // the next fc1's input
            }
        }
        lds_barrier();
    };
    // NB0 (nblocks = 0, a separate instantiation: no runtime branch joins the ring's streams here)
    if constexpr (!NB0) {
        for (int b = 0; b + 1 < net.NB; b++) block(b, std::false_type{});
        block(net.NB - 1, std::true_type{});
    } else {
        if (wave < 4) build_tiles(wave);  // (no block: read after the heads' LayerNorm barrier)
        // no last fc2 GEMM streamed v_head.2's tile into the ring the heads read (VHP): load it here
        if constexpr (VHP) {
            if (gw) {
#pragma unroll
                for (int ks = 0; ks < KS; ks++) {
                    if constexpr (DUAL) ring2[ks][0] = ld_w2<PL>(net.w_v1, KS, vwave, ks, lane);
                    else ring[ks][0] = ld_w2<PL>(net.w_v1, KS, vwave, ks, lane);
                }
            }
        }
    }

    // heads: pi_head = LN -> SiLU -> Linear; v_head = LN -> SiLU -> Linear -> SiLU -> Linear -> tanh.
    // One ring streams v_head.2 (one 16-column tile per wave, first) and then the policy head;
    // its first slices fly under the LayerNorms.  a_pi's planes go to P, a_v's to T's storage.
    constexpr int RD = pw_of(PL) < KS ? pw_of(PL) : KS;  // policy ring depth (slices)
    static_assert(KS % RD == 0 && KS % RW == 0, "a ring's refills cross into the next chunk / layer slot-aligned");
    _Float16* PV = reinterpret_cast<_Float16*>(T);
    // chunk width: 4 tiles per wave at 8 waves; 2 at 16 waves (128 VGPRs), the same bytes in flight
    constexpr int PC = NW == 16 ? 2 : PCH;
    W2 pring[RD][PC];
    if constexpr (!VHP) {
#pragma unroll
        for (int ks = 0; ks < RD; ks++) pring[ks][0] = ld_w2<PL>(net.w_v1, KS, vwave, ks, lane);
    }
    if constexpr (VPL % 2 == 0) {
        // both heads' LayerNorms see the same row: one set of statistics, two affine maps
        f2v x[RPWN][VPL / 2], y[RPWN][VPL / 2];
#pragma unroll
        for (int rr = 0; rr < RPWN; rr++)
#pragma unroll
            for (int i = 0; i < VPL / 2; i++) x[rr][i] = y[rr][i] = ld2(X + (wave * RPWN + rr) * LD + c0 + 2 * i);
        float mean[RPWN], rstd[RPWN];
        ln_stats2<VPL / 2, RPWN>(x, mean, rstd, H);
        ln_apply2<VPL / 2, RPWN>(x, mean, rstd, VS + VS_GPI * H, VS + VS_BEPI * H, c0);
        ln_apply2<VPL / 2, RPWN>(y, mean, rstd, VS + VS_GV * H, VS + VS_BEV * H, c0);
        float h2[RPWN];
#pragma unroll
        for (int rr = 0; rr < RPWN; rr++) {
            const int r = wave * RPWN + rr;
            f2v a = {0.f, 0.f};
#pragma unroll
            for (int i = 0; i < VPL / 2; i++) {
                x[rr][i] = silu2(x[rr][i]);  // a_pi
                y[rr][i] = silu2(y[rr][i]);  // a_v
                a = a + x[rr][i] * x[rr][i];
            }
            put_planes2<PL, VPL / 2>(P, SA, r, c0, x[rr]);
            put_planes2<PL, VPL / 2>(PV, SA, r, c0, y[rr]);
            h2[rr] = a.x + a.y;
        }
#pragma unroll
        for (int rr = 0; rr < RPWN; rr++) {
            const float t = wave_sum(h2[rr]);
            if (lane == 0) HN[wave * RPWN + rr] = t;
        }
    } else {
#pragma unroll
        for (int rr = 0; rr < RPWN; rr++) {
            const int r = wave * RPWN + rr;
            float x[VPL], y[VPL];
#pragma unroll
            for (int i = 0; i < VPL; i++) x[i] = y[i] = X[r * LD + c0 + i];
            layernorm<VPL>(x, VS + VS_GPI * H, VS + VS_BEPI * H, c0, H);
            layernorm<VPL>(y, VS + VS_GV * H, VS + VS_BEV * H, c0, H);
#pragma unroll
            for (int i = 0; i < VPL; i++) {
                x[i] = silu(x[i]);  // a_pi
                y[i] = silu(y[i]);  // a_v
            }
            put_planes<PL, VPL>(P, SA, r, c0, x);
            put_planes<PL, VPL>(PV, SA, r, c0, y);
            float h2 = 0.f;
#pragma unroll
            for (int i = 0; i < VPL; i++) h2 += x[i] * x[i];
            h2 = wave_sum(h2);
            if (lane == 0) HN[r] = h2;
        }
    }
    lds_barrier();
    // The policy head over all real tiles (full) or over the union of the rows' valid columns.
    // A row's softmax runs over every action (`allc`: the reference's exp(log_softmax), NNet.py:193)
    // or - engine rows - over the tiles holding its valid actions: pi_a / sum_valid(pi) (MCTS.py:88-91)
    // is the same number either way up to rounding, unless every valid pi underflows in the full softmax
    // (the reference then falls back to uniform, :93-107), which needs a valid logit ~100 below an
    // invalid one.  |logit_a - b_a| <= |W_a| |a_pi| bounds the spread of a row's logits by
    // (bmax - bmin) + 2 wmax |a_pi|; a row over FULL_SPREAD keeps the full softmax.  The choice
    // depends on the row alone, so a row's result does not depend on its workgroup.
    auto row_allc = [&](int r) {
        const uint32_t md = VD[r] & 0xF;
        return md == LM_ALL || (md != LM_NONE && net.pi_bspread + 2.f * net.pi_wmax * sqrtf(HN[r]) > FULL_SPREAD);
    };
    // lane r < ROWS decides row r (one round of LDS reads for all rows, not a chain of 16)
    const uint32_t allrows = (uint32_t)__ballot(lane < ROWS && row_allc(lane));
    const bool full = allrows != 0u;
    const int cnt_all = full ? REAL_TILES : __builtin_amdgcn_readfirstlane(TC);
    const int lo = cnt_all * part / parts, cnt = cnt_all * (part + 1) / parts - lo;  // this part's slice
    // this wave's list entries k = 0 .. m-1 (list index lo + wave + NW k): nf full chunks in list
    // order, then a last chunk of l entries.  Every workgroup walks its list in ascending tile
    // order: workgroups reading the same weight lines together is faster than spreading them
    // (a per-workgroup rotation of the chunk order cost 0.5 us)
    const int m = cnt > wave ? (cnt - wave + NW - 1) / NW : 0;
    const int nf = m / PC, l = m % PC, nch = nf + (l ? 1 : 0);

    auto chunk_tiles = [&](int c, int (&tl)[PC]) {  // (the PC list reads unconditional: one LDS round trip)
        const int k0 = PC * c;
        int v[PC];
#pragma unroll
        for (int t = 0; t < PC; t++) v[t] = TL[min(lo + wave + NW * (k0 + t), PI_TILES - 1)];
#pragma unroll
        for (int t = 0; t < PC; t++) {
            const int i = lo + wave + NW * (k0 + t);
            tl[t] = c < nch && k0 + t < m ? (full ? i : __builtin_amdgcn_readfirstlane(v[t])) : 0;
        }
    };
    auto chunk_n = [&](int c) { return c < nf ? PC : c < nch ? l : 0; };
    floatx4 av[1];  // v_head.2: Linear(H, 128), tile `wave`; its refills stream the first policy chunk
    const float* bpi = VS + vs_bpi(H);
    int tcur[PC], tnxt[PC];
    chunk_tiles(0, tcur);
    if constexpr (VHP) {
        // the first policy chunk's first RD slices (every slot: a short chunk's extra ones read tile 0),
        // then v_head.2 from the trunk ring (slice ks of tile vwave in slot ks, tile 0; same products
        // and order as ring_chunk's)
#pragma unroll
        for (int ks = 0; ks < RD; ks++)
#pragma unroll
            for (int t = 0; t < PC; t++) pring[ks][t] = ld_w2<PL>(net.w_pi, KS, tcur[t], ks, lane);
        __builtin_amdgcn_sched_barrier(0);
        auto vhead = [&](auto& vr) __attribute__((always_inline)) {
            const APtr ap = a_ptr(PV, SA);
            Acc3 c;
            acc_zero(c);
#pragma unroll
            for (int ks = 0; ks < KS; ks++) {
                const float4 ah = ld_a(ap.h, ks);
                const float4 al = PL == 2 ? ld_a(ap.l, ks) : ah;
                mma3<PL>(c, ah, al, vr[ks][0]);
            }
            av[0] = combine<PL>(c);
        };
        if constexpr (DUAL) vhead(ring2);
        else vhead(ring);
    } else {
        int vt[PC] = {};
        vt[0] = vwave;
        static_assert(PC == 4 || PC == 2, "chunk-shape dispatch below");
        switch (chunk_n(0)) {
            case 0: ring_chunk<PL, KS, 1, 0, PC>(PV, SA, pring, av, net.w_v1, vt, net.w_pi, tcur); break;
            case 1: ring_chunk<PL, KS, 1, 1, PC>(PV, SA, pring, av, net.w_v1, vt, net.w_pi, tcur); break;
            case 2: ring_chunk<PL, KS, 1, 2, PC>(PV, SA, pring, av, net.w_v1, vt, net.w_pi, tcur); break;
            case 3:
                if constexpr (PC >= 3) ring_chunk<PL, KS, 1, (PC >= 3 ? 3 : 1), PC>(PV, SA, pring, av, net.w_v1, vt, net.w_pi, tcur);
                break;
            default:
                ring_chunk<PL, KS, 1, PC, PC>(PV, SA, pring, av, net.w_v1, vt, net.w_pi, tcur);
                break;
        }
    }
    // v_head.2's columns into X (the trunk output, read by the heads' LayerNorms only), counted: waves
    // 0-3 compute the value head from them after their policy chunks, before the younger waves end
    // theirs (a wave's LDS operations complete in order, so its count follows its stores)
    constexpr uint32_t NVW = NW < 8 ? NW : 8;
    if (NW == 8 || wave < 8) {
        store_acc<1>(X, LD, vwave, av, VS + VS_BV1 * H);
        // the count's increment follows the column stores in this wave's LDS order (a wave's DS
        // operations execute in issue order), and the compiler fence keeps the stores ahead of it in
        // the code; a release atomic instead costs an lgkmcnt(0) drain here and ~0.5 us per forward
        // (profiles/r06g_forward_sync_ab.log)
        __atomic_signal_fence(__ATOMIC_RELEASE);
        if (lane == 0) atomicAdd(&VHC, 1u);
    }
    float sm[4], ss[4];  // running max and sum exp of the lane's rows 4 q + j
    bool allc[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        sm[j] = -INFINITY;
        ss[j] = 0.f;
        allc[j] = (allrows >> (4 * (lane >> 4) + j)) & 1u;
    }
#define YK_PI_CHUNK(NTL, NXT) \
    pi_chunk<PL, KS, NTL, NXT, PC>(P, SA, pring, net.w_pi, tcur, tnxt, bpi, logits, row0, n, sm, ss, TRB, allc)
#pragma unroll 1
    for (int c = 0; c < nch; c++) {
        chunk_tiles(c + 1, tnxt);
        const int nx = chunk_n(c + 1);
        if constexpr (PC == 4) {
            if (c < nf) {
                switch (nx) {
                    case 0: YK_PI_CHUNK(4, 0); break;
                    case 1: YK_PI_CHUNK(4, 1); break;
                    case 2: YK_PI_CHUNK(4, 2); break;
                    case 3: YK_PI_CHUNK(4, 3); break;
                    default: YK_PI_CHUNK(4, 4); break;
                }
            } else {
                switch (l) {
                    case 1: YK_PI_CHUNK(1, 0); break;
                    case 2: YK_PI_CHUNK(2, 0); break;
                    default: YK_PI_CHUNK(3, 0); break;
                }
            }
        } else {
            if (c < nf) {
                switch (nx) {
                    case 0: YK_PI_CHUNK(2, 0); break;
                    case 1: YK_PI_CHUNK(2, 1); break;
                    default: YK_PI_CHUNK(2, 2); break;
                }
            } else {
                YK_PI_CHUNK(1, 0);
            }
        }
#pragma unroll
        for (int t = 0; t < PC; t++) tcur[t] = tnxt[t];
    }
#undef YK_PI_CHUNK
    if (wave < 4) {  // SiLU -> Linear(128, 1) -> tanh  YachtNNet.py:49-52,69, rows 4 wave .. 4 wave + 3
        // (bounded: a wave that never sees every count flags the net's error word instead of hanging
        // the grid; yk_net_errors / the engine's ERR_FWD_SYNC report it)
        // (a relaxed atomic load is a ds_read; a volatile access through the generic pointer was a
        // flat load, whose wait also drained the wave's logit stores)
        int it = 0;
        for (; it < (1 << 20) && __hip_atomic_load(&VHC, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < NVW; it++)
            __builtin_amdgcn_s_sleep(1);
        // (reads of X stay after the count's: compiler fence; a timeout is flagged, reported at the
        // kernel's very end, where a global write adds no wait to any load in flight)
        __atomic_signal_fence(__ATOMIC_ACQUIRE);
        const bool lost = it >= (1 << 20);  // (wave-uniform)
        (void)lost;
#if FWD_SYNC_MODE == 1
        if (lane == 0 && __hip_atomic_load(&VHC, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < NVW) SYNC_LOST = 1u;
#elif FWD_SYNC_MODE == 3
        if (lost && lane == 0) SYNC_LOST = 1u;
#elif FWD_SYNC_MODE == 4
        // (here, in the older waves' slack before the end: only their own logit stores are in flight)
        if (lost && lane == 0 && net.err) atomicOr(net.err, FWD_ERR_SYNC);
#endif
#pragma unroll
        for (int rr = 0; rr < ROWS / 4; rr++) {
            const int r = wave * (ROWS / 4) + rr;
            const int row = row0 + r;
            const float* wv2 = VS + VS_BV1 * H + 128;
            float s = silu(X[r * LD + 2 * lane]) * wv2[2 * lane] + silu(X[r * LD + 2 * lane + 1]) * wv2[2 * lane + 1];
            s = wave_sum(s);
#if FWD_SYNC_MODE == 2
            const float vv = lost ? __builtin_nanf("") : tanhf(s + bv2);  // (a timed-out hand-off: NaN, never stale)
#else
            const float vv = tanhf(s + bv2);
#endif
            if (lane == 0 && part == 0 && row < n && ((amask >> r) & 1u)) vout[row] = vv;  // active rows only
        }
    }
    // softmax statistics of the policy logits per row: over the 16 column lanes, then the waves
    float2* SS = reinterpret_cast<float2*>(T);  // T (a_v's planes) is no longer read
    if (mlse) {  // over the 16 column lanes: the max first, then one rescale per lane and a sum (4 exps, not 32)
        float mm[4], t[4];
#pragma unroll
        for (int j = 0; j < 4; j++) mm[j] = fmaxf(sm[j], xlane<1>(sm[j]));
#pragma unroll
        for (int j = 0; j < 4; j++) mm[j] = fmaxf(mm[j], xlane<2>(mm[j]));
#pragma unroll
        for (int j = 0; j < 4; j++) mm[j] = fmaxf(mm[j], xlane<4>(mm[j]));
#pragma unroll
        for (int j = 0; j < 4; j++) mm[j] = fmaxf(mm[j], xlane<8>(mm[j]));
#pragma unroll
        for (int j = 0; j < 4; j++) t[j] = sm[j] == -INFINITY ? 0.f : ss[j] * __expf(sm[j] - mm[j]);
#pragma unroll
        for (int j = 0; j < 4; j++) t[j] += xlane<1>(t[j]);
#pragma unroll
        for (int j = 0; j < 4; j++) t[j] += xlane<2>(t[j]);
#pragma unroll
        for (int j = 0; j < 4; j++) t[j] += xlane<4>(t[j]);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            t[j] += xlane<8>(t[j]);
            sm[j] = mm[j];
            ss[j] = t[j];
        }
    }
    lds_barrier();  // every wave is done with v_head.2 (reads of T) and stored its av columns
    if (mlse && (lane & 15) == 0) {
#pragma unroll
        for (int j = 0; j < 4; j++) SS[wave * ROWS + 4 * (lane >> 4) + j] = make_float2(sm[j], ss[j]);
    }
    if (mlse) {
        lds_barrier();
        if (tid < ROWS && row0 + tid < n && ((amask >> tid) & 1u)) {  // (max, log sum exp(x - max)) of the row
            float2 q[NW];
            float m = -INFINITY, sm = 0.f;
#pragma unroll
            for (int w = 0; w < NW; w++) {
                q[w] = SS[w * ROWS + tid];
                m = fmaxf(m, q[w].x);
            }
#pragma unroll
            for (int w = 0; w < NW; w++) sm += q[w].x == -INFINITY ? 0.f : q[w].y * __expf(q[w].x - m);
            mlse[(long)part * mstride + row0 + tid] = make_float2(m, parts > 1 ? sm : logf(sm));
        }
    }
    // the last statement: a branch around a global atomic earlier would merge the wait counters of
    // its paths at the join and drain the policy ring's loads in flight (section 8-)
#if FWD_SYNC_MODE == 1 || FWD_SYNC_MODE == 3
    if (wave < 4 && lane == 0 && SYNC_LOST && net.err) atomicOr(net.err, FWD_ERR_SYNC);
#endif
}

}  // namespace
}  // namespace ykf
