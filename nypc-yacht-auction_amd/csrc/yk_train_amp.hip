// yk_train_amp.hip - NNetWrapper.train's mixed-precision step on MI355X: the reference trains on
// the GPU under autocast('cuda') with a GradScaler (yacht/NNet.py:113-116, 141-155): fp16 Linear
// layers (fp16 inputs, weights and outputs, f32 accumulation), LayerNorm / cross-entropy / MSE
// in f32, the loss scaled before backward, the gradients unscaled, clip_grad_norm_(5.0), AdamW,
// and the step skipped (scale halved) when a gradient overflows.  This file restates that
// arithmetic - the fp16 rounding points included - on hand-written v_mfma_f32_16x16x32_f16
// kernels instead of library GEMMs (yk_train.hip keeps the f32 rocBLAS step for the f32 mode).
//
// A step is seven launches (yk_train_amp.h):
//   k_amp_fwd      one 512-thread workgroup per 8 rows (TRV; the MFMAs run 16): features -> input
//                  layer -> the residual blocks -> the heads' LayerNorms, every dense layer from a
//                  register ring of fp16 weight fragments that streams the next layer during the
//                  row pass; saves what the backward needs (fp16 pre-activations, LayerNorm
//                  statistics, the GEMM inputs in the T layout the weight-gradient GEMMs read)
//   k_amp_head     16-row tile x column part: the policy logits (fp16-rounded) and their per-part
//                  softmax statistics; one more part per tile computes v_head.2
//   k_amp_headbwd  16-row tile x action slice: the scaled fp16 logits gradient, its T layout, and a
//                  split-K slice of pi_head.2's input gradient; one more part per tile the loss rows
//                  (a wave per example: cross-entropy, the value head's tail, the MSE, gradients)
//   k_amp_bwd      one workgroup per 8 rows: the heads' LayerNorm backward and the trunk's
//                  backward chain (LayerNorm / SiLU / dropout backward, the dX GEMMs) to the input
//   k_amp_grads    the trunk's weight gradients (13 GEMMs, K = the batch; the heads' 2 run in
//                  k_amp_bwd's launch) and, in more blocks, the bias / LayerNorm gradients and the
//                  loss sums: fixed-order column sums
//   k_amp_sq       unscale + the gradient norm
//   k_amp_update   clip + AdamW (or skip), GradScaler update and the fp16 weight copies for the
//                  next step, a 32 x 32 weight tile (or a vector slice) per workgroup; extra blocks
//                  make the next step's dropout keep bits (k_amp_masks when they could not)
// Weight fragments use yk_net.h's packing (one plane): for W[N][K], the 1 KB piece (nt, ks) holds
// W[16 nt + (l & 15)][32 ks + 8 (l >> 4) + j] for lane l, j < 8.  The T layout of an activation
// matrix X[rows][C] is the same packing of X^T (piece (ct, rs): X[32 rs + 8 (l >> 4) + j][16 ct +
// (l & 15)]), so dW = dU^T X is an MFMA over 32-row slices with both operands read whole.
#include <algorithm>
#include <cmath>
#include <vector>

#include "yk_api.h"
#include "yk_common.h"
#include "yk_train_amp.h"

using namespace yk;

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int TR = 16;          // rows per tile (the MFMA M): the heads' row tiles
constexpr int TRV = 8;          // rows per trunk workgroup (k_amp_fwd / k_amp_bwd): the MFMAs still
                                // run 16 rows, the last 8 of them ignored, so a 512-example step
                                // spreads its row passes (the VALU-bound part of a layer) over 64
                                // CUs instead of 32 (each still streams the whole weight set)
constexpr int TW = 8;           // waves per trunk workgroup
constexpr int TTHR = 64 * TW;
constexpr int TRPW = TRV / TW;  // rows per wave in the row passes
constexpr int LDL = 3264;       // logits row stride: 204 tiles of 16 columns
constexpr int PT = LDL / 16;    // policy column tiles
constexpr int PKS = LDL / 32;   // 32-deep action slices
#ifndef YK_HQ
#define YK_HQ 8
#endif
#ifndef YK_BQ
#define YK_BQ 12
#endif
constexpr int HQ = YK_HQ;       // policy-head column parts per row tile (+1 part: v_head.2)
constexpr int BQ = YK_BQ;       // head-backward action parts per row tile (12: 6 -> 12 took the step
                                // 102.5 -> 99.0 us at batch 64, +-0 at 512; 16 and 24 slower at 512,
                                // profiles/r05ze_head_parts_trainab.log)
constexpr int VH = 128;         // v_head hidden width
constexpr int SQ_BLOCKS = 1024;
#ifndef YK_DW_KG
#define YK_DW_KG 2  // column tiles per trunk dW item
#endif

struct Scaler {  // GradScaler('cuda') state + the AdamW step count (device)
    float scale;
    int tracker;
    int64_t steps;
    int found_inf;
    int growth_interval;
};

// Everything the kernels address: parameters (f32, state_dict order), fp16 weight fragments
// (float4 = 8 halves), saved activations, gradients.
struct AmpDev {
    int H, NB, Bmax, RS, TMAX, NVEC;
    const float* P;
    float* G;
    const long* off;                      // tensor offsets (device)
    const float4 *win_f, *w1f, *w2f, *w1t, *w2t, *wpif, *wpit, *wv1f, *wv1t;
    _Float16 *xT, *hT, *r1T, *apiT, *avT, *api_rm, *av_rm;
    float *z0, *u1, *u2, *hF, *stats;
    float *logits, *zv1;
    float2* mlq;
    uint8_t* masks;                       // [1 + NB][Bmax][H / 4] the step's dropout keep bits (k_amp_masks)
    _Float16 *dz1_rm, *dz1T, *dlT, *dz0T, *du1T, *du2T;
    float *dz1f, *v2prod, *dzv2, *dpart, *dbpi_part, *colpart;
    Scaler* sc;
};
// tensor indices in state_dict order (YachtNNet.py:30-52)
enum { T_WIN = 0, T_BIN, T_GIN, T_BEIN };
__host__ __device__ inline int t_blk(int b, int k) { return 4 + 8 * b + k; }
__host__ __device__ inline int t_head(int NB, int k) { return 4 + 8 * NB + k; }
// offset of tensor k in the flat buffer (closed form of the state_dict sizes: no memory load,
// so nothing the kernels read waits behind the weight ring in the in-order vmcnt queue)
__host__ __device__ inline long poff(int H, int NB, int k) {
    const long h = H, hh = h * h;
    if (k < 4) return k == 0 ? 0 : FEAT * h + (k - 1) * h;
    const long base = (FEAT + 3) * h;
    if (k < 4 + 8 * NB) {
        const int b = (k - 4) / 8, s = (k - 4) % 8;
        const long o = base + b * (2 * hh + 6 * h);
        const long so[8] = {0, hh, hh + h, hh + 2 * h, hh + 3 * h, 2 * hh + 3 * h, 2 * hh + 4 * h, 2 * hh + 5 * h};
        return o + so[s];
    }
    const int s = k - 4 - 8 * NB;
    const long o = base + NB * (2 * hh + 6 * h), A = ASIZE;
    const long so[10] = {0, h, 2 * h, 2 * h + A * h, 2 * h + A * h + A, 3 * h + A * h + A, 4 * h + A * h + A,
                         4 * h + A * h + A + 128 * h, 4 * h + A * h + A + 128 * h + 128,
                         4 * h + A * h + A + 128 * h + 256};
    return o + so[s];
}
enum { HP_G = 0, HP_B = 1, HP_W = 2, HP_BIAS = 3, HV_G = 4, HV_B = 5, HV_W1 = 6, HV_B1 = 7, HV_W2 = 8, HV_B2 = 9 };
// column-partial vectors of k_amp_bwd (colpart[tile][v][H])
enum { CV_BIN = 0, CV_GIN, CV_BEIN, CV_GPI, CV_BEPI, CV_GV, CV_BEV, CV_BLK };  // + 6 b + {b1 g1 be1 b2 g2 be2}

__device__ __forceinline__ float r16(float x) { return (float)(_Float16)x; }  // an fp16 tensor's value
__device__ __forceinline__ floatx4 mfma(float4 a, float4 b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, a), __builtin_bit_cast(half8, b), c, 0, 0, 0);
}
__device__ __forceinline__ floatx4 zero4() { return floatx4{0.f, 0.f, 0.f, 0.f}; }
// Accesses through pointers read from job tables compile to flat_load / flat_store, which count in
// lgkmcnt too (so every LDS / scalar wait also drains them); these go through the global address space
typedef float f4v_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 gld4(const float4* p) {
    return __builtin_bit_cast(float4, *(const __attribute__((address_space(1))) f4v_t*)p);
}
typedef __attribute__((address_space(1))) float gfloat_t;
__device__ __forceinline__ gfloat_t* gptr(float* p) { return (gfloat_t*)p; }
__device__ __forceinline__ void gst4(float* p, float4 v) {
    *(__attribute__((address_space(1))) f4v_t*)p = __builtin_bit_cast(f4v_t, v);
}
__device__ __forceinline__ void gsth8(float4* p, half8 v) { *(__attribute__((address_space(1))) half8*)p = v; }
__device__ __forceinline__ float wsum(float v) { return xlane_sum(v); }
// two full-wave sums at once on the DPP path (quad / row shuffles, row broadcasts, lane 63 read):
// the row passes' reductions, whose latency is on every layer's critical path
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROW_MASK, 0xF, false));
}
__device__ __forceinline__ void wsum2(float& a, float& b) {
    a += dpp<0xB1, 0xF>(a);   b += dpp<0xB1, 0xF>(b);    // quad_perm [1,0,3,2]
    a += dpp<0x4E, 0xF>(a);   b += dpp<0x4E, 0xF>(b);    // quad_perm [2,3,0,1]
    a += dpp<0x141, 0xF>(a);  b += dpp<0x141, 0xF>(b);   // row_half_mirror
    a += dpp<0x140, 0xF>(a);  b += dpp<0x140, 0xF>(b);   // row_mirror: 16-lane row sums
    a += dpp<0x142, 0xA>(a);  b += dpp<0x142, 0xA>(b);   // row_bcast15
    a += dpp<0x143, 0xC>(a);  b += dpp<0x143, 0xC>(b);   // row_bcast31
    a = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, a), 63));
    b = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, b), 63));
}
// the logistic as the inference forward computes it (yk_fwd.h silu): the native exp and reciprocal.
// Autocast rounds SiLU's result to fp16 (or feeds it to an fp16 Linear), so their ~1e-6 relative
// error moves only the rare value that sits within it of an fp16 rounding boundary; the library
// expf + IEEE division cost 15 us of a 192 us step (k_amp_fwd 59.8 -> 51.3 us, k_amp_bwd 64.5 -> 58.7)
__device__ __forceinline__ float sigm(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
__device__ __forceinline__ float silu(float x) { return x * sigm(x); }
__device__ __forceinline__ float silu_grad(float x) {
    const float s = sigm(x);
    return s * (1.0f + x * (1.0f - s));
}
// workgroup barrier that does not drain the weight ring's outstanding loads (vmcnt)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ void stat_merge(float& m, float& s, float m2, float s2) {
    const float mm = fmaxf(m, m2);
    if (mm == -INFINITY) return;
    s = s * __expf(m - mm) + s2 * __expf(m2 - mm);
    m = mm;
}

// The tile's R rows (R = 8 or 16) of an fp16 plane (LDS, row stride sa halves; columns col0 ..
// col0 + C) into the T layout at column tile offset ct0: a 32-row slice holds 32 / R tiles, lane
// group q = lane >> 4 rows 8 q .. 8 q + 7 of it.  The batch's last tile (zero_rest) also zeroes
// the rest of its slice (rows past the batch must not enter a weight gradient).
// nthr > 0: only threads 0 .. nthr-1 (whole waves) take part (default: the whole workgroup)
template <int R>
__device__ __forceinline__ void write_tl(const _Float16* A, int sa, int col0, int C, _Float16* dst, int RS, int ct0,
                                         int tile, bool zero_rest, int nthr = 0) {
    constexpr int QPT = R / 8, TPS = 32 / R;  // lane groups per tile, tiles per slice
    const int nt = nthr > 0 ? nthr : (int)blockDim.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = nt >> 6;
    const int h = tile % TPS, rs = tile / TPS, q = lane >> 4;
    const bool mine = q / QPT == h, after = q / QPT > h;
    if constexpr (R == 8) {  // one 8-row piece per column: every thread takes half of one (4 rows, 8 bytes)
        for (int i = threadIdx.x; i < C * 2; i += nt) {
            const int cc = i >> 1, hf = i & 1, ct = cc >> 4, cl = cc & 15;
            half4 v;
#pragma unroll
            for (int j = 0; j < 4; j++) v[j] = A[(4 * hf + j) * sa + col0 + cc];
            *reinterpret_cast<half4*>(dst + (((long)(ct0 + ct) * RS + rs) * 64 + cl + 16 * h) * 8 + 4 * hf) = v;
        }
        if (!zero_rest) return;  // the batch's last tile: the slice's later pieces are zeros
        for (int ct = wave; ct < C / 16; ct += nw)
            if (after) *reinterpret_cast<half8*>(dst + (((long)(ct0 + ct) * RS + rs) * 64 + lane) * 8) = half8{};
        return;
    }
    for (int ct = wave; ct < C / 16; ct += nw) {
        half8 v = {};
        if (mine) {
#pragma unroll
            for (int j = 0; j < 8; j++) v[j] = A[(8 * (q - QPT * h) + j) * sa + col0 + 16 * ct + (lane & 15)];
        }
        if (mine || (zero_rest && after))
            *reinterpret_cast<half8*>(dst + (((long)(ct0 + ct) * RS + rs) * 64 + lane) * 8) = v;
    }
}

// acc[t] = A[16 x K] (fp16 plane in LDS) x W^T over this wave's NT column tiles, weights from the
// register ring (slice ks in slot ks % RW); a consumed slot is refilled with slice ks + RW of
// this matrix (cur) or, past its end, of the next one (nxt, same shape; none if null).
// DEF > 0: the last DEF slots' next-matrix refills are left to the caller (ring_part during the row
// pass that follows, where the CU's vector-memory path is otherwise idle; yk_fwd.h mma_ring)
template <int KS, int NT, int RW, int DEF = 0>
__device__ __forceinline__ void gemm_ring(const _Float16* A, int sa, float4 (&ring)[RW][NT], floatx4 (&acc)[NT],
                                          const float4* __restrict__ cur, const float4* __restrict__ nxt, int nt0) {
    static_assert(KS % RW == 0, "ring slots align with layers");
    static_assert(0 <= DEF && DEF <= KS - RW + DEF && (DEF == 0 || RW == KS), "deferred refills within a one-matrix ring");
    const int lane = threadIdx.x & 63;
    const _Float16* ap = A + (lane & 15) * sa + 8 * (lane >> 4);
#pragma unroll
    for (int t = 0; t < NT; t++) acc[t] = zero4();
    float4 a = *reinterpret_cast<const float4*>(ap);
#pragma unroll
    for (int ks = 0; ks < KS; ks++) {
        const float4 an = *reinterpret_cast<const float4*>(ap + 32 * ((ks + 1) % KS));
        float4(&w)[NT] = ring[ks % RW];
#pragma unroll
        for (int t = 0; t < NT; t++) acc[t] = mfma(a, w[t], acc[t]);
        const int g = ks + RW;
        if (g < KS) {
#pragma unroll
            for (int t = 0; t < NT; t++) w[t] = cur[((long)(nt0 + t) * KS + g) * 64 + lane];
        } else if (ks < KS - DEF) {  // the next layer's slices; after the last layer `cur` again (unused):
                  // the refills stay unconditional, so the wait counters after this loop are exact (no vmcnt(0) drains)
            const float4* src = nxt ? nxt : cur;
#pragma unroll
            for (int t = 0; t < NT; t++) w[t] = src[((long)(nt0 + t) * KS + g - KS) * 64 + lane];
        }
        __builtin_amdgcn_sched_barrier(0);
        a = an;
    }
}
// slots S0 .. S1-1 refilled with the same slices of the next matrix (gemm_ring's deferred refills;
// RW == KS, so slot s holds slice s of every matrix)
template <int KS, int NT, int RW, int S0, int S1>
__device__ __forceinline__ void ring_part(float4 (&ring)[RW][NT], const float4* __restrict__ W, int nt0) {
    static_assert(RW == KS || S0 == S1, "deferred refills need a one-matrix ring");
    static_assert(0 <= S0 && S0 <= S1 && S1 <= RW, "slots within the ring");
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int s = S0; s < S1; s++)
#pragma unroll
        for (int t = 0; t < NT; t++) ring[s][t] = W[((long)(nt0 + t) * KS + s) * 64 + lane];
    __builtin_amdgcn_sched_barrier(0);
}
template <int KS, int NT, int RW>
__device__ __forceinline__ void ring_fill(float4 (&ring)[RW][NT], const float4* __restrict__ W, int nt0) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int s = 0; s < RW; s++)
#pragma unroll
        for (int t = 0; t < NT; t++) ring[s][t] = W[((long)(nt0 + t) * KS + s) * 64 + lane];
}
// accumulator tile t -> T[row][col] (+ bias16, fp16-rounded when `round`); lane holds rows
// 4 (l >> 4) + j of column 16 (nt0 + t) + (l & 15)
template <int NT>
__device__ __forceinline__ void store_acc(float* T, int ld, int nt0, const floatx4 (&acc)[NT]) {
    const int lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
#pragma unroll
    for (int t = 0; t < NT; t++)
#pragma unroll
        for (int j = 0; j < 4; j++) T[(4 * q + j) * ld + 16 * (nt0 + t) + r] = acc[t][j];
}
// LayerNorm statistics (biased variance, eps 1e-5) of a row held VPL per lane: one pass of sums
// shifted by the row's first value (so E[(x-k)^2] - E[x-k]^2 does not cancel), one reduction
template <int VPL>
__device__ __forceinline__ void ln_stats(const float (&x)[VPL], int H, float& mu, float& rs) {
    const float k = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, x[0])));
    float s = 0.f, q = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; i++) {
        const float d = x[i] - k;
        s += d;
        q += d * d;
    }
    wsum2(s, q);
    const float m = s / (float)H;
    mu = k + m;
    rs = 1.0f / sqrtf(fmaxf(q / (float)H - m * m, 0.f) + 1e-5f);
}
// LayerNorm input gradient from dL/dxhat (dx, in place): rs / H (H dx - sum dx - xhat sum(dx xhat))
template <int VPL>
__device__ __forceinline__ void ln_bwd(const float (&xh)[VPL], float (&dx)[VPL], int H, float rs) {
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; i++) {
        a += dx[i];
        b += dx[i] * xh[i];
    }
    wsum2(a, b);
#pragma unroll
    for (int i = 0; i < VPL; i++) dx[i] = rs / (float)H * ((float)H * dx[i] - a - xh[i] * b);
}
__device__ __forceinline__ float* stat_ptr(const AmpDev& d, int layer, int which) {
    return d.stats + ((long)layer * 2 + which) * d.Bmax;
}
// the keep bits of the lane's VPL elements c0 .. c0 + VPL - 1 (bit i: element c0 + i) of dropout
// layer L (0: inp, 1 + b: block b's fc1) in row `row`, from the bytes k_amp_masks wrote (4 bits each)
template <int VPL>
__device__ __forceinline__ uint32_t mask_bits(const AmpDev& d, int L, int row, int c0) {
    const int H = VPL * 64;
    const uint8_t* m = d.masks + ((long)L * d.Bmax + row) * (H / 4) + (c0 >> 2);
    if constexpr (VPL == 8) {
        const uint32_t w = *reinterpret_cast<const uint16_t*>(m);
        return (w & 15u) | ((w >> 4) & 0xF0u);
    } else if constexpr (VPL == 4) {
        return *m;
    } else {
        return ((uint32_t)*m >> (c0 & 3)) & ((1u << VPL) - 1u);
    }
}
// per-wave column partials of up to 3 vectors (LDS CP[TW][3][H]) summed over the waves in wave
// order into colpart[tile][v0 + k][H]
template <int H>
__device__ __forceinline__ void colpart_flush(const AmpDev& d, const float* CP, int tile, int v0, int nv) {
    for (int i = threadIdx.x; i < nv * H; i += TTHR) {
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < TW; w++) s += CP[w * 3 * H + i];
        d.colpart[((long)tile * d.NVEC + v0) * H + i] = s;
    }
}

// The step's dropout keep bits (the draws dropout_keep makes, yk_common.h) for every dropout layer,
// generated across the whole chip before the forward: the 32 row tiles of k_amp_fwd / k_amp_bwd then
// read 4 bits per byte instead of each running the Philox rounds in its row passes (~2K ticks per
// dropout layer and tile, on 32 CUs).  One thread per byte: layer, row, 4-element group.
__global__ __launch_bounds__(256) void k_amp_masks(AmpDev d, int B, float p, uint64_t seed, uint64_t step,
                                                   int64_t row_base) {
    const int q4 = d.H / 4;
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= (long)(1 + d.NB) * B * q4) return;
    const int q = (int)(i % q4), row = (int)((i / q4) % B), L = (int)(i / ((long)q4 * B));
    d.masks[((long)L * d.Bmax + row) * q4 + q] =
        (uint8_t)dropout_bits(seed, L, step, (row_base + row) * q4 + q, p);
}

// ------------------------------------------------------------------ forward (trunk)
template <int H>
__global__ __launch_bounds__(TTHR) void k_amp_fwd(AmpDev d, const yk_state_t* __restrict__ states,
                                                  const int32_t* __restrict__ idx, int B, float p, uint64_t seed,
                                                  uint64_t step, int64_t row_base) {
    constexpr int LD = H + 4, SA = H + 8, VPL = H / 64, KS = H / 32;
    constexpr int NT = H >= 128 ? H / 128 : 1, NACT = H / (16 * NT);
    constexpr int RW = KS * NT <= 16 ? KS : 16 / NT;
    // each trunk GEMM's last FDEF ring slots are refilled in the row pass that follows (gemm_ring): the
    // refills stall a wave while every wave's loads share the CU's vector-memory path, which is idle
    // during the row passes.  AMP step 122.6 -> 115.3 us with 6 in both kernels (4: 116.0, 8: 116.5;
    // profiles/r05m_amp_defer_*trainab.log)
    // (hidden >= 256 only: at KS < 8 a GEMM has too few slices to leave 6 to the row pass)
    constexpr int FDEF = (RW == KS && KS >= 8) ? 6 : 0;
    __shared__ __attribute__((aligned(16))) float Xs[TR * LD];
    __shared__ __attribute__((aligned(16))) float Ts[TR * LD];
    __shared__ __attribute__((aligned(16))) _Float16 Pa[TR * SA];
    __shared__ __attribute__((aligned(16))) float VL[(3 * H + TTHR - 1) / TTHR * TTHR];  // (padded: unconditional writes)
    const int tile = blockIdx.x, row0 = tile * TRV;
    const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    // every wave owns columns when NACT == TW (hidden >= 128): a compile-time true, so no branch
    // around the weight ring (at a branch join the wait counters merge to the stricter count, and
    // a vmcnt(0) there would drain the ring's in-flight refills)
    const bool gw = NACT == TW || wave < NACT;
    const int nt0 = wave * NT, c0 = lane * VPL;
    const bool zero_rest = row0 + TRV >= B;
    const float sc = p > 0.f ? 1.0f / (1.0f - p) : 1.0f;
    const int NB = d.NB;
    const long HH8 = (long)H * H / 8;  // float4 per packed H x H matrix
    const bool drop = p > 0.f;  // the keep bits: k_amp_masks

    // the input layer's vectors, its weights (K = 64: 2 slices), the first block's ring, then features
    for (int i = tid; i < 3 * H; i += TTHR) VL[i] = d.P[poff(H, d.NB, T_BIN + i / H) + i % H];
    uint32_t mk[TRPW];  // the current dropout layer's keep bits of the wave's rows
#pragma unroll
    for (int rr = 0; rr < TRPW; rr++) {
        const int row = row0 + wave * TRPW + rr;
        mk[rr] = drop ? mask_bits<VPL>(d, 0, row < B ? row : 0, c0) : 0xFFu;
    }
    float4 w0[2][NT];
    if (gw) {
#pragma unroll
        for (int s = 0; s < 2; s++)
#pragma unroll
            for (int t = 0; t < NT; t++) w0[s][t] = d.win_f[((long)(nt0 + t) * 2 + s) * 64 + lane];
    }
    // the heads' LayerNorm affines, needed after the trunk: loaded now, ahead of the weight stream
    float hg[4][VPL];
#pragma unroll
    for (int v = 0; v < 4; v++)
#pragma unroll
        for (int i = 0; i < VPL; i++) hg[v][i] = d.P[poff(H, d.NB, t_head(NB, v == 0 ? HP_G : v == 1 ? HP_B : v == 2 ? HV_G : HV_B)) + c0 + i];
    float4 ring[RW][NT];
    // the first block's ring (whatever NB is: no branch join), in four parts between the prologue's
    // phases when RW == KS (a wave issuing all of them at once stalls on the CU's vector-memory path
    // while the other waves' loads move; yk_fwd.h's prologue does the same)
    const float4* wfirst = NB > 0 ? d.w1f : d.wpif;
    constexpr bool PARTS = RW == KS && KS % 4 == 0;
    if (gw) {
        if constexpr (PARTS) ring_part<KS, NT, RW, 0, KS / 4>(ring, wfirst, nt0);
        else ring_fill<KS, NT, RW>(ring, wfirst, nt0);
    }
#pragma unroll
    for (int k = 0; k < 2; k++) {  // state_to_vec (NNet.py:65-86), K padded to 64 (rows past TRV: zeros)
        const int r = wave + TW * k, row = row0 + r;
        float x = 0.f;
        if (row < B && r < TRV) {
            const int src = __builtin_amdgcn_readfirstlane(idx ? idx[row] : row);
            YkS s;
            const uint64_t* q = reinterpret_cast<const uint64_t*>(states + src);
#pragma unroll
            for (int w = 0; w < 8; w++) s.w[w] = q[w];
            if (lane < FEAT) x = feature(s, lane);
        }
        Pa[r * SA + lane] = (_Float16)x;
    }
    if constexpr (PARTS) if (gw) ring_part<KS, NT, RW, KS / 4, KS / 2>(ring, wfirst, nt0);
    lds_barrier();
    write_tl<TRV>(Pa, SA, 0, 64, d.xT, d.RS, 0, tile, zero_rest);
    floatx4 acc[NT];
    if (gw) {  // inp.0: Z0 = fp16(x16 W_in^T + b16)
        const _Float16* ap = Pa + (lane & 15) * SA + 8 * (lane >> 4);
#pragma unroll
        for (int t = 0; t < NT; t++) acc[t] = zero4();
#pragma unroll
        for (int s = 0; s < 2; s++) {
            const float4 a = *reinterpret_cast<const float4*>(ap + 32 * s);
#pragma unroll
            for (int t = 0; t < NT; t++) acc[t] = mfma(a, w0[s][t], acc[t]);
        }
        store_acc<NT>(Ts, LD, nt0, acc);
    }
    if constexpr (PARTS) if (gw) ring_part<KS, NT, RW, KS / 2, 3 * KS / 4>(ring, wfirst, nt0);
    lds_barrier();
    // inp.1-3: LayerNorm (f32) -> SiLU -> Dropout  YachtNNet.py:30-35
#pragma unroll
    for (int rr = 0; rr < TRPW; rr++) {
        const int r = wave * TRPW + rr, row = row0 + r;
        float x[VPL];
        if (row < B) {
#pragma unroll
            for (int i = 0; i < VPL; i++) {
                x[i] = r16(Ts[r * LD + c0 + i] + r16(VL[c0 + i]));
                d.z0[(long)row * H + c0 + i] = x[i];
            }
            float mu, rs;
            ln_stats<VPL>(x, H, mu, rs);
            if (lane == 0) {
                stat_ptr(d, 0, 0)[row] = mu;
                stat_ptr(d, 0, 1)[row] = rs;
            }
#pragma unroll
            for (int i = 0; i < VPL; i++) {
                const float a = (x[i] - mu) * rs * VL[H + c0 + i] + VL[2 * H + c0 + i];
                const bool k = (mk[rr] >> i) & 1u;
                x[i] = k ? silu(a) * sc : 0.f;
            }
        } else {
#pragma unroll
            for (int i = 0; i < VPL; i++) x[i] = 0.f;
        }
#pragma unroll
        for (int i = 0; i < VPL; i++) {
            Xs[r * LD + c0 + i] = x[i];
            Pa[r * SA + c0 + i] = (_Float16)x[i];
        }
    }
    if constexpr (PARTS) if (gw) ring_part<KS, NT, RW, 3 * KS / 4, KS>(ring, wfirst, nt0);
    lds_barrier();
    // (block 0's input h in the T layout: written by waves 0-3 beside its first GEMM, below)

    // ResidualBlock x NB: h = LN1(SiLU(fc1 x)); h = Dropout(h); h = LN2(SiLU(fc2 h)); x + h  YachtNNet.py:8-21
    for (int b = 0; b < NB; b++) {
        for (int half = 0; half < 2; half++) {
            const int kb = half == 0 ? 1 : 5;  // fc1.bias / fc2.bias
            float vr[(3 * H + TTHR - 1) / TTHR];  // this layer's bias, gamma, beta (issued before the
#pragma unroll                               // ring's refills, so the LDS copy never waits behind them)
            for (int k = 0; k < (3 * H + TTHR - 1) / TTHR; k++) {
                const int i = tid + TTHR * k;
                const int ic = i < 3 * H ? i : 3 * H - 1;  // unconditional: no branch join before the ring
                vr[k] = d.P[poff(H, d.NB, t_blk(b, kb + ic / H)) + ic % H];
            }
            if (half == 0) {  // block b's fc1 dropout bits, with the vectors (ahead of the ring's refills)
#pragma unroll
                for (int rr = 0; rr < TRPW; rr++) {
                    const int row = row0 + wave * TRPW + rr;
                    mk[rr] = drop ? mask_bits<VPL>(d, 1 + b, row < B ? row : 0, c0) : 0xFFu;
                }
            }
            const float4* cur = (half == 0 ? d.w1f : d.w2f) + b * HH8;
            const float4* nxt = half == 0 ? d.w2f + b * HH8 : (b + 1 < NB ? d.w1f + (b + 1) * HH8 : nullptr);
            const float4* dsrc = nxt ? nxt : cur;  // the deferred refills' matrix (as gemm_ring's)
            if (gw) {
                gemm_ring<KS, NT, RW, FDEF>(Pa, SA, ring, acc, cur, nxt, nt0);
                store_acc<NT>(Ts, LD, nt0, acc);
            }
            // this GEMM's input (h_b or r1_b) in the T layout for the weight gradients, by waves 0-3,
            // which reach the barrier below before the younger waves (their weights arrive first);
            // the row pass after it overwrites Pa
            if (wave < 4)
                write_tl<TRV>(Pa, SA, 0, H, (half == 0 ? d.hT : d.r1T) + (long)b * (H / 16) * d.RS * 512, d.RS, 0, tile,
                              zero_rest, 256);
#pragma unroll
            for (int k = 0; k < (3 * H + TTHR - 1) / TTHR; k++) VL[tid + TTHR * k] = vr[k];
            lds_barrier();
            float* U = (half == 0 ? d.u1 : d.u2) + (long)b * d.Bmax * H;
            const int L = 1 + 2 * b + half;
            // the GEMM's deferred refills, half before the row pass and half after it (unconditional:
            // every row of the tile reads the next GEMM's weights)
            if constexpr (FDEF > 0) if (gw) ring_part<KS, NT, RW, KS - FDEF, KS - FDEF / 2>(ring, dsrc, nt0);
#pragma unroll
            for (int rr = 0; rr < TRPW; rr++) {
                const int r = wave * TRPW + rr, row = row0 + r;
                float x[VPL];
                if (row < B) {
                    float s[VPL];
#pragma unroll
                    for (int i = 0; i < VPL; i++) {
                        const float u = r16(Ts[r * LD + c0 + i] + r16(VL[c0 + i]));  // fc out (fp16)
                        U[(long)row * H + c0 + i] = u;
                        s[i] = r16(silu(u));                                          // SiLU on fp16
                    }
                    float mu, rs;
                    ln_stats<VPL>(s, H, mu, rs);
                    if (lane == 0) {
                        stat_ptr(d, L, 0)[row] = mu;
                        stat_ptr(d, L, 1)[row] = rs;
                    }
#pragma unroll
                    for (int i = 0; i < VPL; i++) {
                        const float l = (s[i] - mu) * rs * VL[H + c0 + i] + VL[2 * H + c0 + i];
                        if (half == 0) {
                            const bool k = (mk[rr] >> i) & 1u;
                            x[i] = k ? l * sc : 0.f;
                        } else {
                            x[i] = Xs[r * LD + c0 + i] + l;  // residual (f32)
                        }
                    }
                } else {
#pragma unroll
                    for (int i = 0; i < VPL; i++) x[i] = 0.f;
                }
#pragma unroll
                for (int i = 0; i < VPL; i++) {
                    if (half == 1) Xs[r * LD + c0 + i] = x[i];
                    Pa[r * SA + c0 + i] = (_Float16)x[i];
                }
            }
            if constexpr (FDEF > 0) if (gw) ring_part<KS, NT, RW, KS - FDEF / 2, KS>(ring, dsrc, nt0);
            lds_barrier();
        }
    }

    // the heads' LayerNorms (one set of statistics, two affine maps) -> SiLU: a_pi, a_v (f32),
    // cast to fp16 for pi_head.2 / v_head.2  YachtNNet.py:40-52
    _Float16* Pv = reinterpret_cast<_Float16*>(Ts);
    lds_barrier();  // every wave is done reading Ts
#pragma unroll
    for (int rr = 0; rr < TRPW; rr++) {
        const int r = wave * TRPW + rr, row = row0 + r;
        float x[VPL];
#pragma unroll
        for (int i = 0; i < VPL; i++) x[i] = Xs[r * LD + c0 + i];
        if (row < B) {
            float mu, rs;
            ln_stats<VPL>(x, H, mu, rs);
            if (lane == 0) {
                stat_ptr(d, 1 + 2 * NB, 0)[row] = mu;
                stat_ptr(d, 1 + 2 * NB, 1)[row] = rs;
            }
#pragma unroll
            for (int i = 0; i < VPL; i++) {
                d.hF[(long)row * H + c0 + i] = x[i];
                const float xh = (x[i] - mu) * rs;
                Pa[r * SA + c0 + i] = (_Float16)silu(xh * hg[0][i] + hg[1][i]);
                Pv[r * SA + c0 + i] = (_Float16)silu(xh * hg[2][i] + hg[3][i]);
            }
        } else {
#pragma unroll
            for (int i = 0; i < VPL; i++) {
                Pa[r * SA + c0 + i] = (_Float16)0.f;
                Pv[r * SA + c0 + i] = (_Float16)0.f;
            }
        }
    }
    lds_barrier();
    write_tl<TRV>(Pa, SA, 0, H, d.apiT, d.RS, 0, tile, zero_rest);
    write_tl<TRV>(Pv, SA, 0, H, d.avT, d.RS, 0, tile, zero_rest);
    for (int i = tid; i < TRV * H / 8; i += TTHR) {  // row-major copies: the head kernel's A operands
        const int r = i / (H / 8), c8 = i % (H / 8), row = row0 + r;
        if (row < B) {
            reinterpret_cast<float4*>(d.api_rm + (long)row * H)[c8] = *reinterpret_cast<const float4*>(Pa + r * SA + 8 * c8);
            reinterpret_cast<float4*>(d.av_rm + (long)row * H)[c8] = *reinterpret_cast<const float4*>(Pv + r * SA + 8 * c8);
        }
    }
}

// ------------------------------------------------------------------ heads
// policy logits = fp16(a_pi16 Wpi16^T + bpi16) over this part's column tiles, and per row the
// part's (max, sum exp); part HQ: v_head.2 z1 = fp16(a_v16 Wv1^T + bv1_16)
template <int H>
__global__ __launch_bounds__(TTHR) void k_amp_head(AmpDev d, int B) {
    constexpr int SA = H + 8, KS = H / 32;
    __shared__ __attribute__((aligned(16))) _Float16 A[TR * SA];
    __shared__ float2 red[TW][TR];
    const int tile = blockIdx.x, part = blockIdx.y, row0 = tile * TR;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, q = lane >> 4;
    const bool vpart = part == HQ;
    const _Float16* src = vpart ? d.av_rm : d.api_rm;
    for (int i = tid; i < TR * H / 8; i += TTHR) {
        const int r = i / (H / 8), c8 = i % (H / 8);
        const float4 v = row0 + r < B ? reinterpret_cast<const float4*>(src + (long)(row0 + r) * H)[c8]
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
        *reinterpret_cast<float4*>(A + r * SA + 8 * c8) = v;
    }
    __syncthreads();
    const _Float16* ap = A + (lane & 15) * SA + 8 * (lane >> 4);
    if (vpart) {  // 8 tiles of 16 columns, one per wave
        const int nt = wave;
        floatx4 acc = zero4();
#pragma unroll
        for (int ks = 0; ks < KS; ks++)
            acc = mfma(*reinterpret_cast<const float4*>(ap + 32 * ks), d.wv1f[((long)nt * KS + ks) * 64 + lane], acc);
        const int col = 16 * nt + (lane & 15);
        const float bias = r16(d.P[poff(H, d.NB, t_head(d.NB, HV_B1)) + col]);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int row = row0 + 4 * q + j;
            if (row < B) d.zv1[(long)row * VH + col] = r16(acc[j] + bias);
        }
        return;
    }
    const int t0 = part * PT / HQ, t1 = (part + 1) * PT / HQ;
    const float* bpi = d.P + poff(H, d.NB, t_head(d.NB, HP_BIAS));
    float m[4], s[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        m[j] = -INFINITY;
        s[j] = 0.f;
    }
    // a tile's bias is loaded with its weight slices (ahead of them: the in-order wait counter
    // would otherwise make the bias wait drain the next tile's slices in flight)
    auto load = [&](float4(&w)[KS], float& bias, int n) {
        bias = bpi[min(16 * n + (lane & 15), ASIZE - 1)];
#pragma unroll
        for (int ks = 0; ks < KS; ks++) w[ks] = d.wpif[((long)n * KS + ks) * 64 + lane];
    };
    auto do_tile = [&](const float4(&w)[KS], float bias_raw, int n) {
        floatx4 acc = zero4();
#pragma unroll
        for (int ks = 0; ks < KS; ks++) acc = mfma(*reinterpret_cast<const float4*>(ap + 32 * ks), w[ks], acc);
        const int col = 16 * n + (lane & 15);
        if (col < ASIZE) {
            const float bias = r16(bias_raw);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int row = row0 + 4 * q + j;
                const float x = r16(acc[j] + bias);
                if (row < B) d.logits[(long)row * LDL + col] = x;
                if (x > m[j]) {
                    s[j] = s[j] * __expf(m[j] - x) + 1.0f;
                    m[j] = x;
                } else {
                    s[j] += __expf(x - m[j]);
                }
            }
        }
    };
    float4 wa[KS], wb[KS];  // two tiles' slices: the wave's next tile streams in under this one
    float ba = 0.f, bb = 0.f;
    int nt = t0 + wave;
    if (nt < t1) load(wa, ba, nt);
    for (; nt < t1; nt += 2 * TW) {
        const int n2 = nt + TW;
        if (n2 < t1) load(wb, bb, n2);
        do_tile(wa, ba, nt);
        if (n2 >= t1) break;
        if (n2 + TW < t1) load(wa, ba, n2 + TW);
        do_tile(wb, bb, n2);
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
        stat_merge(m[j], s[j], xlane<1>(m[j]), xlane<1>(s[j]));
        stat_merge(m[j], s[j], xlane<2>(m[j]), xlane<2>(s[j]));
        stat_merge(m[j], s[j], xlane<4>(m[j]), xlane<4>(s[j]));
        stat_merge(m[j], s[j], xlane<8>(m[j]), xlane<8>(s[j]));
    }
    if ((lane & 15) == 0) {
#pragma unroll
        for (int j = 0; j < 4; j++) red[wave][4 * q + j] = make_float2(m[j], s[j]);
    }
    __syncthreads();
    if (tid < TR && row0 + tid < B) {
        float mm = -INFINITY, ss = 0.f;
#pragma unroll
        for (int w2 = 0; w2 < TW; w2++) stat_merge(mm, ss, red[w2][tid].x, red[w2][tid].y);
        d.mlq[(long)part * d.Bmax + row0 + tid] = make_float2(mm, ss);
    }
}

// one wave per example: CE (f32, NNet.py:145-146), the value head's tail in fp16 (SiLU ->
// Linear(128, 1) -> tanh), MSE (f32), and the scaled gradients of both: d v_head.2 output (dz1,
// fp16) and the rows whose column sums are v_head.4's gradients.  Rows past the batch (up to the
// last 32-row slice) only zero their dz1 T-layout entries.
// The row's log-sum-exp from the head parts' (max, sum exp), merged in part order
__device__ __forceinline__ float row_lse(const AmpDev& d, int row) {
    float m = -INFINITY, s = 0.f;
    for (int qq = 0; qq < HQ; qq++) {
        const float2 ms = d.mlq[(long)qq * d.Bmax + row];
        stat_merge(m, s, ms.x, ms.y);
    }
    return m + logf(s);
}
// One example's losses (one wave): cross-entropy from the row's log-sum-exp; the fp16 value-head
// tail (SiLU, Linear(128, 1), tanh), the MSE and their backward into dz1 / v_head.4's product
// terms; rows past the batch (up to the 32-row slice) zero their dz1 T-layout entries.
__device__ __forceinline__ void loss_row(const AmpDev& d, const int32_t* __restrict__ tgt_all,
                                         const float* __restrict__ v_all, const int32_t* __restrict__ idx, int B,
                                         float vw, float2* __restrict__ lrow, int row, int lane) {
    if (row >= d.RS * 32) return;
    if (row >= B) {
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const int c = 2 * lane + k;
            const int ct = c >> 4, rs = row >> 5, l = (c & 15) + 16 * ((row & 31) >> 3);
            d.dz1T[(((long)ct * d.RS + rs) * 64 + l) * 8 + (row & 7)] = (_Float16)0.f;
        }
        return;
    }
    const float S = d.sc->scale, invB = 1.0f / (float)B;
    const int src = idx ? idx[row] : row;
    const int t = tgt_all[src];
    const float z = v_all[src];
    const float lse = row_lse(d, row);
    const float ce = lse - d.logits[(long)row * LDL + t];
    const float* wv2 = d.P + poff(d.H, d.NB, t_head(d.NB, HV_W2));
    const float bv2 = r16(d.P[poff(d.H, d.NB, t_head(d.NB, HV_B2))]);
    float z1[2], s16[2], w2[2];
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const int c = 2 * lane + k;
        z1[k] = d.zv1[(long)row * VH + c];
        s16[k] = r16(silu(z1[k]));  // v_head.3 SiLU on fp16
        w2[k] = r16(wv2[c]);
        acc += s16[k] * w2[k];
    }
    const float z2 = r16(wsum(acc) + bv2);  // v_head.4 (fp16 out)
    const float v = r16(tanhf(z2));         // tanh on fp16
    const float e = v - z;
    const float dv = r16(S * vw * 2.0f * e * invB);  // MSE backward (f32) -> fp16 grad of v
    const float dz2 = r16(dv * (1.0f - v * v));      // tanh backward (fp16)
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const int c = 2 * lane + k;
        d.v2prod[(long)row * VH + c] = dz2 * s16[k];
        const float ds = r16(dz2 * w2[k]);
        const float dz1 = r16(ds * silu_grad(z1[k]));  // v_head.3 SiLU backward (fp16)
        d.dz1_rm[(long)row * VH + c] = (_Float16)dz1;
        d.dz1f[(long)row * VH + c] = dz1;
        const int ct = c >> 4, rs = row >> 5, l = (c & 15) + 16 * ((row & 31) >> 3);
        d.dz1T[(((long)ct * d.RS + rs) * 64 + l) * 8 + (row & 7)] = (_Float16)dz1;
    }
    if (lane == 0) {
        d.dzv2[row] = dz2;
        lrow[row] = make_float2(ce, e * e);
    }
}

// dlogits = fp16(S (softmax - onehot(t)) / B) for the tile's rows over this part's action slices
// (LDS); their T layout (pi_head.2 weight gradient), their column sums over the 16 rows (bias
// gradient partial), and dA_pi's split-K partial = dlogits16 Wpi16 over these slices.  One more
// part per tile runs its loss rows (loss_row, a wave per row; the last tile the slice's rows past
// it too) beside them - one launch fewer than a separate loss kernel.
template <int H>
__global__ __launch_bounds__(TTHR) void k_amp_headbwd(AmpDev d, const int32_t* __restrict__ tgt_all,
                                                      const float* __restrict__ v_all, const int32_t* __restrict__ idx,
                                                      int B, float vw, float2* __restrict__ lrow) {
    constexpr int NT = H >= 128 ? H / 128 : 1, NACT = H / (16 * NT);
    constexpr int SPMAX = (PKS + BQ - 1) / BQ;
    constexpr int SD = SPMAX * 32 + 8;
    constexpr int RD = 4;  // weight ring depth (slices)
    __shared__ __attribute__((aligned(16))) _Float16 DL[TR * SD];
    __shared__ float LSE[TR];
    __shared__ int TG[TR];
    const int tile = blockIdx.x, part = blockIdx.y, row0 = tile * TR;
    const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    if (part == BQ) {  // the loss part: the tile's rows (and, in the last tile, the slice's rows past it)
#pragma unroll
        for (int k = 0; k < 2 * TR / TW; k++)
            if (k < TR / TW || tile == (int)gridDim.x - 1) loss_row(d, tgt_all, v_all, idx, B, vw, lrow, row0 + TW * k + wave, lane);
        return;
    }
    const int ks0 = part * PKS / BQ, ks1 = (part + 1) * PKS / BQ, ns = ks1 - ks0;
    // every wave owns columns when NACT == TW (hidden >= 128): a compile-time true, so no branch
    // around the weight ring (at a branch join the wait counters merge to the stricter count, and
    // a vmcnt(0) there would drain the ring's in-flight refills)
    const bool gw = NACT == TW || wave < NACT;
    const int nt0 = wave * NT;
    if (tid < TR) {
        const int row = row0 + tid;
        LSE[tid] = row < B ? row_lse(d, row) : 0.f;
        TG[tid] = row < B ? tgt_all[idx ? idx[row] : row] : -1;
    }
    // this part's logits first (every thread's, unconditionally, clamped), then the first slices
    // of Wpi^T: the gradient block then waits for the logits only (vmcnt retires in order)
    const int W = ns * 32;
    constexpr int LPT = (TR * SPMAX * 32 + TTHR - 1) / TTHR;  // logits per thread
    float lg[LPT];
#pragma unroll
    for (int k = 0; k < LPT; k++) {
        const int i = tid + TTHR * k, r = min(i / W, TR - 1), c = i - (i / W) * W;
        const int row = min(row0 + r, B - 1), a = min(32 * ks0 + c, ASIZE - 1);
        lg[k] = d.logits[(long)row * LDL + a];
    }
    float4 ring[RD][NT];
    if (gw) {  // the first slices of Wpi^T stream in while the gradient block is built
#pragma unroll
        for (int s = 0; s < RD; s++)
#pragma unroll
            for (int t = 0; t < NT; t++) ring[s][t] = d.wpit[((long)(nt0 + t) * PKS + min(ks0 + s, PKS - 1)) * 64 + lane];
    }
    __syncthreads();
    const float S = d.sc->scale, invB = 1.0f / (float)B;
#pragma unroll
    for (int k = 0; k < LPT; k++) {
        const int i = tid + TTHR * k;
        if (i < TR * W) {
            const int r = i / W, c = i - r * W, a = 32 * ks0 + c, row = row0 + r;
            float g = 0.f;
            if (row < B && a < ASIZE) g = r16(S * (expf(lg[k] - LSE[r]) - (a == TG[r] ? 1.0f : 0.0f)) * invB);
            DL[r * SD + c] = (_Float16)g;
        }
    }
    lds_barrier();
    write_tl<TR>(DL, SD, 0, W, d.dlT, d.RS, 2 * ks0, tile, row0 + TR >= B);
    for (int c = tid; c < W; c += TTHR) {  // the bias gradient's partial over these 16 rows
        float s = 0.f;
#pragma unroll
        for (int r = 0; r < TR; r++) s += (float)DL[r * SD + c];
        d.dbpi_part[(long)tile * LDL + 32 * ks0 + c] = s;
    }
    if (!gw) return;
    const _Float16* ap = DL + (lane & 15) * SD + 8 * (lane >> 4);
    floatx4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; t++) acc[t] = zero4();
    for (int k0 = 0; k0 < ns; k0 += RD) {
#pragma unroll
        for (int j = 0; j < RD; j++) {  // static ring slots
            const int k = k0 + j;
            const float4 a = *reinterpret_cast<const float4*>(ap + 32 * min(k, SPMAX - 1));
            const bool on = k < ns;  // (a select, not a branch: the refills below stay unconditional)
#pragma unroll
            for (int t = 0; t < NT; t++) {
                const floatx4 r = mfma(a, ring[j][t], acc[t]);
                acc[t] = on ? r : acc[t];
            }
#pragma unroll
            for (int t = 0; t < NT; t++)  // clamped; unused past the part's slices
                ring[j][t] = d.wpit[((long)(nt0 + t) * PKS + min(ks0 + k + RD, PKS - 1)) * 64 + lane];
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    const int r = lane & 15, q = lane >> 4;
#pragma unroll
    for (int t = 0; t < NT; t++)
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int row = row0 + 4 * q + j;
            if (row < B) d.dpart[((long)part * d.Bmax + row) * H + 16 * (nt0 + t) + r] = acc[t][j];
        }
}

struct DwJob {
    const float4* A;  // T layout of dU [B][N]
    const float4* X;  // T layout of X [B][K]
    float* dst;       // gradient [N][K] in the flat buffer
    int N, K;
};
// one weight-gradient item for one wave: (job, 16-row tile of W, up to 4 column tiles), summed over
// the batch's 32-row slices
// norm: returns the item's sum of (g / scale)^2 over what it writes, in every lane (yk_trainer_step's
// fused gradient norm: the grads k_amp_sq would read, summed where they are made); else 0
__device__ __forceinline__ double wave_dsum(double x) { return xlane_sum(x); }
#ifndef AMP_DW_SPLIT
#define AMP_DW_SPLIT 1  // waves per trunk dW item in k_amp_grads (2, 4: the batch's slices split; slower, r06p)
#endif
#ifndef AMP_VS_PAIRS
#define AMP_VS_PAIRS 4  // row pairs per batch of a column sum's loads (8, 16: within 0.3 us, r06r)
#endif
#ifndef AMP_DW_CH
// slices whose fragments a dW item loads at once: 8 (AMP step at batch 512 111.9 -> 109.5 us; 4: 110.2,
// 2: 112.2; at batch 64 8 costs 1 us over 4 - the reference trains at 512; profiles/r06q_dw_chunk_trainab.log)
#define AMP_DW_CH 8
#endif
constexpr int DW_IPB = 4 / AMP_DW_SPLIT;  // trunk dW items per 4-wave k_amp_grads block
// one dW item over S waves of the block (S = AMP_DW_SPLIT in k_amp_grads): wave part p sums slices
// [p rsn / S, (p + 1) rsn / S), AMP_DW_CH slices' fragments loaded at once (global loads, unconditional:
// past the part's last slice they re-read it), the MFMAs in slice order; part 0 adds
// the others' accumulators in part order (through LDS) and stores.  Every wave of the block calls it
// (has: whether its item exists), for the barrier.
template <int NK, int S = AMP_DW_SPLIT>
__device__ __forceinline__ double dw_item_split(const DwJob& jb, bool has, int nt, int kt0, int RS, int rsn, int lane,
                                                int part, bool norm, float inv, float* red, int wave) {
    constexpr int CH = AMP_DW_CH;
    floatx4 acc[NK];
#pragma unroll
    for (int t = 0; t < NK; t++) acc[t] = zero4();
    const int lo = part * rsn / S, hi = (part + 1) * rsn / S;
    if (has && hi > lo) {
        const float4* A = jb.A + (long)nt * RS * 64 + lane;
        const float4* X[NK];
#pragma unroll
        for (int t = 0; t < NK; t++) X[t] = jb.X + (long)(kt0 + t) * RS * 64 + lane;
        for (int r0 = lo; r0 < hi; r0 += CH) {
            float4 a[CH], x[CH][NK];
#pragma unroll
            for (int p = 0; p < CH; p++) {
                const int s0 = min(r0 + p, hi - 1);
                a[p] = gld4(A + (long)s0 * 64);
#pragma unroll
                for (int t = 0; t < NK; t++) x[p][t] = gld4(X[t] + (long)s0 * 64);
            }
#pragma unroll
            for (int p = 0; p < CH; p++)
                if (r0 + p < hi) {
#pragma unroll
                    for (int t = 0; t < NK; t++) acc[t] = mfma(a[p], x[p][t], acc[t]);
                }
        }
    }
    if (S > 1) {
        if (part > 0) {
#pragma unroll
            for (int t = 0; t < NK; t++)
#pragma unroll
                for (int j = 0; j < 4; j++) red[((wave * 4 + t) * 4 + j) * 64 + lane] = acc[t][j];
        }
        __syncthreads();
        if (part == 0) {
#pragma unroll
            for (int q = 1; q < S; q++)
#pragma unroll
                for (int t = 0; t < NK; t++)
#pragma unroll
                    for (int j = 0; j < 4; j++) acc[t][j] += red[(((wave + q) * 4 + t) * 4 + j) * 64 + lane];
        }
    }
    double ss = 0.0;
    if (has && part == 0) {
        const int q = lane >> 4, c = lane & 15;
#pragma unroll
        for (int t = 0; t < NK; t++) {
            const int k = 16 * (kt0 + t) + c;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int n = 16 * nt + 4 * q + j;
                if (n < jb.N && k < jb.K) {
                    const float g = r16(acc[t][j]);  // fp16 grad_weight
                    gptr(jb.dst)[(long)n * jb.K + k] = g;
                    const double x2 = (double)(g * inv);
                    ss += x2 * x2;
                }
            }
        }
    }
    return norm ? wave_dsum(ss) : 0.0;
}
// one weight-gradient item for one wave (the heads' items inside k_amp_bwd): the chunked form, unsplit
__device__ __forceinline__ double dw_item(const DwJob* __restrict__ jobs, const int4 it, int RS, int rsn, int lane,
                                          bool norm = false, float inv = 1.f) {
    const DwJob jb = jobs[it.x];
    switch (it.w) {  // (uniform: the item's column tiles; amp_create's kg 2 or 4 divides every job's)
        case 1: return dw_item_split<1, 1>(jb, true, it.y, it.z, RS, rsn, lane, 0, norm, inv, nullptr, 0);
        case 2: return dw_item_split<2, 1>(jb, true, it.y, it.z, RS, rsn, lane, 0, norm, inv, nullptr, 0);
        case 3: return dw_item_split<3, 1>(jb, true, it.y, it.z, RS, rsn, lane, 0, norm, inv, nullptr, 0);
        default: return dw_item_split<4, 1>(jb, true, it.y, it.z, RS, rsn, lane, 0, norm, inv, nullptr, 0);
    }
}
// a block's waves' norm partials -> sqp[slot] (wave order: fixed bits); every thread calls it
template <int NW>
__device__ __forceinline__ void block_norm(double ss, double* __restrict__ sqp, int slot) {
    __shared__ double red[NW];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
#pragma unroll
        for (int k = 0; k < NW; k++) t += red[k];
        sqp[slot] = t;
    }
}

// ------------------------------------------------------------------ backward (trunk)
// What one row pass of k_amp_bwd reads from memory, loaded into registers BEFORE the GEMM that
// precedes it: the GEMM's weight-ring refills are issued after these loads, and vmcnt retires in
// order, so the row pass never waits for the next layer's weights.
template <int VPL>
struct RowPre {
    float u[TRPW][VPL];  // the layer's saved pre-activation (block layers) or Z0 (input layer)
    float mu[TRPW], rs[TRPW];
    float g[VPL], be[VPL];
    uint32_t mk[TRPW];  // the dropout layer's keep bits (k_amp_masks), when the pass has one
};
template <int H>
__device__ __forceinline__ void row_prefetch(RowPre<H / 64>& R, const AmpDev& d, const float* U, int L, int tg, int tb,
                                             int row0, int B, int ML, bool drop) {
    constexpr int VPL = H / 64;
    const int wave = threadIdx.x >> 6, c0 = (threadIdx.x & 63) * VPL;
#pragma unroll
    for (int rr = 0; rr < TRPW; rr++) {
        const int row = row0 + wave * TRPW + rr;
        const int rc = row < B ? row : 0;
#pragma unroll
        for (int i = 0; i < VPL; i++) R.u[rr][i] = U[(long)rc * H + c0 + i];
        R.mu[rr] = stat_ptr(d, L, 0)[rc];
        R.rs[rr] = stat_ptr(d, L, 1)[rc];
        R.mk[rr] = drop ? mask_bits<VPL>(d, ML, rc, c0) : 0xFFu;
    }
    const float* g = d.P + poff(H, d.NB, tg);
    const float* be = d.P + poff(H, d.NB, tb);
#pragma unroll
    for (int i = 0; i < VPL; i++) {
        R.g[i] = g[c0 + i];
        R.be[i] = be[c0 + i];
    }
}
// CP (per-wave partials, slots 0 gamma, 1 beta, 2 bias) summed over the waves into colpart
// vectors vb (bias), vb + 1 (gamma), vb + 2 (beta)
template <int H>
__device__ __forceinline__ void flush_gbb(const AmpDev& d, const float* CP, int tile, int vb) {
    for (int i = threadIdx.x; i < 3 * H; i += TTHR) {
        const int k = i / H, c = i % H;
        const int slot = k == 0 ? 2 : k - 1;
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < TW; w++) s += CP[w * 3 * H + slot * H + c];
        d.colpart[((long)tile * d.NVEC + vb + k) * H + c] = s;
    }
}

template <int H>
__global__ __launch_bounds__(TTHR) void k_amp_bwd(AmpDev d, int B, float p, uint64_t seed, uint64_t step,
                                                  int64_t row_base, const DwJob* __restrict__ jobs,
                                                  const int4* __restrict__ hitems, int nhitems, int rsn,
                                                  double* __restrict__ sqp, int slot0) {
    constexpr int LD = H + 4, SA = H + 8, VPL = H / 64, KS = H / 32;
    constexpr int NT = H >= 128 ? H / 128 : 1, NACT = H / (16 * NT);
    constexpr int RW = KS * NT <= 16 ? KS : 16 / NT;
    constexpr int BDEF = (RW == KS && KS >= 8) ? 6 : 0;  // deferred ring refills per trunk GEMM (k_amp_fwd's FDEF)
    constexpr int SV = VH + 8;
    static_assert(SV <= SA || H == 64, "dz1 rows fit the plane buffer");
    __shared__ __attribute__((aligned(16))) float Xs[TR * LD];
    __shared__ __attribute__((aligned(16))) float Ts[TR * LD];
    __shared__ __attribute__((aligned(16))) _Float16 Pa[TR * (SA > SV ? SA : SV)];
    __shared__ __attribute__((aligned(16))) float CP[TW * 3 * H];
    const int tile = blockIdx.x, row0 = tile * TRV;
    const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    if (row0 >= B) {  // the blocks past the row tiles: the heads' weight gradients (their operands are
                      // done before this launch), on the CUs the trunk's 8-row workgroups leave idle
        const int hb = tile - (B + TRV - 1) / TRV, w = hb * TW + wave;
        double ss = 0.0;
        if (w < nhitems) ss = dw_item(jobs, hitems[w], d.RS, rsn, lane, sqp != nullptr, sqp ? 1.0f / d.sc->scale : 1.f);
        if (sqp) block_norm<TW>(ss, sqp, slot0 + hb);
        return;
    }
    // every wave owns columns when NACT == TW (hidden >= 128): a compile-time true, so no branch
    // around the weight ring (at a branch join the wait counters merge to the stricter count, and
    // a vmcnt(0) there would drain the ring's in-flight refills)
    const bool gw = NACT == TW || wave < NACT;
    const int nt0 = wave * NT, c0 = lane * VPL;
    const bool zero_rest = row0 + TRV >= B;
    const float sc = p > 0.f ? 1.0f / (1.0f - p) : 1.0f;
    const int NB = d.NB;
    const long HH8 = (long)H * H / 8;
    const bool drop = p > 0.f;  // the keep bits: k_amp_masks
    const long TLH = (long)(H / 16) * d.RS * 512;  // halves per T-layout [32 RS][H] matrix
    float* cp = CP + wave * 3 * H;

    // dA_v = fp16(dz1_16 Wv1_16): K = 128 (4 slices), the dz1 rows staged in Pa
    float4 wv[4][NT];
    if (gw) {
#pragma unroll
        for (int s = 0; s < 4; s++)
#pragma unroll
            for (int t = 0; t < NT; t++) wv[s][t] = d.wv1t[((long)(nt0 + t) * 4 + s) * 64 + lane];
    }
    for (int i = tid; i < TR * VH / 8; i += TTHR) {  // (clamped loads, zeroed by a select: no branch;
        const int r = i / (VH / 8), c8 = i % (VH / 8), row = row0 + r;  // rows past TRV: zeros)
        const float4 v = reinterpret_cast<const float4*>(d.dz1_rm + (long)min(row, B - 1) * VH)[c8];
        *reinterpret_cast<float4*>(Pa + r * SV + 8 * c8) = row < B && r < TRV ? v : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    lds_barrier();
    floatx4 acc[NT];
    if (gw) {
        const _Float16* ap = Pa + (lane & 15) * SV + 8 * (lane >> 4);
#pragma unroll
        for (int t = 0; t < NT; t++) acc[t] = zero4();
#pragma unroll
        for (int s = 0; s < 4; s++) {
            const float4 a = *reinterpret_cast<const float4*>(ap + 32 * s);
#pragma unroll
            for (int t = 0; t < NT; t++) acc[t] = mfma(a, wv[s][t], acc[t]);
        }
        store_acc<NT>(Ts, LD, nt0, acc);
    }
    // the heads pass's operands (the split-K parts of dA_pi, the trunk output, its statistics,
    // the heads' LayerNorm affines) are loaded before the trunk ring starts streaming
    float dapi[TRPW][VPL], hx[TRPW][VPL], hmu[TRPW], hrs[TRPW];
    float gp[VPL], bp[VPL], gv[VPL], bv[VPL];
#pragma unroll
    for (int rr = 0; rr < TRPW; rr++) {
        const int row = row0 + wave * TRPW + rr, rc = row < B ? row : 0;
#pragma unroll
        for (int i = 0; i < VPL; i++) {
            float a = 0.f;
#pragma unroll
            for (int qq = 0; qq < BQ; qq++) a += d.dpart[((long)qq * d.Bmax + rc) * H + c0 + i];
            dapi[rr][i] = r16(a);  // fp16(dlogits16 Wpi16)
            hx[rr][i] = d.hF[(long)rc * H + c0 + i];
        }
        hmu[rr] = stat_ptr(d, 1 + 2 * NB, 0)[rc];
        hrs[rr] = stat_ptr(d, 1 + 2 * NB, 1)[rc];
    }
#pragma unroll
    for (int i = 0; i < VPL; i++) {
        gp[i] = d.P[poff(H, NB, t_head(NB, HP_G)) + c0 + i];
        bp[i] = d.P[poff(H, NB, t_head(NB, HP_B)) + c0 + i];
        gv[i] = d.P[poff(H, NB, t_head(NB, HV_G)) + c0 + i];
        bv[i] = d.P[poff(H, NB, t_head(NB, HV_B)) + c0 + i];
    }
    RowPre<VPL> R;  // (one call on selected operands, and the ring filled whatever NB is - from a large
                    // enough matrix when NB = 0 - so no branch joins before the heads pass's waits)
    row_prefetch<H>(R, d, NB > 0 ? d.u2 + (long)(NB - 1) * d.Bmax * H : d.z0, NB > 0 ? 2 * NB : 0,
                    NB > 0 ? t_blk(NB - 1, 6) : (int)T_GIN, NB > 0 ? t_blk(NB - 1, 7) : (int)T_BEIN, row0, B, 0, drop);
    __builtin_amdgcn_sched_barrier(0);
    float4 ring[RW][NT];
    // (the first trunk GEMM's last BDEF slots are loaded in the row pass before it, as every later
    // GEMM's: gemm_ring's deferred refills)
    if (gw) {
        const float4* first = NB > 0 ? d.w2t + (NB - 1) * HH8 : d.wpit;
        if constexpr (BDEF > 0) ring_part<KS, NT, RW, 0, KS - BDEF>(ring, first, nt0);
        else ring_fill<KS, NT, RW>(ring, first, nt0);
    }
    lds_barrier();
    // heads backward (YachtNNet.py:40-52): dT = dA SiLU'(T) for both heads (f32), one LayerNorm
    // backward over the shared statistics -> dh
    {
        float dgv[TRPW][VPL], dbev[TRPW][VPL];
#pragma unroll
        for (int rr = 0; rr < TRPW; rr++) {
            const int r = wave * TRPW + rr, row = row0 + r;
            float dx[VPL], xh[VPL];
#pragma unroll
            for (int i = 0; i < VPL; i++) {
                const int c = c0 + i;
                xh[i] = (hx[rr][i] - hmu[rr]) * hrs[rr];
                const float dtp = row < B ? dapi[rr][i] * silu_grad(xh[i] * gp[i] + bp[i]) : 0.f;
                const float dtv = row < B ? r16(Ts[r * LD + c]) * silu_grad(xh[i] * gv[i] + bv[i]) : 0.f;
                cp[c] = (rr == 0 ? 0.f : cp[c]) + dtp * xh[i];  // pi_head.0.weight
                cp[H + c] = (rr == 0 ? 0.f : cp[H + c]) + dtp;  // pi_head.0.bias
                dgv[rr][i] = dtv * xh[i];
                dbev[rr][i] = dtv;
                dx[i] = dtp * gp[i] + dtv * gv[i];
            }
            if (row < B) ln_bwd<VPL>(xh, dx, H, hrs[rr]);
#pragma unroll
            for (int i = 0; i < VPL; i++) Xs[r * LD + c0 + i] = row < B ? dx[i] : 0.f;
        }
        lds_barrier();
        colpart_flush<H>(d, CP, tile, CV_GPI, 2);
        lds_barrier();
#pragma unroll
        for (int i = 0; i < VPL; i++) {
            float g2 = 0.f, b2 = 0.f;
#pragma unroll
            for (int rr = 0; rr < TRPW; rr++) {
                g2 += dgv[rr][i];
                b2 += dbev[rr][i];
            }
            cp[c0 + i] = g2;
            cp[H + c0 + i] = b2;
        }
        lds_barrier();
        colpart_flush<H>(d, CP, tile, CV_GV, 2);
        lds_barrier();
    }

    // the trunk, last block first: per block  LN2 bwd -> dU2 -> dR1 = dU2 W2 -> dropout, LN1 bwd ->
    // dU1 -> dh += dU1 W1; the ring streams W2^T[b], W1^T[b], W2^T[b-1], ...
    for (int b = NB - 1; b >= 0; b--) {
        for (int half = 1; half >= 0; half--) {
            // row pass: (half 1) dL2 = dh; (half 0) dL1 = Dropout'(fp16(dR1)).  LayerNorm backward on
            // S = fp16(SiLU(U)), dU = fp16(fp16(dS) SiLU'(U)); partials: gamma, beta, bias
            const float4* cur = (half == 1 ? d.w2t : d.w1t) + b * HH8;
            // this step's GEMM's last BDEF slots (the previous GEMM deferred them), half before the row
            // pass and half after it
            if constexpr (BDEF > 0) if (gw) ring_part<KS, NT, RW, KS - BDEF, KS - BDEF / 2>(ring, cur, nt0);
#pragma unroll
            for (int rr = 0; rr < TRPW; rr++) {
                const int r = wave * TRPW + rr, row = row0 + r;
                float dx[VPL], xh[VPL];
#pragma unroll
                for (int i = 0; i < VPL; i++) {
                    const int c = c0 + i;
                    xh[i] = (r16(silu(R.u[rr][i])) - R.mu[rr]) * R.rs[rr];
                    float dl = 0.f;
                    if (row < B) {
                        if (half == 1) {
                            dl = Xs[r * LD + c];
                        } else {
                            const bool k = (R.mk[rr] >> i) & 1u;
                            dl = k ? r16(Ts[r * LD + c]) * sc : 0.f;
                        }
                    }
                    cp[c] = (rr == 0 ? 0.f : cp[c]) + dl * xh[i];
                    cp[H + c] = (rr == 0 ? 0.f : cp[H + c]) + dl;
                    dx[i] = dl * R.g[i];
                }
                if (row < B) ln_bwd<VPL>(xh, dx, H, R.rs[rr]);
#pragma unroll
                for (int i = 0; i < VPL; i++) {
                    dx[i] = row < B ? r16(r16(dx[i]) * silu_grad(R.u[rr][i])) : 0.f;  // dU (fp16)
                    cp[2 * H + c0 + i] = (rr == 0 ? 0.f : cp[2 * H + c0 + i]) + dx[i];
                    Pa[r * SA + c0 + i] = (_Float16)dx[i];
                }
            }
            if constexpr (BDEF > 0) if (gw) ring_part<KS, NT, RW, KS - BDEF / 2, KS>(ring, cur, nt0);
            lds_barrier();
            flush_gbb<H>(d, CP, tile, CV_BLK + 6 * b + (half == 0 ? 0 : 3));
            write_tl<TRV>(Pa, SA, 0, H, (half == 0 ? d.du1T : d.du2T) + b * TLH, d.RS, 0, tile, zero_rest);
            // the next row pass's operands, then dX = fp16(dU16 W16) (W2 of half 1, W1 of half 0)
            // (one call on selected operands: loads in one code path keep the wait counters exact)
            {
                const bool h1 = half == 1, more = b > 0;
                const float* Up = h1 ? d.u1 + (long)b * d.Bmax * H : more ? d.u2 + (long)(b - 1) * d.Bmax * H : d.z0;
                const int Lp = h1 ? 1 + 2 * b : more ? 2 * b : 0;
                const int tg = h1 ? t_blk(b, 2) : more ? t_blk(b - 1, 6) : (int)T_GIN;
                const int tb = h1 ? t_blk(b, 3) : more ? t_blk(b - 1, 7) : (int)T_BEIN;
                row_prefetch<H>(R, d, Up, Lp, tg, tb, row0, B, h1 ? 1 + b : 0, drop);  // (next: b's fc1 dropout / inp's)
            }
            __builtin_amdgcn_sched_barrier(0);
            const float4* nxt = half == 1 ? d.w1t + b * HH8 : (b > 0 ? d.w2t + (b - 1) * HH8 : nullptr);
            if (gw) {
                gemm_ring<KS, NT, RW, BDEF>(Pa, SA, ring, acc, cur, nxt, nt0);
                store_acc<NT>(Ts, LD, nt0, acc);
            }
            lds_barrier();
            if (half == 0) {  // residual: dh_b = dh_{b+1} + fp16(dU1 W1)
#pragma unroll
                for (int rr = 0; rr < TRPW; rr++) {
                    const int r = wave * TRPW + rr;
#pragma unroll
                    for (int i = 0; i < VPL; i++) Xs[r * LD + c0 + i] += r16(Ts[r * LD + c0 + i]);
                }
                lds_barrier();
            }
        }
    }
    // inp (YachtNNet.py:30-35): dh0 -> Dropout' -> SiLU'(a) -> LayerNorm backward -> dZ0 (fp16)
#pragma unroll
    for (int rr = 0; rr < TRPW; rr++) {
        const int r = wave * TRPW + rr, row = row0 + r;
        float dx[VPL], xh[VPL];
#pragma unroll
        for (int i = 0; i < VPL; i++) {
            const int c = c0 + i;
            xh[i] = (R.u[rr][i] - R.mu[rr]) * R.rs[rr];
            float ds = 0.f;
            if (row < B) {
                const bool k = (R.mk[rr] >> i) & 1u;
                const float da = k ? Xs[r * LD + c] * sc : 0.f;
                ds = da * silu_grad(xh[i] * R.g[i] + R.be[i]);
            }
            cp[c] = (rr == 0 ? 0.f : cp[c]) + ds * xh[i];
            cp[H + c] = (rr == 0 ? 0.f : cp[H + c]) + ds;
            dx[i] = ds * R.g[i];
        }
        if (row < B) ln_bwd<VPL>(xh, dx, H, R.rs[rr]);
#pragma unroll
        for (int i = 0; i < VPL; i++) {
            dx[i] = row < B ? r16(dx[i]) : 0.f;
            cp[2 * H + c0 + i] = (rr == 0 ? 0.f : cp[2 * H + c0 + i]) + dx[i];
            Pa[r * SA + c0 + i] = (_Float16)dx[i];
        }
    }
    lds_barrier();
    flush_gbb<H>(d, CP, tile, CV_BIN);
    write_tl<TRV>(Pa, SA, 0, H, d.dz0T, d.RS, 0, tile, zero_rest);
}

// ------------------------------------------------------------------ weight gradients

// fixed-order column sums: dst[c] = sum_r src[r * ld + c] over `rows` rows (tiles or examples).
// Block = one job's 16 columns x 16 row groups (row r to group r % 16), the groups added in order.
struct VsJob {
    const float* src;
    float* dst;
    int ld, N, per_example, round16;  // per_example: rows are 0 trunk tiles, 1 examples, 2 head tiles
    int in_grad;                      // dst is part of the gradient buffer (not the loss sums)
};
// one column-sum item for a 256-thread block: 16 columns of a job, 16 row groups, fixed order
__device__ __forceinline__ void vecsum_item(const VsJob* __restrict__ jobs, const int2 it, int ntiles, int nhtiles,
                                            int B, float (&part)[16][17], double* __restrict__ sqp = nullptr,
                                            int slot = 0, float inv = 1.f) {
    const VsJob jb = jobs[it.x];
    const int c = it.y + (threadIdx.x & 15), g = threadIdx.x >> 4;
    const int rows = jb.per_example == 1 ? B : jb.per_example == 2 ? nhtiles : ntiles;
    float a0 = 0.f, a1 = 0.f;
    typedef const __attribute__((address_space(1))) float gfloat;  // (global loads, not flat)
    gfloat* src = (gfloat*)jb.src;
    if (c < jb.N) {
        int r = g;
        // per-example jobs (B rows): 2 VSP loads in flight per batch, added in the same order (a0: rows
        // g, g + 32, ..; a1: g + 16, g + 48, ..) as the one-pair loop below
        constexpr int VSP = AMP_VS_PAIRS;
        for (; r + 16 + 32 * (VSP - 1) < rows; r += 32 * VSP) {
            float v[2 * VSP];
#pragma unroll
            for (int k = 0; k < VSP; k++) {
                v[2 * k] = src[(long)(r + 32 * k) * jb.ld + c];
                v[2 * k + 1] = src[(long)(r + 32 * k + 16) * jb.ld + c];
            }
#pragma unroll
            for (int k = 0; k < VSP; k++) {
                a0 += v[2 * k];
                a1 += v[2 * k + 1];
            }
        }
        for (; r + 16 < rows; r += 32) {
            a0 += src[(long)r * jb.ld + c];
            a1 += src[(long)(r + 16) * jb.ld + c];
        }
        for (; r < rows; r += 16) a0 += src[(long)r * jb.ld + c];
    }
    part[g][threadIdx.x & 15] = a0 + a1;
    __syncthreads();
    double ss = 0.0;
    if (g == 0 && c < jb.N) {
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < 16; k++) s += part[k][threadIdx.x];
        const float v = jb.round16 ? r16(s) : s;
        gptr(jb.dst)[c] = v;
        const double x = jb.in_grad ? (double)(v * inv) : 0.0;
        ss = x * x;
    }
    if (sqp && threadIdx.x < 64) {  // (the 16 column threads are wave 0's lanes 0-15)
        ss = wave_dsum(ss);
        if (threadIdx.x == 0) sqp[slot] = ss;
    }
}
// after k_amp_bwd: the trunk's weight gradients (dw_item, a wave each; the heads' ran inside
// k_amp_bwd's launch) and, in the blocks past them, the bias / LayerNorm gradients and loss sums
// (vecsum_item, a block each) - one launch for both
// With sqp (yk_trainer_step): every block's norm partial into its slot (this launch's dW blocks
// 0 .., k_amp_bwd's dW blocks after them, the column sums after all nall dW blocks);
// k_amp_update sums the slots (a last-block reduction here instead would need an agent-scope
// release per block - an L2 writeback on this multi-XCD part: 12 -> 96 us measured).
__global__ __launch_bounds__(256) void k_amp_grads(const DwJob* __restrict__ jobs, const int4* __restrict__ items,
                                                   int nitems, int RS, int rsn, const VsJob* __restrict__ vjobs,
                                                   const int2* __restrict__ vitems, int nvitems, int ntiles,
                                                   int nhtiles, int B, double* __restrict__ sqp, int nall,
                                                   const Scaler* __restrict__ sc) {
    __shared__ float part[16][17];
    __shared__ float red[AMP_DW_SPLIT > 1 ? 4 * 4 * 4 * 64 : 1];  // the split dW items' partial accumulators
    const float inv = sqp ? 1.0f / sc->scale : 1.f;
    const int ndb = (nitems + DW_IPB - 1) / DW_IPB;
    if ((int)blockIdx.x >= ndb) {
        const int v = (int)blockIdx.x - ndb;
#ifndef AMP_DIAG_NO_VS
        if (v < nvitems) vecsum_item(vjobs, vitems[v], ntiles, nhtiles, B, part, sqp, nall + v, inv);
#endif
    } else {
        const int wave = threadIdx.x >> 6;
        const int w = blockIdx.x * DW_IPB + wave / AMP_DW_SPLIT;
        double ss = 0.0;
#ifndef AMP_DIAG_NO_DW
        const bool has = w < nitems;
        const int4 it = items[has ? w : 0];
        const DwJob jb = jobs[it.x];
        // (every trunk item has YK_DW_KG column tiles: amp_create builds them so, and every trunk
        // matrix's column-tile count, H / 16 or 4 for the input layer, is a multiple of it)
        ss = dw_item_split<YK_DW_KG>(jb, has, it.y, it.z, RS, rsn, threadIdx.x & 63, wave % AMP_DW_SPLIT, sqp != nullptr,
                                     inv, red, wave);
#endif
        if (sqp) block_norm<4>(ss, sqp, blockIdx.x);
    }
}

// ------------------------------------------------------------------ optimiser

// GradScaler.unscale_: the norm of the unscaled gradients (an inf / nan anywhere makes it so)
__global__ void k_amp_sq(const float* __restrict__ g, long n, const Scaler* sc, double* __restrict__ part) {
    __shared__ double red[4];
    const float inv = 1.0f / sc->scale;
    double s = 0.0;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const double x = (double)(g[i] * inv);
        s += x * x;
    }
    s = xlane_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}
// n norm partials summed by a 256-thread block in one fixed order (every caller gets the same
// bits): strided per thread, the wave butterflies, the 4 waves in order
__device__ __forceinline__ double sq_total(const double* part, int n) {
    __shared__ double red[4];
    double t = 0.0;
#pragma unroll 8
    for (int i = threadIdx.x; i < n; i += 256) t += part[i];
    t = xlane_sum(t);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = t;
    __syncthreads();
    const double tot = (red[0] + red[1]) + (red[2] + red[3]);
    __syncthreads();
    return tot;
}
// fp16 fragments of one weight matrix W[N][K] (f32, row-major): `trans` packs W^T
struct PackJob {
    const float* W;
    float4* dst;
    int N, K, Np, Kp, trans;  // packed shape Np x Kp (of W or of W^T)
    long first;               // first item (float4) of this job
};
// the fp16 weight copies of the parameters (creation, a parameter load); the optimiser step
// refreshes them itself (k_amp_update).  blk_job[b]: the job of block b (every job's item count
// is a multiple of the block size, so a block lies in one job; checked in amp_create)
__global__ void k_amp_pack(const PackJob* __restrict__ jobs, const uint8_t* __restrict__ blk_job, long total) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const PackJob jb = jobs[blk_job[blockIdx.x]];
    const long e = i - jb.first;
    const int KS = jb.Kp / 32;
    const int lane = (int)(e % 64);
    const long pc = e / 64;
    const int nt = (int)(pc / KS), ks = (int)(pc % KS);
    const int n = 16 * nt + (lane & 15), k0 = 32 * ks + 8 * (lane >> 4);
    half8 v;
#pragma unroll
    for (int t = 0; t < 8; t++) {
        const int k = k0 + t;
        float x = 0.f;
        if (!jb.trans) {
            if (n < jb.N && k < jb.K) x = jb.W[(long)n * jb.K + k];
        } else {  // W^T[n][k] = W[k][n]
            if (k < jb.N && n < jb.K) x = jb.W[(long)k * jb.K + n];
        }
        v[t] = (_Float16)x;
    }
    *reinterpret_cast<half8*>(jb.dst + e) = v;
}

// scaler.step + scaler.update + the fp16 repack in one launch: a block owns a 32 x 32 tile of one
// weight matrix - AdamW on its 1024 elements (torch's single-tensor update), then both fp16
// fragment orientations of the tile from LDS -
// or a 1024-element slice of the vectors (biases, LayerNorms, v_head.4).  The GradScaler state is
// double-buffered: every block reads `sc`, block 0 writes the updated state to `sc_next` (the
// host swaps them), so no block can see a half-updated scale.
struct UpdJob {
    float *W, *Gm, *Mm, *Vm;  // the matrix [N][K] in the parameter / gradient / moment buffers (or a vector range)
    float4 *dstN, *dstT;      // fp16 fragments of W (packed columns KpN) and of W^T (packed columns KpT), or null
    int N, K, KpN, KpT;
};
struct UpdItem {
    int job, n0, k0;  // a matrix tile's first row / column; a vector slice: n0 = first element, k0 = count
};
__device__ __forceinline__ void adamw_elem(float& p, float& g, float& m, float& v, float inv, float coef,
                                           float decay, float b1, float b2, float eps, float step_size,
                                           float bc2_sqrt) {  // torch.optim.AdamW's single-tensor step
    // Its multiply-adds fused explicitly, one per torch op, as the GPU build of ATen's pointwise
    // formulas contracts them (lerp_ below weight 0.5: self + w (end - self); addcmul_: self + value
    // (t1 t2); addcdiv_: self + value (t1 / t2)) - not left to -ffp-contract=fast, whose choice
    // of which product to fuse moved with the surrounding code (train losses changed with the
    // update kernel's block shape alone, profiles/r05zb_update_items_trainab.log).
#pragma clang fp contract(off)
    const float gi = (g * inv) * coef;  // unscale_, then clip_grad_norm_'s mul_
    g = gi;
    const float pi = p * decay;                            // p.mul_(1 - lr wd)
    const float mi = __builtin_fmaf(1.0f - b1, gi - m, m);  // m.lerp_(g, 1 - b1)
    const float vi = __builtin_fmaf(1.0f - b2, gi * gi, v * b2);  // v.mul_(b2).addcmul_(g, g, 1 - b2)
    m = mi;
    v = vi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;        // (v.sqrt() / bc2_sqrt).add_(eps)
    p = __builtin_fmaf(-step_size, mi / denom, pi);        // p.addcdiv_(m, denom, -step_size)
}
// the fp16 copy of a stored float32 weight, rounded from that float32: the value is opaque to the
// compiler, which would otherwise fold the conversion into the weight's fma as one v_fma_mixlo_f16
// (a single rounding to fp16 - unlike k_amp_pack's and torch's autocast cast of the stored weight)
__device__ __forceinline__ _Float16 f16_of_stored(float x) {
    asm volatile("" : "+v"(x));
    return (_Float16)x;
}
__global__ __launch_bounds__(256) void k_amp_update(const UpdJob* __restrict__ jobs, const UpdItem* __restrict__ items,
                                                    const double* __restrict__ part, double* sq_out,
                                                    const Scaler* __restrict__ sc, Scaler* __restrict__ sc_next,
                                                    float max_norm, float lr, float wd, float b1, float b2, float eps,
                                                    int n_upd, AmpDev d, float mp, uint64_t mseed, uint64_t mstep,
                                                    int npart) {
    __shared__ _Float16 Tl[32][40];
    if ((int)blockIdx.x >= n_upd) {  // the blocks past the update's: the next step's dropout draws
        const int q4 = d.H / 4;       // (k_amp_masks' work for row offset 0 and every row of Bmax)
        const long i = (long)(blockIdx.x - n_upd) * 256 + threadIdx.x;
        if (i < (long)(1 + d.NB) * d.Bmax * q4) {
            const int q = (int)(i % q4), row = (int)((i / q4) % d.Bmax), L = (int)(i / ((long)q4 * d.Bmax));
            d.masks[((long)L * d.Bmax + row) * q4 + q] = (uint8_t)dropout_bits(mseed, L, mstep, (long)row * q4 + q, mp);
        }
        return;
    }
    const double total = sq_total(part, npart);  // (k_amp_sq's SQ_BLOCKS partials or the fused norm's slots)
    const Scaler s0 = *sc;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        *sq_out = total;
        Scaler n = s0;  // GradScaler('cuda').update: growth 2, backoff 0.5
        if (!isfinite(total)) {
            n.scale *= 0.5f;
            n.tracker = 0;
            n.found_inf = 1;
        } else {
            n.steps += 1;
            n.found_inf = 0;
            if (++n.tracker == n.growth_interval) {
                n.scale *= 2.0f;
                n.tracker = 0;
            }
        }
        *sc_next = n;
    }
    const float inv = 1.0f / s0.scale;
    if (!isfinite(total)) {  // step skipped: parameters and their fp16 copies unchanged.  The gradient
        // buffer ends as p.grad does in torch: unscale_ (x 1/scale), then clip_grad_norm_'s multiply by
        // its clamped coefficient max_norm / (total_norm + 1e-6) - 0 for an infinite norm (finite entries
        // -> +-0, infinite ones -> nan), nan for a nan norm
        float cf = max_norm / ((float)sqrt(total) + 1e-6f);
        cf = cf > 1.0f ? 1.0f : cf;
        const UpdItem it = items[blockIdx.x];
        const UpdJob jb = jobs[it.job];
        const int t = threadIdx.x;
        if (!jb.dstN) {
            for (int i = 0; i < 4; i++)
                if (4 * t + i < it.k0) gptr(jb.Gm)[(long)it.n0 + 4 * t + i] = (gptr(jb.Gm)[(long)it.n0 + 4 * t + i] * inv) * cf;
        } else {
            const int n = it.n0 + (t >> 3);
            for (int i = 0; i < 4; i++) {
                const int k = it.k0 + (t & 7) * 4 + i;
                if (n < jb.N && k < jb.K) gptr(jb.Gm)[(long)n * jb.K + k] = (gptr(jb.Gm)[(long)n * jb.K + k] * inv) * cf;
            }
        }
        return;
    }
    const double st = (double)(s0.steps + 1);
    const float step_size = (float)((double)lr / (1.0 - pow((double)b1, st)));
    const float bc2_sqrt = (float)sqrt(1.0 - pow((double)b2, st));
    const float norm = (float)sqrt(total);
    float coef = max_norm / (norm + 1e-6f);
    coef = coef > 1.0f ? 1.0f : coef;
    const float decay = 1.0f - lr * wd;
    const UpdItem it = items[blockIdx.x];
    const UpdJob jb = jobs[it.job];
    const int t = threadIdx.x;
    if (!jb.dstN) {  // a vector slice: 4 consecutive elements per thread
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int e = 4 * t + i;
            if (e < it.k0) {
                const long o = (long)it.n0 + e;
                float p = gptr(jb.W)[o], g = gptr(jb.Gm)[o], m = gptr(jb.Mm)[o], v = gptr(jb.Vm)[o];
                adamw_elem(p, g, m, v, inv, coef, decay, b1, b2, eps, step_size, bc2_sqrt);
                gptr(jb.W)[o] = p;
                gptr(jb.Gm)[o] = g;
                gptr(jb.Mm)[o] = m;
                gptr(jb.Vm)[o] = v;
            }
        }
        return;
    }
    const int r = t >> 3, c = (t & 7) * 4;
    const int n = it.n0 + r;
    const long o4 = (long)n * jb.K + it.k0 + c;
    const bool vec = (jb.K & 3) == 0 && n < jb.N && it.k0 + c + 3 < jb.K &&
                     ((reinterpret_cast<uintptr_t>(jb.W) | reinterpret_cast<uintptr_t>(jb.Gm) |
                       reinterpret_cast<uintptr_t>(jb.Mm) | reinterpret_cast<uintptr_t>(jb.Vm)) & 15) == 0;
    if (vec) {  // 16-byte aligned rows: four elements per load
        const long o = o4;
        float4 p = gld4(reinterpret_cast<const float4*>(jb.W + o)), g = gld4(reinterpret_cast<const float4*>(jb.Gm + o));
        float4 m = gld4(reinterpret_cast<const float4*>(jb.Mm + o)), v = gld4(reinterpret_cast<const float4*>(jb.Vm + o));
        adamw_elem(p.x, g.x, m.x, v.x, inv, coef, decay, b1, b2, eps, step_size, bc2_sqrt);
        adamw_elem(p.y, g.y, m.y, v.y, inv, coef, decay, b1, b2, eps, step_size, bc2_sqrt);
        adamw_elem(p.z, g.z, m.z, v.z, inv, coef, decay, b1, b2, eps, step_size, bc2_sqrt);
        adamw_elem(p.w, g.w, m.w, v.w, inv, coef, decay, b1, b2, eps, step_size, bc2_sqrt);
        gst4(jb.W + o, p);
        gst4(jb.Gm + o, g);
        gst4(jb.Mm + o, m);
        gst4(jb.Vm + o, v);
        Tl[r][c] = f16_of_stored(p.x);
        Tl[r][c + 1] = f16_of_stored(p.y);
        Tl[r][c + 2] = f16_of_stored(p.z);
        Tl[r][c + 3] = f16_of_stored(p.w);
    } else {
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int k = it.k0 + c + i;
            float pv = 0.f;
            if (n < jb.N && k < jb.K) {
                const long o = (long)n * jb.K + k;
                float p = gptr(jb.W)[o], g = gptr(jb.Gm)[o], m = gptr(jb.Mm)[o], v = gptr(jb.Vm)[o];
                adamw_elem(p, g, m, v, inv, coef, decay, b1, b2, eps, step_size, bc2_sqrt);
                gptr(jb.W)[o] = p;
                gptr(jb.Gm)[o] = g;
                gptr(jb.Mm)[o] = m;
                gptr(jb.Vm)[o] = v;
                pv = p;
            }
            Tl[r][c + i] = f16_of_stored(pv);
        }
    }
    __syncthreads();
    const int f = (t >> 6) & 1, l = t & 63;
    half8 h;
    if (t < 128) {  // W: fragment (n0 / 16 + f, k0 / 32), lane l = W[16 nt + (l & 15)][32 ks + 8 (l >> 4) + j]
        const int rr = 16 * f + (l & 15), kk = 8 * (l >> 4);
#pragma unroll
        for (int j = 0; j < 8; j++) h[j] = Tl[rr][kk + j];
        gsth8(jb.dstN + ((long)(it.n0 / 16 + f) * (jb.KpN / 32) + it.k0 / 32) * 64 + l, h);
    } else if (jb.dstT) {  // W^T: fragment (k0 / 16 + f, n0 / 32), lane l = W[32 ks + 8 (l >> 4) + j][16 nt + (l & 15)]
        const int kk = 16 * f + (l & 15), rr = 8 * (l >> 4);
#pragma unroll
        for (int j = 0; j < 8; j++) h[j] = Tl[rr + j][kk];
        gsth8(jb.dstT + ((long)(it.k0 / 16 + f) * (jb.KpT / 32) + it.n0 / 32) * 64 + l, h);
    }
}


}  // namespace

// ------------------------------------------------------------------ host
namespace yk {

struct AmpTrain {
    int H = 0, NB = 0, Bmax = 0, RS = 0, TMAX = 0;
    AmpDev d{};
    std::vector<void*> allocs;
    long* off_dev = nullptr;
    DwJob* dw_jobs = nullptr;
    int4* dw_items = nullptr;
    int n_dw_items = 0;
    int n_dw_trunk = 0;  // items [0, n_dw_trunk): k_amp_grads; the rest (the heads'): inside k_amp_bwd
    int n_norm_dw = 0;   // the fused norm's slots of the dW blocks (k_amp_grads' 4-wave, k_amp_bwd's TW-wave)
    std::vector<int4> dw_items_host;
    std::vector<int> dw_job_rows;  // for each item: unused (all jobs span the batch)
    VsJob* vs_jobs = nullptr;
    int2* vs_items = nullptr;
    int n_vs_items = 0;
    PackJob* pk_jobs = nullptr;
    uint8_t* pk_blk = nullptr;  // per pack block: its job
    int n_pk_jobs = 0;
    long pk_total = 0;
    double* sqpart = nullptr;
    double* sq_items = nullptr;     // the fused norm's per-item partials (yk_trainer_step)
    bool norm_ready = false;        // the last backward left the total in sq_tot
    Scaler* sc = nullptr;       // the current GradScaler state
    Scaler* sc_next = nullptr;  // k_amp_update writes the next one here; the host swaps the two
    // what d.masks holds: the draws of (seed, step, row offset, p) for rows 0 .. mask_rows - 1
    bool mask_valid = false;
    uint64_t mask_seed = 0, mask_step = 0;
    int64_t mask_row_base = 0;
    float mask_p = 0.f;
    int mask_rows = 0;
    UpdJob* upd_jobs = nullptr;
    UpdItem* upd_items = nullptr;
    int n_upd_items = 0;
    const float *upd_M = nullptr, *upd_V = nullptr;  // the moment buffers the jobs were built for
    const long* off_host = nullptr;                    // (amp_create's offsets, kept for the jobs)
    std::vector<long> offs;
    float4 *win_f = nullptr, *w1f = nullptr, *w2f = nullptr, *w1t = nullptr, *w2t = nullptr, *wpif = nullptr,
           *wpit = nullptr, *wv1f = nullptr, *wv1t = nullptr;
    float* lsum_src_dummy = nullptr;
    float2* lrow = nullptr;
    float* lsum = nullptr;
};

namespace {
template <class T>
int aalloc(AmpTrain* a, T** p, size_t count) {
    void* q = nullptr;
    if (hipMalloc(&q, sizeof(T) * (count ? count : 1)) != hipSuccess) {
        (void)hipGetLastError();
        return YK_ERR_NOMEM;
    }
    a->allocs.push_back(q);
    *p = static_cast<T*>(q);
    return YK_OK;
}
}  // namespace

int amp_create(AmpTrain** out, int H, int NB, int Bmax, float* P, float* G, const long* off, float init_scale,
               int growth_interval) {
    if (!(H == 64 || H == 128 || H == 256 || H == 512)) return YK_ERR_ARG;
    AmpTrain* a = new AmpTrain();
    a->H = H;
    a->NB = NB;
    a->Bmax = Bmax;
    a->RS = (Bmax + 31) / 32;
    a->TMAX = (Bmax + TRV - 1) / TRV;  // (>= the heads' 16-row tiles: dbpi_part shares the size)
    AmpDev& d = a->d;
    d.H = H;
    d.NB = NB;
    d.Bmax = Bmax;
    d.RS = a->RS;
    d.TMAX = a->TMAX;
    d.NVEC = CV_BLK + 6 * NB;
    d.P = P;
    d.G = G;
    const int ntens = 14 + 8 * NB;
    const size_t HH = (size_t)H * H, RS = (size_t)a->RS, Bm = (size_t)Bmax, T = (size_t)a->TMAX;
    const size_t tlH = (size_t)(H / 16) * RS * 512;  // halves of one T-layout [32 RS][H] matrix
    int rc = YK_OK;
#define AA(p, n) \
    if (rc == YK_OK) rc = aalloc(a, &(p), (n))
    AA(a->off_dev, (size_t)ntens);
    // fp16 weight fragments (float4 = 8 halves)
    float4 *win_f = nullptr, *w1f = nullptr, *w2f = nullptr, *w1t = nullptr, *w2t = nullptr, *wpif = nullptr,
           *wpit = nullptr, *wv1f = nullptr, *wv1t = nullptr;
    AA(win_f, (size_t)H * 64 / 8);
    AA(w1f, NB * HH / 8 + 1);
    AA(w2f, NB * HH / 8 + 1);
    AA(w1t, NB * HH / 8 + 1);
    AA(w2t, NB * HH / 8 + 1);
    AA(wpif, (size_t)LDL * H / 8);
    AA(wpit, (size_t)LDL * H / 8);
    AA(wv1f, (size_t)VH * H / 8);
    AA(wv1t, (size_t)VH * H / 8);
    d.win_f = win_f; d.w1f = w1f; d.w2f = w2f; d.w1t = w1t; d.w2t = w2t;
    d.wpif = wpif; d.wpit = wpit; d.wv1f = wv1f; d.wv1t = wv1t;
    a->win_f = win_f; a->w1f = w1f; a->w2f = w2f; a->w1t = w1t; a->w2t = w2t;
    a->wpif = wpif; a->wpit = wpit; a->wv1f = wv1f; a->wv1t = wv1t;
    AA(d.xT, (size_t)4 * RS * 512);
    AA(d.hT, NB * tlH + 1);
    AA(d.r1T, NB * tlH + 1);
    AA(d.apiT, tlH);
    AA(d.avT, tlH);
    AA(d.api_rm, Bm * H);
    AA(d.av_rm, Bm * H);
    AA(d.z0, Bm * H);
    AA(d.u1, NB * Bm * H + 1);
    AA(d.u2, NB * Bm * H + 1);
    AA(d.hF, Bm * H);
    AA(d.stats, (size_t)(2 + 2 * NB) * 2 * Bm);
    AA(d.logits, Bm * LDL);
    AA(d.zv1, Bm * VH);
    AA(d.mlq, (size_t)HQ * Bm);
    AA(d.masks, (size_t)(1 + NB) * Bm * (H / 4));
    AA(d.dz1_rm, Bm * VH);
    AA(d.dz1T, (size_t)(VH / 16) * RS * 512);
    AA(d.dlT, (size_t)PT * RS * 512);
    AA(d.dz0T, tlH);
    AA(d.du1T, NB * tlH + 1);
    AA(d.du2T, NB * tlH + 1);
    AA(d.dz1f, Bm * VH);
    AA(d.v2prod, Bm * VH);
    AA(d.dzv2, Bm);
    AA(d.dpart, (size_t)BQ * Bm * H);
    AA(d.dbpi_part, T * LDL);
    AA(d.colpart, T * d.NVEC * H);
    AA(a->sqpart, (size_t)SQ_BLOCKS);
    AA(a->sc, 1);
    AA(a->sc_next, 1);
    if (rc != YK_OK) {
        amp_destroy(a);
        return rc;
    }
    for (int k = 0; k < ntens; k++)  // the kernels' closed-form offsets are the trainer's
        if (poff(H, NB, k) != off[k]) {
            amp_destroy(a);
            return YK_ERR_ARG;
        }
    d.off = a->off_dev;
    d.sc = a->sc;
    std::vector<long> offv(off, off + ntens);
    a->offs = offv;
    YK_HIP(hipMemcpy(a->off_dev, offv.data(), sizeof(long) * ntens, hipMemcpyHostToDevice));
    Scaler s0{init_scale > 0.f ? init_scale : 65536.0f, 0, 0, 0, growth_interval > 0 ? growth_interval : 2000};
    YK_HIP(hipMemcpy(a->sc, &s0, sizeof(Scaler), hipMemcpyHostToDevice));
    // weight-gradient jobs: (dU T layout, X T layout, gradient, N, K)
    std::vector<DwJob> jobs;
    auto tl4 = [](const _Float16* p) { return reinterpret_cast<const float4*>(p); };
    jobs.push_back({tl4(d.dz0T), tl4(d.xT), G + off[T_WIN], H, FEAT});
    for (int b = 0; b < NB; b++) {
        jobs.push_back({tl4(d.du1T + b * tlH), tl4(d.hT + b * tlH), G + off[t_blk(b, 0)], H, H});
        jobs.push_back({tl4(d.du2T + b * tlH), tl4(d.r1T + b * tlH), G + off[t_blk(b, 4)], H, H});
    }
    jobs.push_back({tl4(d.dlT), tl4(d.apiT), G + off[t_head(NB, HP_W)], ASIZE, H});
    jobs.push_back({tl4(d.dz1T), tl4(d.avT), G + off[t_head(NB, HV_W1)], VH, H});
    // a workgroup's four waves take four consecutive row tiles of the same 64 columns, so they read
    // the same X slices together (one fetch from L2 for the four) - the policy head's dW (3226 x 256)
    // re-read its 256 KB X once per 16-row tile before (202 x)
    std::vector<int4> items;
    for (size_t j = 0; j < jobs.size(); j++) {
        const int ntn = (jobs[j].N + 15) / 16, ntk = (jobs[j].K + 15) / 16;
        const int kg = (int)j < 1 + 2 * NB ? YK_DW_KG : 4;  // (k tiles per item: the trunk's fill more SIMDs with fewer)
        for (int k0 = 0; k0 < ntk; k0 += kg)
            for (int nt = 0; nt < ntn; nt++) items.push_back(make_int4((int)j, nt, k0, std::min(kg, ntk - k0)));
    }
    a->n_dw_items = (int)items.size();
    for (const int4& it : items)  // (k_amp_grads runs the trunk's items as YK_DW_KG-tile items)
        if (it.x < 1 + 2 * NB && it.w != YK_DW_KG) {
            amp_destroy(a);
            return YK_ERR_ARG;
        }
    a->n_dw_trunk = 0;  // the items of the input layer's and the blocks' matrices come first
    while (a->n_dw_trunk < a->n_dw_items && items[a->n_dw_trunk].x < 1 + 2 * NB) a->n_dw_trunk++;
    a->n_norm_dw = (a->n_dw_trunk + DW_IPB - 1) / DW_IPB + (a->n_dw_items - a->n_dw_trunk + TW - 1) / TW;
    // column-sum jobs: bias / LayerNorm gradients and the two loss sums
    std::vector<VsJob> vj;
    const int ldc = d.NVEC * H;
    auto colv = [&](int v) { return d.colpart + (size_t)v * H; };
    vj.push_back({colv(CV_BIN), G + off[T_BIN], ldc, H, 0, 1, 1});
    vj.push_back({colv(CV_GIN), G + off[T_GIN], ldc, H, 0, 0, 1});
    vj.push_back({colv(CV_BEIN), G + off[T_BEIN], ldc, H, 0, 0, 1});
    for (int b = 0; b < NB; b++) {
        const int vb = CV_BLK + 6 * b;
        vj.push_back({colv(vb + 0), G + off[t_blk(b, 1)], ldc, H, 0, 1, 1});
        vj.push_back({colv(vb + 1), G + off[t_blk(b, 2)], ldc, H, 0, 0, 1});
        vj.push_back({colv(vb + 2), G + off[t_blk(b, 3)], ldc, H, 0, 0, 1});
        vj.push_back({colv(vb + 3), G + off[t_blk(b, 5)], ldc, H, 0, 1, 1});
        vj.push_back({colv(vb + 4), G + off[t_blk(b, 6)], ldc, H, 0, 0, 1});
        vj.push_back({colv(vb + 5), G + off[t_blk(b, 7)], ldc, H, 0, 0, 1});
    }
    vj.push_back({colv(CV_GPI), G + off[t_head(NB, HP_G)], ldc, H, 0, 0, 1});
    vj.push_back({colv(CV_BEPI), G + off[t_head(NB, HP_B)], ldc, H, 0, 0, 1});
    vj.push_back({colv(CV_GV), G + off[t_head(NB, HV_G)], ldc, H, 0, 0, 1});
    vj.push_back({colv(CV_BEV), G + off[t_head(NB, HV_B)], ldc, H, 0, 0, 1});
    vj.push_back({d.dbpi_part, G + off[t_head(NB, HP_BIAS)], LDL, ASIZE, 2, 1, 1});
    vj.push_back({d.dz1f, G + off[t_head(NB, HV_B1)], VH, VH, 1, 1, 1});
    vj.push_back({d.v2prod, G + off[t_head(NB, HV_W2)], VH, VH, 1, 1, 1});
    vj.push_back({d.dzv2, G + off[t_head(NB, HV_B2)], 1, 1, 1, 1, 1});
    const size_t loss_job = vj.size();  // (the trainer's lrow / lsum: filled in per call)
    vj.push_back({nullptr, nullptr, 2, 2, 1, 0, 0});
    std::vector<int2> vitems;
    for (size_t j = 0; j < vj.size(); j++)
        for (int c = 0; c < vj[j].N; c += 16) vitems.push_back(make_int2((int)j, c));
    a->n_vs_items = (int)vitems.size();
    // fp16 pack jobs
    std::vector<PackJob> pj;
    long first = 0;
    auto pack = [&](const float* W, float4* dst, int N, int K, int Np, int Kp, int trans) {
        pj.push_back({W, dst, N, K, Np, Kp, trans, first});
        first += (long)Np * Kp / 8;
    };
    pack(P + off[T_WIN], win_f, H, FEAT, H, 64, 0);
    for (int b = 0; b < NB; b++) {
        pack(P + off[t_blk(b, 0)], w1f + b * HH / 8, H, H, H, H, 0);
        pack(P + off[t_blk(b, 4)], w2f + b * HH / 8, H, H, H, H, 0);
        pack(P + off[t_blk(b, 0)], w1t + b * HH / 8, H, H, H, H, 1);
        pack(P + off[t_blk(b, 4)], w2t + b * HH / 8, H, H, H, H, 1);
    }
    pack(P + off[t_head(NB, HP_W)], wpif, ASIZE, H, LDL, H, 0);
    pack(P + off[t_head(NB, HP_W)], wpit, ASIZE, H, H, LDL, 1);
    pack(P + off[t_head(NB, HV_W1)], wv1f, VH, H, VH, H, 0);
    pack(P + off[t_head(NB, HV_W1)], wv1t, VH, H, H, VH, 1);
    a->n_pk_jobs = (int)pj.size();
    a->pk_total = first;
    std::vector<uint8_t> pblk;
    for (size_t j = 0; j < pj.size(); j++) {
        const long n = (j + 1 < pj.size() ? pj[j + 1].first : first) - pj[j].first;
        if (n % 256 != 0 || pj.size() > 255) {  // a block would straddle two jobs
            amp_destroy(a);
            return YK_ERR_ARG;
        }
        pblk.insert(pblk.end(), (size_t)(n / 256), (uint8_t)j);
    }
    if (aalloc(a, &a->dw_jobs, jobs.size()) || aalloc(a, &a->dw_items, items.size()) ||
        aalloc(a, &a->vs_jobs, vj.size()) || aalloc(a, &a->vs_items, vitems.size()) ||
        aalloc(a, &a->pk_jobs, pj.size()) || aalloc(a, &a->pk_blk, pblk.size()) ||
        aalloc(a, &a->sq_items, (size_t)(a->n_dw_items + a->n_vs_items))) {  // (>= the blocks')
        amp_destroy(a);
        return YK_ERR_NOMEM;
    }
    YK_HIP(hipMemcpy(a->dw_jobs, jobs.data(), sizeof(DwJob) * jobs.size(), hipMemcpyHostToDevice));
    YK_HIP(hipMemcpy(a->dw_items, items.data(), sizeof(int4) * items.size(), hipMemcpyHostToDevice));
    YK_HIP(hipMemcpy(a->vs_items, vitems.data(), sizeof(int2) * vitems.size(), hipMemcpyHostToDevice));
    YK_HIP(hipMemcpy(a->pk_jobs, pj.data(), sizeof(PackJob) * pj.size(), hipMemcpyHostToDevice));
    YK_HIP(hipMemcpy(a->pk_blk, pblk.data(), pblk.size(), hipMemcpyHostToDevice));
    // the loss-sum job's buffers are the trainer's; amp_backward patches them in on first use
    YK_HIP(hipMemcpy(a->vs_jobs, vj.data(), sizeof(VsJob) * vj.size(), hipMemcpyHostToDevice));
    a->lsum_src_dummy = nullptr;
    (void)loss_job;
    *out = a;
    return YK_OK;
}

void amp_destroy(AmpTrain* a) {
    if (!a) return;
    for (void* p : a->allocs) (void)hipFree(p);
    delete a;
}

int amp_pack(AmpTrain* a, hipStream_t s) {
    hipLaunchKernelGGL(k_amp_pack, dim3((unsigned)((a->pk_total + 255) / 256)), dim3(256), 0, s, a->pk_jobs,
                       a->pk_blk, a->pk_total);
    YK_LAUNCHED();
    return YK_OK;
}

int amp_backward(AmpTrain* a, const yk_state_t* states, const int32_t* targets, const float* values,
                 const int32_t* idx, int B, float dropout, uint64_t seed, uint64_t step, int64_t row_base,
                 float vloss_weight, float2* lrow, float* lsum, bool fuse_norm, hipStream_t s) {
    if (B <= 0 || B > a->Bmax) return YK_ERR_ARG;
    a->norm_ready = false;
    double* sqp = fuse_norm ? a->sq_items : nullptr;
    AmpDev& d = a->d;
    if (a->lrow != lrow || a->lsum != lsum) {  // the loss-sum job reads the trainer's row losses
        const int j = 3 + 6 * a->NB + 4 + 4;
        VsJob jb{reinterpret_cast<const float*>(lrow), lsum, 2, 2, 1, 0, 0};
        YK_HIP(hipMemcpy(a->vs_jobs + j, &jb, sizeof(VsJob), hipMemcpyHostToDevice));
        a->lrow = lrow;
        a->lsum = lsum;
    }
    // T: the heads' 16-row tiles; TT: the trunk's TRV-row workgroups
    const int T = (B + TR - 1) / TR, TT = (B + TRV - 1) / TRV, rsn = (B + 31) / 32;
    if (dropout > 0.f && !(a->mask_valid && a->mask_seed == seed && a->mask_step == step && a->mask_row_base == row_base &&
                           a->mask_p == dropout && a->mask_rows >= B)) {  // (not made ahead by the last update)
        const long nm = (long)(1 + a->NB) * B * (a->H / 4);
        hipLaunchKernelGGL(k_amp_masks, dim3((unsigned)((nm + 255) / 256)), dim3(256), 0, s, d, B, dropout, seed, step,
                           row_base);
        YK_LAUNCHED();
    }
    a->mask_valid = false;  // consumed by this step: the next update writes the next step's
    switch (a->H) {
#define YK_AMP_FWD(HH)                                                                                              \
    case HH:                                                                                                        \
        hipLaunchKernelGGL(k_amp_fwd<HH>, dim3(TT), dim3(TTHR), 0, s, d, states, idx, B, dropout, seed, step, row_base); \
        YK_LAUNCHED();                                                                                              \
        hipLaunchKernelGGL(k_amp_head<HH>, dim3(T, HQ + 1), dim3(TTHR), 0, s, d, B);                               \
        YK_LAUNCHED();                                                                                              \
        hipLaunchKernelGGL(k_amp_headbwd<HH>, dim3(T, BQ + 1), dim3(TTHR), 0, s, d, targets, values, idx, B,       \
                           vloss_weight, lrow);                                                                     \
        YK_LAUNCHED();                                                                                              \
        hipLaunchKernelGGL(k_amp_bwd<HH>, dim3(TT + (a->n_dw_items - a->n_dw_trunk + TW - 1) / TW), dim3(TTHR), 0, s, \
                           d, B, dropout, seed, step, row_base, a->dw_jobs, a->dw_items + a->n_dw_trunk,          \
                           a->n_dw_items - a->n_dw_trunk, rsn, sqp, (a->n_dw_trunk + DW_IPB - 1) / DW_IPB);        \
        YK_LAUNCHED();                                                                                              \
        break;
        YK_AMP_FWD(64)
        YK_AMP_FWD(128)
        YK_AMP_FWD(256)
        YK_AMP_FWD(512)
#undef YK_AMP_FWD
        default: return YK_ERR_ARG;
    }
    hipLaunchKernelGGL(k_amp_grads, dim3((unsigned)((a->n_dw_trunk + DW_IPB - 1) / DW_IPB + a->n_vs_items)), dim3(256), 0, s,
                       a->dw_jobs, a->dw_items, a->n_dw_trunk, a->RS, rsn, a->vs_jobs, a->vs_items, a->n_vs_items, TT, T,
                       B, sqp, a->n_norm_dw, a->sc);
    YK_LAUNCHED();
    a->norm_ready = fuse_norm;
    return YK_OK;
}

// k_amp_update's work list: a 32 x 32 tile of every packed weight matrix, and 1024-element slices
// of the parameters no matrix covers
static int build_update_jobs(AmpTrain* a, long nparams, float* M, float* V) {
    const int H = a->H, NB = a->NB;
    const long* off = a->offs.data();
    const size_t HH = (size_t)H * H;
    float* P = const_cast<float*>(a->d.P);
    float* G = a->d.G;
    std::vector<UpdJob> jobs;
    std::vector<UpdItem> items;
    std::vector<std::pair<long, long>> mats;
    auto mat = [&](long o, int N, int K, float4* dN, int KpN, float4* dT, int KpT) {
        const int j = (int)jobs.size();
        jobs.push_back({P + o, G + o, M + o, V + o, dN, dT, N, K, KpN, KpT});
        for (int n0 = 0; n0 < N; n0 += 32)
            for (int k0 = 0; k0 < K; k0 += 32) items.push_back({j, n0, k0});
        mats.push_back({o, o + (long)N * K});
    };
    mat(off[T_WIN], H, FEAT, a->win_f, 64, nullptr, 0);
    for (int b = 0; b < NB; b++) {
        mat(off[t_blk(b, 0)], H, H, a->w1f + b * HH / 8, H, a->w1t + b * HH / 8, H);
        mat(off[t_blk(b, 4)], H, H, a->w2f + b * HH / 8, H, a->w2t + b * HH / 8, H);
    }
    mat(off[t_head(NB, HP_W)], ASIZE, H, a->wpif, H, a->wpit, LDL);
    mat(off[t_head(NB, HV_W1)], VH, H, a->wv1f, H, a->wv1t, VH);
    std::sort(mats.begin(), mats.end());
    const int jv = (int)jobs.size();
    jobs.push_back({P, G, M, V, nullptr, nullptr, 0, 0, 0, 0});
    long pos = 0;
    mats.push_back({nparams, nparams});
    for (const auto& m : mats) {
        for (long e = pos; e < m.first; e += 1024) items.push_back({jv, (int)e, (int)std::min<long>(1024, m.first - e)});
        pos = std::max(pos, m.second);
    }
    if (!a->upd_jobs && (aalloc(a, &a->upd_jobs, jobs.size()) || aalloc(a, &a->upd_items, items.size())))
        return YK_ERR_NOMEM;
    YK_HIP(hipMemcpy(a->upd_jobs, jobs.data(), sizeof(UpdJob) * jobs.size(), hipMemcpyHostToDevice));
    YK_HIP(hipMemcpy(a->upd_items, items.data(), sizeof(UpdItem) * items.size(), hipMemcpyHostToDevice));
    a->n_upd_items = (int)items.size();
    a->upd_M = M;
    a->upd_V = V;
    return YK_OK;
}

int amp_apply(AmpTrain* a, long nparams, float* M, float* V, double* sq_out, float max_norm, float lr, float wd,
              float b1, float b2, float eps, float dropout, uint64_t seed, uint64_t next_step, hipStream_t s) {
    if (a->upd_M != M || a->upd_V != V) {  // the update jobs address the trainer's moment buffers
        const int rc = build_update_jobs(a, nparams, M, V);
        if (rc != YK_OK) return rc;
    }
    const bool fused = a->norm_ready;  // (yk_trainer_step: k_amp_grads summed the norm; no all-reduce between)
    a->norm_ready = false;
    if (!fused) {
        hipLaunchKernelGGL(k_amp_sq, dim3(SQ_BLOCKS), dim3(256), 0, s, a->d.G, nparams, a->sc, a->sqpart);
        YK_LAUNCHED();
    }
    const long nm = dropout > 0.f ? (long)(1 + a->NB) * a->Bmax * (a->H / 4) : 0;
    hipLaunchKernelGGL(k_amp_update, dim3((unsigned)(a->n_upd_items + (nm + 255) / 256)), dim3(256), 0, s, a->upd_jobs,
                       a->upd_items, fused ? a->sq_items : a->sqpart, sq_out, a->sc, a->sc_next, max_norm, lr, wd, b1, b2, eps, a->n_upd_items,
                       a->d, dropout, seed, next_step, fused ? a->n_norm_dw + a->n_vs_items : SQ_BLOCKS);
    YK_LAUNCHED();
    a->mask_valid = nm > 0;
    a->mask_seed = seed;
    a->mask_step = next_step;
    a->mask_row_base = 0;
    a->mask_p = dropout;
    a->mask_rows = a->Bmax;
    std::swap(a->sc, a->sc_next);  // the next launches read the updated GradScaler state
    a->d.sc = a->sc;
    return YK_OK;
}

int amp_state(AmpTrain* a, double* out) {
    Scaler sc;
    YK_HIP(hipDeviceSynchronize());
    YK_HIP(hipMemcpy(&sc, a->sc, sizeof(Scaler), hipMemcpyDeviceToHost));
    out[0] = sc.scale;
    out[1] = sc.tracker;
    out[2] = (double)sc.steps;
    out[3] = sc.found_inf;
    return YK_OK;
}

int64_t amp_steps(AmpTrain* a) {
    Scaler sc;
    if (hipDeviceSynchronize() != hipSuccess) return YK_ERR_HIP;
    if (hipMemcpy(&sc, a->sc, sizeof(Scaler), hipMemcpyDeviceToHost) != hipSuccess) return YK_ERR_HIP;
    return sc.steps;
}

int amp_set_steps(AmpTrain* a, int64_t steps) {
    Scaler sc;
    YK_HIP(hipDeviceSynchronize());
    YK_HIP(hipMemcpy(&sc, a->sc, sizeof(Scaler), hipMemcpyDeviceToHost));
    sc.steps = steps;
    YK_HIP(hipMemcpy(a->sc, &sc, sizeof(Scaler), hipMemcpyHostToDevice));
    return YK_OK;
}

}  // namespace yk
