// yk_net.hip - NNetWrapper.predict (yacht/NNet.py:177-195) over YachtNNet
// (yacht/pytorch/YachtNNet.py:8-70), batched over all pending leaves, float32.
//
// One kernel, k_forward, carries all 3,320,576 FLOP per row (hidden 256, 6 blocks): a
// 1024-thread workgroup (16 waves, 4 per SIMD) owns 16 rows and keeps their activations in
// LDS through featurize -> Linear/LN/SiLU -> 6 x ResidualBlock -> head LayerNorms ->
// policy logits (204 x 16 columns) and the value head.  Every dense layer runs on
// v_mfma_f32_16x16x4_f32 (exact f32: fmaf chains), so results track torch's float32 CPU
// path within the north star's 1e-5 (tests/test_gpu_net.py).  Weights are pre-packed in
// MFMA fragment order (yk_net.h) so each wave streams them as contiguous 1 KB loads, and
// the next layer's slice is issued before the LayerNorm phase so it flies under it.
#include <vector>

#include "yk_api.h"
#include "yk_common.h"
#include "yk_net.h"

using namespace yk;

typedef float floatx4 __attribute__((ext_vector_type(4)));

// Diagnostic builds only (tools/trunk_ablate.cpp): 2 = no MFMA, 3 = no weight loads.
#ifndef YK_ABL
#define YK_ABL 0
#endif

namespace {

constexpr int ROWS = 16;  // rows per workgroup
constexpr int FPAD = 68;  // feature tile row stride (64 + 4)
constexpr int PCH = 4;    // policy-head tiles per chunk (accumulators in flight per wave)

__device__ __forceinline__ float silu(float x) { return x / (1.0f + expf(-x)); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops, NOT for its
// outstanding global loads (a __syncthreads() would drain vmcnt and expose the weight
// stream's latency at every layer).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ float4 ld_frag(const float* __restrict__ P, int KB, int nt, int kb, int lane) {
#if YK_ABL == 3
    return make_float4(1e-3f * kb, 1e-3f * nt, 2e-3f, 3e-3f + P[0] * 0.f);
#else
    return *reinterpret_cast<const float4*>(P + ((long)(nt * KB + kb) * 64 + lane) * 4);
#endif
}

// A wave's weight slice for one dense layer: NT 16-column tiles starting at tile nt0, all K.
template <int K, int NT>
struct WSlice {
    float4 b[K / 16][NT];
};
template <int K, int NT>
__device__ __forceinline__ void load_w(WSlice<K, NT>& ws, const float* __restrict__ P, int nt0) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int kb = 0; kb < K / 16; kb++)
#pragma unroll
        for (int t = 0; t < NT; t++) ws.b[kb][t] = ld_frag(P, K / 16, nt0 + t, kb, lane);
    __builtin_amdgcn_sched_barrier(0);  // issue them here, ahead of the work that hides them
}

// acc[t] = A[16 x K] (LDS, row stride lda) x slice^T.  Lane l supplies A[l&15][16kb + 4(l>>4) + i]
// and W[.][16kb + 4(l>>4) + i] to MFMA i of each 16-deep k-block.  Two partial accumulators
// keep consecutive MFMAs independent (40-cycle dependent latency vs 32-cycle issue).
template <int K, int NT>
__device__ __forceinline__ void mma16(const float* A, int lda, const WSlice<K, NT>& ws, floatx4 (&acc)[NT]) {
    const int lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
    floatx4 acc2[NT];
#pragma unroll
    for (int t = 0; t < NT; t++) acc[t] = acc2[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    const float* ap = A + r * lda + 4 * q;
#if YK_ABL == 2
    acc[0][0] = ap[0] + ws.b[0][0].x;
    return;
#endif
#pragma unroll
    for (int kb = 0; kb < K / 16; kb++) {
        const float4 a = *reinterpret_cast<const float4*>(ap + 16 * kb);
#pragma unroll
        for (int t = 0; t < NT; t++) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, ws.b[kb][t].x, acc[t], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < NT; t++) acc2[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, ws.b[kb][t].y, acc2[t], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < NT; t++) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, ws.b[kb][t].z, acc[t], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < NT; t++) acc2[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, ws.b[kb][t].w, acc2[t], 0, 0, 0);
    }
#pragma unroll
    for (int t = 0; t < NT; t++) acc[t] += acc2[t];
}

// D[16 x 16] tile t of the wave: lane holds rows 4(l>>4)+j, column 16(nt0 + t) + (l&15)
template <int NT>
__device__ __forceinline__ void store_acc(float* D, int ldd, int nt0, const floatx4 (&acc)[NT],
                                          const float* __restrict__ bias) {
    const int lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
#pragma unroll
    for (int t = 0; t < NT; t++) {
        const int c = 16 * (nt0 + t) + r;
        const float b = bias[c];
#pragma unroll
        for (int j = 0; j < 4; j++) D[(4 * q + j) * ldd + c] = acc[t][j] + b;
    }
}

// nn.LayerNorm over H values held VPL per lane (two-pass, biased variance, eps 1e-5)
template <int VPL>
__device__ __forceinline__ void layernorm(float (&x)[VPL], const float* __restrict__ g, const float* __restrict__ b,
                                          int c0, int H) {
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

// Dense layers: wave w owns output tiles [NT w, NT (w+1)); row passes (LayerNorm / SiLU /
// residual): wave w owns row w; policy head: wave w owns tiles w, w + 16, w + 32, ...
template <int H>
__global__ __launch_bounds__(1024) void k_forward(NetDev net, const yk_state_t* __restrict__ states,
                                                 const float* __restrict__ xin, const int32_t* __restrict__ rows,
                                                 const int32_t* __restrict__ count, int n,
                                                 float* __restrict__ logits, float* __restrict__ vout) {
    constexpr int LD = (H > 128 ? H : 128) + 4;  // X also holds the 128-wide v_head hidden
    constexpr int NT = H >= 256 ? H / 256 : 1;    // 16-col tiles per wave in H-wide layers
    constexpr int NACT = H / (16 * NT);           // waves with columns of the H-wide layers
    constexpr int VPL = H / 64;                   // values per lane in row passes
    constexpr int KB = H / 16;
    __shared__ __attribute__((aligned(16))) float X[ROWS * LD];
    __shared__ __attribute__((aligned(16))) float T[ROWS * LD];
    __shared__ __attribute__((aligned(16))) float F[ROWS * FPAD];

    if (count) n = min(n, *count);
    const int row0 = blockIdx.x * ROWS;
    if (row0 >= n) return;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const bool gw = wave < NACT;           // owns columns of the H-wide layers
    const bool vw = wave * 16 * NT < 128;  // owns columns of v_head.2
    const int nt0 = wave * NT;
    const int r = wave;  // row of the row passes
    const int c0 = lane * VPL;

    // featurize (state_to_vec, NNet.py:65-86), zero padded to K = 64: one value per thread
    {
        const int rr = tid >> 6, f = tid & 63;
        const int row = row0 + rr;
        float val = 0.f;
        if (row < n && f < FEAT) {
            const int src = rows ? rows[row] : row;
            if (xin) {
                val = xin[(long)src * FEAT + f];
            } else {
                const uint4* p = reinterpret_cast<const uint4*>(states + src);
                YkS s;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    uint4 u = p[k];
                    s.w[2 * k] = (uint64_t)u.x | ((uint64_t)u.y << 32);
                    s.w[2 * k + 1] = (uint64_t)u.z | ((uint64_t)u.w << 32);
                }
                val = feature(s, f);
            }
        }
        F[rr * FPAD + f] = val;
    }
    lds_barrier();

    floatx4 acc[NT];
    WSlice<H, NT> ws;  // next dense layer's weights, in flight during the row passes
    // inp: Linear -> LayerNorm -> SiLU (-> Dropout, identity in eval)  YachtNNet.py:30-35
    if (gw) {
        WSlice<64, NT> w0;
        load_w<64, NT>(w0, net.w_in, nt0);
        if (net.NB > 0) load_w<H, NT>(ws, net.w1, nt0);
        mma16<64, NT>(F, FPAD, w0, acc);
        store_acc<NT>(T, LD, nt0, acc, net.b_in);
    }
    lds_barrier();
    {
        float x[VPL];
#pragma unroll
        for (int i = 0; i < VPL; i++) x[i] = T[r * LD + c0 + i];
        layernorm<VPL>(x, net.g_in, net.be_in, c0, H);
#pragma unroll
        for (int i = 0; i < VPL; i++) X[r * LD + c0 + i] = silu(x[i]);
    }
    lds_barrier();

    // ResidualBlock x NB: h = LN1(SiLU(fc1 x)); h = LN2(SiLU(fc2 h)); x + h  YachtNNet.py:17-21
    for (int b = 0; b < net.NB; b++) {
        const long wo = (long)b * H * H, bo = (long)b * H;
        if (gw) {
            mma16<H, NT>(X, LD, ws, acc);
            load_w<H, NT>(ws, net.w2 + wo, nt0);  // fc2 weights fly during LN1
            store_acc<NT>(T, LD, nt0, acc, net.b1 + bo);
        }
        lds_barrier();
        {
            float x[VPL];
#pragma unroll
            for (int i = 0; i < VPL; i++) x[i] = silu(T[r * LD + c0 + i]);
            layernorm<VPL>(x, net.g1 + bo, net.be1 + bo, c0, H);
#pragma unroll
            for (int i = 0; i < VPL; i++) T[r * LD + c0 + i] = x[i];
        }
        lds_barrier();
        if (gw) mma16<H, NT>(T, LD, ws, acc);
        if (b + 1 < net.NB) {
            if (gw) load_w<H, NT>(ws, net.w1 + wo + (long)H * H, nt0);  // next fc1
        } else if (vw) {
            load_w<H, NT>(ws, net.w_v1, nt0);  // v_head.2
        }
        lds_barrier();
        if (gw) store_acc<NT>(T, LD, nt0, acc, net.b2 + bo);
        lds_barrier();
        {
            float x[VPL];
#pragma unroll
            for (int i = 0; i < VPL; i++) x[i] = silu(T[r * LD + c0 + i]);
            layernorm<VPL>(x, net.g2 + bo, net.be2 + bo, c0, H);
#pragma unroll
            for (int i = 0; i < VPL; i++) X[r * LD + c0 + i] += x[i];
        }
        lds_barrier();
    }

    // heads: pi_head = LN -> SiLU -> Linear; v_head = LN -> SiLU -> Linear -> SiLU -> Linear -> tanh
    {
        float x[VPL], y[VPL];
#pragma unroll
        for (int i = 0; i < VPL; i++) x[i] = y[i] = X[r * LD + c0 + i];
        layernorm<VPL>(x, net.g_pi, net.be_pi, c0, H);
        layernorm<VPL>(y, net.g_v, net.be_v, c0, H);
#pragma unroll
        for (int i = 0; i < VPL; i++) {
            X[r * LD + c0 + i] = silu(x[i]);  // a_pi (each wave rewrites only its own row)
            T[r * LD + c0 + i] = silu(y[i]);  // a_v
        }
    }
    lds_barrier();
    floatx4 av[NT];
    if (vw) {  // v_head.2: Linear(H, 128) (weights already in flight)
        if (net.NB == 0) load_w<H, NT>(ws, net.w_v1, nt0);
        mma16<H, NT>(T, LD, ws, av);
    }
    // policy head (pi_head.2): 204 tiles of 16 columns over the 16 waves, PCH at a time,
    // with the next k-block's weight fragments in flight
    for (int c = 0; c * 16 * PCH < PI_TILES; c++) {
        floatx4 pa[PCH];
        float4 wb[2][PCH];
        const int tbase = wave + 16 * PCH * c;  // tile of slot t: tbase + 16 t (wave-uniform)
        const int ntile = min(PCH, (PI_TILES - tbase + 15) / 16);
        if (ntile <= 0) break;
#pragma unroll
        for (int t = 0; t < PCH; t++) {
            pa[t] = floatx4{0.f, 0.f, 0.f, 0.f};
            if (t < ntile) wb[0][t] = ld_frag(net.w_pi, KB, tbase + 16 * t, 0, lane);
        }
        const float* ap = X + (lane & 15) * LD + 4 * (lane >> 4);
#pragma unroll
        for (int kb = 0; kb < KB; kb++) {
            if (kb + 1 < KB) {
#pragma unroll
                for (int t = 0; t < PCH; t++)
                    if (t < ntile) wb[(kb + 1) & 1][t] = ld_frag(net.w_pi, KB, tbase + 16 * t, kb + 1, lane);
            }
            const float4 a = *reinterpret_cast<const float4*>(ap + 16 * kb);
            const int cb = kb & 1;
#if YK_ABL != 2
            if (ntile == PCH) {
#pragma unroll
                for (int t = 0; t < PCH; t++) pa[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, wb[cb][t].x, pa[t], 0, 0, 0);
#pragma unroll
                for (int t = 0; t < PCH; t++) pa[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, wb[cb][t].y, pa[t], 0, 0, 0);
#pragma unroll
                for (int t = 0; t < PCH; t++) pa[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, wb[cb][t].z, pa[t], 0, 0, 0);
#pragma unroll
                for (int t = 0; t < PCH; t++) pa[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, wb[cb][t].w, pa[t], 0, 0, 0);
            } else {
#pragma unroll
                for (int t = 0; t < PCH; t++)
                    if (t < ntile) {
                        pa[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, wb[cb][t].x, pa[t], 0, 0, 0);
                        pa[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, wb[cb][t].y, pa[t], 0, 0, 0);
                        pa[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, wb[cb][t].z, pa[t], 0, 0, 0);
                        pa[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, wb[cb][t].w, pa[t], 0, 0, 0);
                    }
            }
#else
            pa[0][0] += a.x + wb[cb][0].x;
#endif
        }
        const int rr = lane & 15, q = lane >> 4;
#pragma unroll
        for (int t = 0; t < PCH; t++) {
            if (t < ntile) {
                const int col = 16 * (tbase + 16 * t) + rr;
                const float bias = net.b_pi[col];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int row = row0 + 4 * q + j;
                    if (row < n) logits[(long)row * PI_LD + col] = pa[t][j] + bias;
                }
            }
        }
    }
    lds_barrier();  // every wave is done reading a_pi (X)
    if (vw) store_acc<NT>(X, LD, nt0, av, net.b_v1);
    lds_barrier();
    {  // SiLU -> Linear(128, 1) -> tanh  YachtNNet.py:49-52,69
        const int row = row0 + r;
        float s = silu(X[r * LD + 2 * lane]) * net.w_v2[2 * lane] + silu(X[r * LD + 2 * lane + 1]) * net.w_v2[2 * lane + 1];
        s = wave_sum(s);
        if (lane == 0 && row < n) vout[row] = tanhf(s + net.b_v2[0]);
    }
}

// exp(log_softmax(x)) over the first 3226 columns; one wavefront per row
__global__ void k_softmax(const float* __restrict__ logits, float* __restrict__ pi, int n) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= n) return;
    const float* x = logits + (long)row * PI_LD;
    float m = -INFINITY;
    for (int a = lane; a < ASIZE; a += 64) m = fmaxf(m, x[a]);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    float s = 0.f;
    for (int a = lane; a < ASIZE; a += 64) s += expf(x[a] - m);
    const float lse = logf(wave_sum(s));
    for (int a = lane; a < ASIZE; a += 64) pi[(long)row * ASIZE + a] = expf(x[a] - m - lse);
}

}  // namespace

namespace yk {

int launch_forward(const NetDev& net, const yk_state_t* states, const float* x, const int32_t* rows,
                   const int32_t* count, int n, float* logits, float* v, hipStream_t stream) {
    if (n <= 0) return YK_OK;
    const dim3 grid((n + ROWS - 1) / ROWS), block(1024);
    switch (net.H) {
        case 64: hipLaunchKernelGGL(k_forward<64>, grid, block, 0, stream, net, states, x, rows, count, n, logits, v); break;
        case 128: hipLaunchKernelGGL(k_forward<128>, grid, block, 0, stream, net, states, x, rows, count, n, logits, v); break;
        case 256: hipLaunchKernelGGL(k_forward<256>, grid, block, 0, stream, net, states, x, rows, count, n, logits, v); break;
        case 512: hipLaunchKernelGGL(k_forward<512>, grid, block, 0, stream, net, states, x, rows, count, n, logits, v); break;
        default: return YK_ERR_ARG;
    }
    YK_LAUNCHED();
    return YK_OK;
}

int launch_softmax(const float* logits, float* pi, int n, hipStream_t stream) {
    if (n <= 0) return YK_OK;
    hipLaunchKernelGGL(k_softmax, dim3((n + 3) / 4), dim3(256), 0, stream, logits, pi, n);
    YK_LAUNCHED();
    return YK_OK;
}

}  // namespace yk

extern "C" {

int yk_net_create(yk_net_t** out, int H, int NB, const float* const* p, int nparams) {
    if (!out || !p) return YK_ERR_ARG;
    if (!(H == 64 || H == 128 || H == 256 || H == 512) || NB < 0 || NB > 64) return YK_ERR_ARG;
    if (nparams != 14 + 8 * NB) return YK_ERR_ARG;
    // host staging of the device layout (every block 256-byte aligned)
    std::vector<float> h;
    auto put = [&](size_t n) { size_t o = h.size(); h.resize(o + ((n + 63) / 64) * 64, 0.f); return o; };
    // torch [N][K] row-major (K valid columns) -> fragment order, N padded to Np, K to Kp
    auto pack = [&](size_t dst, const float* W, int N, int K, int Np, int Kp) {
        const int KBp = Kp / 16;
        for (int nt = 0; nt < Np / 16; nt++)
            for (int kb = 0; kb < KBp; kb++)
                for (int l = 0; l < 64; l++)
                    for (int i = 0; i < 4; i++) {
                        const int nn = 16 * nt + (l & 15), kk = 16 * kb + 4 * (l >> 4) + i;
                        h[dst + (((size_t)nt * KBp + kb) * 64 + l) * 4 + i] =
                            (nn < N && kk < K) ? W[(size_t)nn * K + kk] : 0.f;
                    }
    };
    const size_t o_win = put((size_t)H * 64), o_bin = put(H), o_gin = put(H), o_bein = put(H);
    const size_t o_w1 = put((size_t)NB * H * H), o_b1 = put((size_t)NB * H), o_g1 = put((size_t)NB * H),
                 o_be1 = put((size_t)NB * H);
    const size_t o_w2 = put((size_t)NB * H * H), o_b2 = put((size_t)NB * H), o_g2 = put((size_t)NB * H),
                 o_be2 = put((size_t)NB * H);
    const size_t o_gpi = put(H), o_bepi = put(H), o_wpi = put((size_t)PI_LD * H), o_bpi = put(PI_LD);
    const size_t o_gv = put(H), o_bev = put(H), o_wv1 = put((size_t)128 * H), o_bv1 = put(128), o_wv2 = put(128),
                 o_bv2 = put(1);
    int k = 0;
    auto cp = [&](size_t off, size_t n) { std::copy(p[k], p[k] + n, h.begin() + off); k++; };
    pack(o_win, p[k++], H, FEAT, H, 64);
    cp(o_bin, H); cp(o_gin, H); cp(o_bein, H);
    for (int b = 0; b < NB; b++) {
        pack(o_w1 + (size_t)b * H * H, p[k++], H, H, H, H); cp(o_b1 + (size_t)b * H, H);
        cp(o_g1 + (size_t)b * H, H); cp(o_be1 + (size_t)b * H, H);
        pack(o_w2 + (size_t)b * H * H, p[k++], H, H, H, H); cp(o_b2 + (size_t)b * H, H);
        cp(o_g2 + (size_t)b * H, H); cp(o_be2 + (size_t)b * H, H);
    }
    cp(o_gpi, H); cp(o_bepi, H);
    pack(o_wpi, p[k++], ASIZE, H, PI_LD, H);
    cp(o_bpi, ASIZE);
    cp(o_gv, H); cp(o_bev, H);
    pack(o_wv1, p[k++], 128, H, 128, H);
    cp(o_bv1, 128); cp(o_wv2, 128); cp(o_bv2, 1);

    yk_net* net = new yk_net();
    net->bytes = h.size() * sizeof(float);
    if (hipMalloc(&net->blob, net->bytes) != hipSuccess) {
        delete net;
        return YK_ERR_NOMEM;
    }
    if (hipMemcpy(net->blob, h.data(), net->bytes, hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(net->blob);
        delete net;
        return YK_ERR_HIP;
    }
    const float* B = net->blob;
    NetDev& d = net->dev;
    d.H = H; d.NB = NB;
    d.w_in = B + o_win; d.b_in = B + o_bin; d.g_in = B + o_gin; d.be_in = B + o_bein;
    d.w1 = B + o_w1; d.b1 = B + o_b1; d.g1 = B + o_g1; d.be1 = B + o_be1;
    d.w2 = B + o_w2; d.b2 = B + o_b2; d.g2 = B + o_g2; d.be2 = B + o_be2;
    d.g_pi = B + o_gpi; d.be_pi = B + o_bepi; d.w_pi = B + o_wpi; d.b_pi = B + o_bpi;
    d.g_v = B + o_gv; d.be_v = B + o_bev; d.w_v1 = B + o_wv1; d.b_v1 = B + o_bv1; d.w_v2 = B + o_wv2; d.b_v2 = B + o_bv2;
    *out = net;
    return YK_OK;
}

int yk_net_destroy(yk_net_t* net) {
    if (!net) return YK_OK;
    (void)hipFree(net->blob);
    delete net;
    return YK_OK;
}

static int predict_common(yk_net_t* net, const yk_state_t* states, const float* x, float* pi, float* v, int n,
                          void* stream) {
    if (!net || !pi || !v || n < 0) return YK_ERR_ARG;
    if (n == 0) return YK_OK;
    hipStream_t s = as_stream(stream);
    float* logits = nullptr;
    YK_HIP(hipMallocAsync((void**)&logits, sizeof(float) * (size_t)n * PI_LD, s));
    int rc = launch_forward(net->dev, states, x, nullptr, nullptr, n, logits, v, s);
    if (rc == YK_OK) rc = launch_softmax(logits, pi, n, s);
    (void)hipFreeAsync(logits, s);
    return rc;
}

int yk_net_predict(yk_net_t* net, const yk_state_t* states, float* pi, float* v, int n, void* stream) {
    if (!states) return YK_ERR_ARG;
    return predict_common(net, states, nullptr, pi, v, n, stream);
}

int yk_net_predict_features(yk_net_t* net, const float* x, float* pi, float* v, int n, void* stream) {
    if (!x) return YK_ERR_ARG;
    return predict_common(net, nullptr, x, pi, v, n, stream);
}

}  // extern "C"
