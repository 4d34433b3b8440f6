// yk_train.hip - NNetWrapper.train (yacht/NNet.py:118-174) on MI355X: one optimiser step of
// YachtNNet (yacht/pytorch/YachtNNet.py:8-70) in float32.
//
// Per minibatch: gather (features from packed states, hard targets, values) -> forward with the
// activations the backward needs -> loss = CE(logits, argmax(pi)) + vloss_weight * MSE(v, z)
// (NNet.py:143-148) -> backward -> [caller all-reduces the gradient buffer for DDP] ->
// clip_grad_norm_(5.0) (NNet.py:152-153) -> AdamW (NNet.py:109-110).
//
// The dense layers are plain GEMMs on a hand-written f32 MFMA kernel (k_sgemm:
// v_mfma_f32_16x16x4_f32, exact f32 products and f32 accumulation).  Everything between them is
// hand-written and fused per row: bias + SiLU + LayerNorm + dropout + residual forward, the
// matching backward (LayerNorm input gradient from the saved statistics), the loss and its
// gradients, column reductions for bias / LayerNorm parameter gradients, the global gradient
// norm and the AdamW update.  Parameters, gradients and the Adam moments are single flat
// buffers in torch state_dict order, so the gradient buffer is one RCCL all-reduce.
#include <algorithm>
#include <cmath>
#include <vector>

#include "yk_api.h"
#include "yk_common.h"
#include "yk_train_amp.h"

using namespace yk;

namespace {

constexpr int TPB = 256;
typedef float floatx4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }
__device__ __forceinline__ float silu_f(float x) { return x * sigm(x); }
__device__ __forceinline__ float silu_grad(float x) {  // d/dx x*s(x) = s(x) (1 + x (1 - s(x)))
    const float s = sigm(x);
    return s * (1.0f + x * (1.0f - s));
}
__device__ __forceinline__ float wsum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wmax(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
// dropout masks: dropout_keep (yk_common.h) of element global row * H + column; the row counts
// from the step's row offset, so the ranks of a split minibatch draw the masks one process
// drawing the whole minibatch would

// LayerNorm of one row held VPL-per-lane (biased variance, eps 1e-5); returns x_hat, mean, rstd
template <int VPL>
__device__ __forceinline__ void ln_row(float (&x)[VPL], int H, float& mu, float& rs) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; i++) s += x[i];
    mu = wsum(s) / (float)H;
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; i++) {
        const float d = x[i] - mu;
        v += d * d;
    }
    rs = 1.0f / sqrtf(wsum(v) / (float)H + 1e-5f);
#pragma unroll
    for (int i = 0; i < VPL; i++) x[i] = (x[i] - mu) * rs;
}
// LayerNorm backward for one row: dxh = dy * gamma; dx = rs/H (H dxh - sum dxh - xh sum(dxh xh))
template <int VPL>
__device__ __forceinline__ void ln_row_bwd(const float (&xh)[VPL], float (&dy)[VPL], const float* g, int c0, int H, float rs) {
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; i++) {
        dy[i] *= g[c0 + i];
        a += dy[i];
        b += dy[i] * xh[i];
    }
    a = wsum(a);
    b = wsum(b);
#pragma unroll
    for (int i = 0; i < VPL; i++) dy[i] = rs / (float)H * ((float)H * dy[i] - a - xh[i] * b);
}

// ---------------------------------------------------------------- forward row kernels (one wave per row)
// inp: Z0 += b; A = LN(Z0) (affine); H0 = dropout(silu(A)).  Saves Z0 (+bias), mu, rs, mask.
template <int VPL>
__global__ void k_inp_fwd(float* Z, const float* b, const float* g, const float* be, float* mu_o, float* rs_o,
                          uint8_t* mask, float* Hout, int B, float p, uint64_t seed, uint64_t step, int64_t row_base) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= B) return;
    constexpr int H = VPL * 64;
    const int c0 = lane * VPL;
    float x[VPL];
#pragma unroll
    for (int i = 0; i < VPL; i++) {
        x[i] = Z[(long)row * H + c0 + i] + b[c0 + i];
        Z[(long)row * H + c0 + i] = x[i];
    }
    float mu, rs;
    ln_row<VPL>(x, H, mu, rs);
    if (lane == 0) {
        mu_o[row] = mu;
        rs_o[row] = rs;
    }
    const float sc = 1.0f / (1.0f - p);
    KeepCache kc;
#pragma unroll
    for (int i = 0; i < VPL; i++) {
        const long idx = (long)row * H + c0 + i;
        const float a = x[i] * g[c0 + i] + be[c0 + i];
        const bool k = dropout_keep(kc, seed, 0, step, (row_base + row) * H + c0 + i, p);
        mask[idx] = k;
        Hout[idx] = k ? silu_f(a) * (p > 0.f ? sc : 1.0f) : 0.0f;
    }
}
// block half 1: U1 += b1; L1 = LN1(silu(U1)); R1 = dropout(L1).  Saves U1 (+bias), mu, rs, mask, R1.
// block half 2 (layer < 0 marks it): U2 += b2; L2 = LN2(silu(U2)); Hout = Hin + L2.
template <int VPL>
__global__ void k_blk_fwd(float* U, const float* b, const float* g, const float* be, float* mu_o, float* rs_o,
                          uint8_t* mask, float* out, const float* Hin, int B, float p, uint64_t seed, uint64_t step,
                          int layer, int64_t row_base) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= B) return;
    constexpr int H = VPL * 64;
    const int c0 = lane * VPL;
    float x[VPL];
#pragma unroll
    for (int i = 0; i < VPL; i++) {
        const float u = U[(long)row * H + c0 + i] + b[c0 + i];
        U[(long)row * H + c0 + i] = u;
        x[i] = silu_f(u);
    }
    float mu, rs;
    ln_row<VPL>(x, H, mu, rs);
    if (lane == 0) {
        mu_o[row] = mu;
        rs_o[row] = rs;
    }
    const float sc = 1.0f / (1.0f - p);
    KeepCache kc;
#pragma unroll
    for (int i = 0; i < VPL; i++) {
        const long idx = (long)row * H + c0 + i;
        const float l = x[i] * g[c0 + i] + be[c0 + i];
        if (Hin) {
            out[idx] = Hin[idx] + l;  // residual
        } else {
            const bool k = dropout_keep(kc, seed, layer, step, (row_base + row) * H + c0 + i, p);
            mask[idx] = k;
            out[idx] = k ? l * (p > 0.f ? sc : 1.0f) : 0.0f;
        }
    }
}
// heads: Tpi = LNpi(h), Api = silu(Tpi); Tv = LNv(h), Av = silu(Tv).  Saves stats of both.
template <int VPL>
__global__ void k_heads_fwd(const float* Hh, const float* gp, const float* bp, const float* gv, const float* bv,
                            float* Api, float* Av, float* mup, float* rsp, float* muv, float* rsv, int B) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= B) return;
    constexpr int H = VPL * 64;
    const int c0 = lane * VPL;
    float x[VPL], y[VPL];
#pragma unroll
    for (int i = 0; i < VPL; i++) x[i] = y[i] = Hh[(long)row * H + c0 + i];
    float m1, r1, m2, r2;
    ln_row<VPL>(x, H, m1, r1);
    ln_row<VPL>(y, H, m2, r2);
    if (lane == 0) {
        mup[row] = m1;
        rsp[row] = r1;
        muv[row] = m2;
        rsv[row] = r2;
    }
#pragma unroll
    for (int i = 0; i < VPL; i++) {
        Api[(long)row * H + c0 + i] = silu_f(x[i] * gp[c0 + i] + bp[c0 + i]);
        Av[(long)row * H + c0 + i] = silu_f(y[i] * gv[c0 + i] + bv[c0 + i]);
    }
}
// v head tail + both losses + the output gradients.  One 256-thread workgroup per row (13 logits
// per lane: four times the memory parallelism of a wave per row); wave 0 also does the v head.
//   Zv1 += bv1 (saved); v = tanh(silu(Zv1) . wv2 + bv2); mse_i = (v - z)^2
//   logits += bpi; ce_i = lse - logit[t]; dlogits = (softmax - onehot(t)) / B
//   dzv2 = vw * 2 (v - z) / B * (1 - v^2); dZv1 = dzv2 wv2 silu'(Zv1)
constexpr int LOSS_T = 256;
constexpr int LOSS_NV = (ASIZE + LOSS_T - 1) / LOSS_T;  // logits per thread
__global__ __launch_bounds__(LOSS_T) void k_loss(const float* logits, const float* bpi, float* Zv1, const float* bv1,
                                                 const float* wv2, const float* bv2, const int32_t* tgt,
                                                 const float* vt, float* dlogits, float* dZv1, float* dzv2,
                                                 float* v2prod, float* vout, float2* lrow, int B, int A, float vw) {
    __shared__ float red[2][LOSS_T / 64];
    const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (row >= B) return;
    const float* z = logits + (long)row * A;
    float x[LOSS_NV];
    float m = -INFINITY;
#pragma unroll
    for (int k = 0; k < LOSS_NV; k++) {
        const int a = tid + LOSS_T * k;
        x[k] = a < A ? z[a] + bpi[a] : -INFINITY;
        m = fmaxf(m, x[k]);
    }
    m = wmax(m);
    if (lane == 0) red[0][w] = m;
    __syncthreads();
    m = fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3]));
    float se = 0.f;
#pragma unroll
    for (int k = 0; k < LOSS_NV; k++) se += expf(x[k] - m);
    se = wsum(se);
    if (lane == 0) red[1][w] = se;
    __syncthreads();
    se = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
    const float lse = m + logf(se);
    const int t = tgt[row];
    const float invB = 1.0f / (float)B;
#pragma unroll
    for (int k = 0; k < LOSS_NV; k++) {
        const int a = tid + LOSS_T * k;
        if (a < A) dlogits[(long)row * A + a] = (expf(x[k] - lse) - (a == t ? 1.0f : 0.0f)) * invB;
    }
    if (w != 0) return;
    const float zt = z[t] + bpi[t];  // the target logit (the same sum as x[k] where a == t)
    // value head tail (128 hidden, 2 per lane)
    float s = 0.f, zz[2];
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const int c = 2 * lane + k;
        zz[k] = Zv1[(long)row * 128 + c] + bv1[c];
        Zv1[(long)row * 128 + c] = zz[k];
        s += silu_f(zz[k]) * wv2[c];
    }
    s = wsum(s) + bv2[0];
    const float v = tanhf(s);
    const float e = v - vt[row];
    const float dv = vw * 2.0f * e * invB * (1.0f - v * v);
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const int c = 2 * lane + k;
        dZv1[(long)row * 128 + c] = dv * wv2[c] * silu_grad(zz[k]);
        v2prod[(long)row * 128 + c] = dv * silu_f(zz[k]);  // rows of dL/d v_head.4.weight
    }
    if (lane == 0) {  // the per-row losses; k_colsums sums them (no contended atomics)
        dzv2[row] = dv;
        vout[row] = v;
        lrow[row] = make_float2(lse - zt, e * e);
    }
}

// ---------------------------------------------------------------- backward row kernels
// heads backward: dApi, dAv -> dTpi, dTv (silu') -> LN backward of both -> dH (sum); writes
// the per-row LayerNorm parameter contributions gpi_row = dTpi * xhat, bpi_row = dTpi (same for v)
template <int VPL>
__global__ void k_heads_bwd(const float* Hh, const float* gp, const float* bp, const float* gv, const float* bv,
                            const float* mup, const float* rsp, const float* muv, const float* rsv, const float* dApi,
                            const float* dAv, float* dH, float* rg_p, float* rb_p, float* rg_v, float* rb_v, int B) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= B) return;
    constexpr int H = VPL * 64;
    const int c0 = lane * VPL;
    float xp[VPL], xv[VPL], dp[VPL], dv[VPL];
    const float m1 = mup[row], r1 = rsp[row], m2 = muv[row], r2 = rsv[row];
#pragma unroll
    for (int i = 0; i < VPL; i++) {
        const long idx = (long)row * H + c0 + i;
        const float h = Hh[idx];
        xp[i] = (h - m1) * r1;
        xv[i] = (h - m2) * r2;
        dp[i] = dApi[idx] * silu_grad(xp[i] * gp[c0 + i] + bp[c0 + i]);
        dv[i] = dAv[idx] * silu_grad(xv[i] * gv[c0 + i] + bv[c0 + i]);
        rg_p[idx] = dp[i] * xp[i];
        rb_p[idx] = dp[i];
        rg_v[idx] = dv[i] * xv[i];
        rb_v[idx] = dv[i];
    }
    ln_row_bwd<VPL>(xp, dp, gp, c0, H, r1);
    ln_row_bwd<VPL>(xv, dv, gv, c0, H, r2);
#pragma unroll
    for (int i = 0; i < VPL; i++) dH[(long)row * H + c0 + i] = dp[i] + dv[i];
}
// block-half backward through LN(silu(U)) (+ dropout on the way in for half 1):
//   dL = dIn (* mask / (1-p) when mask); dS = LN backward (S = silu(U) recomputed); dU = dS silu'(U)
// rg/rb: per-row LayerNorm gamma / beta contributions
template <int VPL>
__global__ void k_blk_bwd(const float* dIn, const uint8_t* mask, float p, const float* U, const float* g,
                          const float* mu, const float* rs, float* dU, float* rg, float* rb, int B) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= B) return;
    constexpr int H = VPL * 64;
    const int c0 = lane * VPL;
    const float m = mu[row], r = rs[row];
    const float sc = p > 0.f ? 1.0f / (1.0f - p) : 1.0f;
    float xh[VPL], d[VPL], u[VPL];
#pragma unroll
    for (int i = 0; i < VPL; i++) {
        const long idx = (long)row * H + c0 + i;
        u[i] = U[idx];
        xh[i] = (silu_f(u[i]) - m) * r;
        d[i] = dIn[idx];
        if (mask) d[i] = mask[idx] ? d[i] * sc : 0.0f;
        rg[idx] = d[i] * xh[i];
        rb[idx] = d[i];
    }
    ln_row_bwd<VPL>(xh, d, g, c0, H, r);
#pragma unroll
    for (int i = 0; i < VPL; i++) dU[(long)row * H + c0 + i] = d[i] * silu_grad(u[i]);
}
// inp backward: dH0 -> dropout -> silu'(A) -> LN backward (input Z0) -> dZ0
template <int VPL>
__global__ void k_inp_bwd(const float* dH0, const uint8_t* mask, float p, const float* Z, const float* g,
                          const float* be, const float* mu, const float* rs, float* dZ, float* rg, float* rb, int B) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= B) return;
    constexpr int H = VPL * 64;
    const int c0 = lane * VPL;
    const float m = mu[row], r = rs[row];
    const float sc = p > 0.f ? 1.0f / (1.0f - p) : 1.0f;
    float xh[VPL], d[VPL];
#pragma unroll
    for (int i = 0; i < VPL; i++) {
        const long idx = (long)row * H + c0 + i;
        xh[i] = (Z[idx] - m) * r;
        float dy = mask[idx] ? dH0[idx] * sc : 0.0f;
        dy *= silu_grad(xh[i] * g[c0 + i] + be[c0 + i]);
        d[i] = dy;
        rg[idx] = dy * xh[i];
        rb[idx] = dy;
    }
    ln_row_bwd<VPL>(xh, d, g, c0, H, r);
#pragma unroll
    for (int i = 0; i < VPL; i++) dZ[(long)row * H + c0 + i] = d[i];
}
// Every column reduction of a step in one launch: job j sums the B rows of src[j] ([B][N_j])
// into dst[j][N_j] (bias and LayerNorm gradients).  Block = one 16-column tile of one job, 16
// row groups x 16 columns, fixed order (deterministic).
struct ColJob {
    const float* src;
    float* dst;
    int N;
};
__global__ __launch_bounds__(256) void k_colsums(const ColJob* jobs, const int2* tiles, int B) {
    __shared__ float part[16][17];
    const int2 t = tiles[blockIdx.x];  // (job, first column)
    const ColJob jb = jobs[t.x];
    const int c = t.y + (threadIdx.x & 15), g = threadIdx.x >> 4;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    if (c < jb.N) {
        int r = g;
        for (; r + 48 < B; r += 64) {
            a0 += jb.src[(long)r * jb.N + c];
            a1 += jb.src[(long)(r + 16) * jb.N + c];
            a2 += jb.src[(long)(r + 32) * jb.N + c];
            a3 += jb.src[(long)(r + 48) * jb.N + c];
        }
        for (; r < B; r += 16) a0 += jb.src[(long)r * jb.N + c];
    }
    part[g][threadIdx.x & 15] = (a0 + a1) + (a2 + a3);
    __syncthreads();
    if (g == 0 && c < jb.N) {
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < 16; k++) s += part[k][threadIdx.x & 15];
        jb.dst[c] = s;
    }
}
// gather a minibatch: features of states[idx[i]], targets, values
__global__ void k_gather(const yk_state_t* states, const int32_t* tgt_all, const float* v_all, const int32_t* idx,
                         float* X, int32_t* tgt, float* vt, int B) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= B * 64) return;
    const int i = t >> 6, f = t & 63;
    const int src = idx ? idx[i] : i;
    if (f < FEAT) {
        const uint4* q = reinterpret_cast<const uint4*>(states + src);
        YkS s;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint4 u = q[k];
            s.w[2 * k] = (uint64_t)u.x | ((uint64_t)u.y << 32);
            s.w[2 * k + 1] = (uint64_t)u.z | ((uint64_t)u.w << 32);
        }
        X[(long)i * FEAT + f] = feature(s, f);
    }
    if (f == 0) {
        tgt[i] = tgt_all[src];
        vt[i] = v_all[src];
    }
}
// sum of squares of the gradient buffer: one double partial per workgroup (no atomics); k_adamw
// adds the SQ_BLOCKS partials in a fixed order
constexpr int SQ_BLOCKS = 1024;
__global__ void k_sqnorm(const float* g, long n, double* part_out) {
    __shared__ double part[TPB / 64];
    double s = 0.0;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const double x = g[i];
        s += x * x;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int w = 0; w < TPB / 64; w++) t += part[w];
        part_out[blockIdx.x] = t;
    }
}
// clip_grad_norm_ (coef = min(1, max_norm / (norm + 1e-6)), NNet.py:152-153) + AdamW
// (torch single-tensor AdamW: decoupled decay, bias-corrected moments)
__global__ void k_adamw(float* p, float* g, float* m, float* v, long n, const double* sq_part, double* sq_out,
                        float max_norm, float lr, float wd, float b1, float b2, float eps, float step_size,
                        float bc2_sqrt) {
    __shared__ double red[TPB / 64];
    __shared__ double sq_total;
    {  // every workgroup adds the SQ_BLOCKS partials in the same fixed order
        static_assert(SQ_BLOCKS % TPB == 0, "partials per thread");
        double t = 0.0;
#pragma unroll
        for (int k = 0; k < SQ_BLOCKS / TPB; k++) t += sq_part[threadIdx.x + TPB * k];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) t += __shfl_xor(t, o, 64);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = t;
        __syncthreads();
        if (threadIdx.x == 0) {
            double u = 0.0;
            for (int k = 0; k < TPB / 64; k++) u += red[k];
            sq_total = u;
            if (blockIdx.x == 0) *sq_out = u;
        }
        __syncthreads();
    }
    const float norm = (float)sqrt(sq_total);
    float coef = max_norm / (norm + 1e-6f);
    coef = coef > 1.0f ? 1.0f : coef;
    const float decay = 1.0f - lr * wd;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const float gi = g[i] * coef;
        g[i] = gi;
        float pi = p[i] * decay;
        const float mi = m[i] + (gi - m[i]) * (1.0f - b1);  // exp_avg.lerp_(grad, 1 - beta1)
        const float vi = v[i] * b2 + (1.0f - b2) * gi * gi;
        m[i] = mi;
        v[i] = vi;
        const float denom = sqrtf(vi) / bc2_sqrt + eps;
        pi -= step_size * (mi / denom);
        p[i] = pi;
    }
}

}  // namespace

// ---------------------------------------------------------------- host object
struct yk_trainer {
    int H = 0, NB = 0, Bmax = 0;
    yk_train_config_t cfg{};
    float *P = nullptr, *G = nullptr, *M = nullptr, *V = nullptr;
    long nparams = 0;
    std::vector<long> off;  // tensor offsets, state_dict order
    std::vector<long> len;
    uint64_t step = 0;
    std::vector<void*> allocs;
    // activations (Bmax rows)
    float *X = nullptr, *vt = nullptr, *vout = nullptr;
    int32_t* tgt = nullptr;
    float *Z0 = nullptr, *mu0 = nullptr, *rs0 = nullptr;
    uint8_t* mask0 = nullptr;
    std::vector<float*> Hs, U1, U2, R1, mu1, rs1, mu2, rs2;
    std::vector<uint8_t*> mask1;
    float *Api = nullptr, *Av = nullptr, *mup = nullptr, *rsp = nullptr, *muv = nullptr, *rsv = nullptr;
    float *logits = nullptr, *Zv1 = nullptr, *dlogits = nullptr, *dZv1 = nullptr, *dzv2 = nullptr;
    float *dA = nullptr, *dAv = nullptr, *dH = nullptr, *dT = nullptr, *v2prod = nullptr;
    // per-stage row buffers whose column sums are gradients (kept until the one k_colsums)
    float *rgp = nullptr, *rbp = nullptr, *rgv = nullptr, *rbv = nullptr, *dZ0 = nullptr, *rg0 = nullptr, *rb0 = nullptr;
    std::vector<float*> dU1, dU2, rg1, rb1, rg2, rb2;
    ColJob* jobs = nullptr;
    int2* tiles = nullptr;
    int ntiles = 0;
    double* acc = nullptr;  // [0] ce sum, [1] mse sum (unused), [2] grad sq norm
    float* gws = nullptr;   // k_sgemm's split-K partial tiles
    double* sqpart = nullptr;  // k_sqnorm partials
    float2* lrow = nullptr;    // per-row (ce, squared value error) of the last batch
    float* lsum = nullptr;     // their column sums (k_colsums)
    double* eloss = nullptr;   // report epoch: [0] sum of per-batch mean losses, [1] batches (k_epoch_loss)
    bool eloss_on = false;
    double eloss_vw = 1.0;
    double host_loss[3] = {0, 0, 0};
    int64_t row_base = 0;        // global row of the next backward's first example (dropout)
    yk::AmpTrain* amp = nullptr;  // mixed-precision mode (yk_train_amp.hip)
};

namespace {
// tensor indices in state_dict order (YachtNNet.py:30-52)
enum { T_WIN = 0, T_BIN, T_GIN, T_BEIN };
inline int t_blk(int b, int k) { return 4 + 8 * b + k; }  // k: 0 fc1.w 1 fc1.b 2 ln1.w 3 ln1.b 4 fc2.w 5 fc2.b 6 ln2.w 7 ln2.b
inline int t_head(int NB, int k) { return 4 + 8 * NB + k; }  // 0 pi.0.w 1 pi.0.b 2 pi.2.w 3 pi.2.b 4 v.0.w 5 v.0.b 6 v.2.w 7 v.2.b 8 v.4.w 9 v.4.b

template <class T>
int talloc(yk_trainer* t, T** p, size_t count) {
    void* q = nullptr;
    if (hipMalloc(&q, sizeof(T) * (count ? count : 1)) != hipSuccess) {
        (void)hipGetLastError();
        return YK_ERR_NOMEM;
    }
    t->allocs.push_back(q);
    *p = static_cast<T*>(q);
    return YK_OK;
}

// row-major C[M][N] = op(A)[M][K] . op(B)[K][N] (+ beta C), op = transpose when ta / tb (A stored
// [K][M], B stored [N][K]).  64 x 64 output tiles per 256-thread workgroup, each wave a 32 x 32
// quarter as 2 x 2 blocks of v_mfma_f32_16x16x4_f32 (f32 operands: exact products, f32
// accumulation, the reference's CPU arithmetic up to summation order), or 32 x 32 tiles (a 16 x 16
// block per wave) for shapes with few tiles.  K goes through LDS 64 (128 for 32 x 32 tiles) deep,
// the next chunk's global reads issued before the current chunk's MFMAs (coalesced along whichever
// dimension is contiguous in memory); LDS rows padded by 16 floats, so a wave's 64 fragment reads
// hit 64 distinct banks (64-wide tiles).  Few output tiles over a long K (dA = dlogits W_pi: K = 3226 over 32
// tiles) split K over blockIdx.z into partial tiles that k_sgemm_reduce sums in split order (the
// result does not depend on scheduling: ranks stay bit-identical).
template <int TM>  // output tile TM x TM: 64 (each wave a 32 x 32 quarter, 2 x 2 MFMA blocks) or 32 (16 x 16)
constexpr int gk_of() { return TM == 64 ? 64 : 128; }  // K per LDS chunk (16 elements per thread either way)
// An operand tile in LDS keeps its memory order, so the staging stores are as contiguous as the
// global reads: [k][row] (stride TM + 16) when the row index is contiguous in memory (a transposed
// operand), else [row][k] (stride GK + 4).  Either way a wave's fragment read - rows l & 15, k
// (l >> 4) - and its staging store hit 64 distinct banks.
template <int TM, bool T>
struct OpTile {
    static constexpr int GK = gk_of<TM>(), LD = T ? TM + 16 : GK + 4, SZ = T ? GK * LD : TM * LD;
    __device__ static __forceinline__ int at(int r, int k) { return T ? k * LD + r : r * LD + k; }
    // element e of the tile (e = tid + 256 i): (row, k) with the memory-contiguous index fastest
    __device__ static __forceinline__ void rc(int e, int& r, int& k) {
        if (T) { r = e % TM; k = e / TM; } else { k = e % GK; r = e / GK; }
    }
};
template <int TM, bool TA, bool TB>
__global__ __launch_bounds__(256) void k_sgemm(int M, int N, int K, int kc, const float* __restrict__ A, int lda,
                                               const float* __restrict__ B, int ldb, float* __restrict__ C, int ldc,
                                               float beta, float* __restrict__ part) {
    using OA = OpTile<TM, TA>;
    using OB = OpTile<TM, !TB>;  // B[k][n] is "transposed" (n contiguous) when stored [K][N], i.e. !tb
    constexpr int GK = gk_of<TM>(), BL = TM / 32, EPT = TM * GK / 256;  // blocks per wave side; elements per thread
    __shared__ float As[OA::SZ];
    __shared__ float Bs[OB::SZ];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int m0 = blockIdx.y * TM, n0 = blockIdx.x * TM;
    const int kb = blockIdx.z * kc, ke = min(K, kb + kc);
    const int wm = (wave >> 1) * (TM / 2), wn = (wave & 1) * (TM / 2);
    floatx4 acc[BL][BL];
#pragma unroll
    for (int i = 0; i < BL; i++)
#pragma unroll
        for (int j = 0; j < BL; j++) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    float av[EPT], bv[EPT];
    auto load = [&](int k0) {
#pragma unroll
        for (int i = 0; i < EPT; i++) {
            const int e = tid + 256 * i;
            int r, k, c, kk;
            OA::rc(e, r, k);
            OB::rc(e, c, kk);
            const int gm = m0 + r, gk = k0 + k, gn = n0 + c, gkb = k0 + kk;
            av[i] = (gm < M && gk < ke) ? (TA ? A[(long)gk * lda + gm] : A[(long)gm * lda + gk]) : 0.f;
            bv[i] = (gn < N && gkb < ke) ? (TB ? B[(long)gn * ldb + gkb] : B[(long)gkb * ldb + gn]) : 0.f;
        }
    };
    load(kb);
    for (int k0 = kb; k0 < ke; k0 += GK) {
#pragma unroll
        for (int i = 0; i < EPT; i++) {
            const int e = tid + 256 * i;
            int r, k, c, kk;
            OA::rc(e, r, k);
            OB::rc(e, c, kk);
            As[OA::at(r, k)] = av[i];
            Bs[OB::at(c, kk)] = bv[i];
        }
        __syncthreads();
        if (k0 + GK < ke) load(k0 + GK);  // the next chunk's reads fly under this chunk's MFMAs
#pragma unroll
        for (int ks = 0; ks < GK; ks += 4) {
            const int k = ks + (lane >> 4);
            float a[BL], b[BL];
#pragma unroll
            for (int i = 0; i < BL; i++) a[i] = As[OA::at(wm + 16 * i + (lane & 15), k)];
#pragma unroll
            for (int j = 0; j < BL; j++) b[j] = Bs[OB::at(wn + 16 * j + (lane & 15), k)];
#pragma unroll
            for (int i = 0; i < BL; i++)
#pragma unroll
                for (int j = 0; j < BL; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        __syncthreads();  // every wave is done reading the chunk before the next one is stored
    }
    // block (i, j): lane l holds rows 4 (l >> 4) + r, column l & 15
#pragma unroll
    for (int i = 0; i < BL; i++)
#pragma unroll
        for (int j = 0; j < BL; j++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int gm = m0 + wm + 16 * i + 4 * (lane >> 4) + r, gn = n0 + wn + 16 * j + (lane & 15);
                if (gm < M && gn < N) {
                    if (part) {
                        part[((long)blockIdx.z * M + gm) * N + gn] = acc[i][j][r];
                    } else {
                        float* c = C + (long)gm * ldc + gn;
                        *c = beta != 0.f ? acc[i][j][r] + beta * *c : acc[i][j][r];
                    }
                }
            }
}
// C = sum over the splits in order (+ beta C)
__global__ void k_sgemm_reduce(int M, int N, int S, const float* __restrict__ part, float* __restrict__ C, int ldc,
                               float beta) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= (long)M * N) return;
    float s = part[i];
    for (int z = 1; z < S; z++) s += part[(long)z * M * N + i];
    float* c = C + (i / N) * ldc + i % N;
    *c = beta != 0.f ? s + beta * *c : s;
}
constexpr long GEMM_WS = 1L << 21;  // split-K workspace (floats): splits x M x N, <= 512 32 x 32 tiles' worth
// tile size and K split for the shape: 64 x 64 tiles when there are >= 128 of them, else 32 x 32;
// K split (a partial pass + k_sgemm_reduce) only for long K over few tiles (dA: K = 3226)
int gemm_rm(hipStream_t s, float* ws, bool ta, bool tb, int M, int N, int K, const float* A, int lda, const float* B,
            int ldb, float* C, int ldc, float beta) {
    const int t64 = ((M + 63) / 64) * ((N + 63) / 64);
    const int TM = t64 >= 128 ? 64 : 32;
    const int tiles = ((M + TM - 1) / TM) * ((N + TM - 1) / TM);
    int S = K >= 1024 ? std::max(1, std::min(512 / tiles, K / 256)) : 1;
    while (S > 1 && (long)S * M * N > GEMM_WS) S--;
    const int GKS = TM == 64 ? gk_of<64>() : gk_of<32>();
    const int kc = ((K + S - 1) / S + GKS - 1) / GKS * GKS;
    S = (K + kc - 1) / kc;
    const dim3 grid((unsigned)((N + TM - 1) / TM), (unsigned)((M + TM - 1) / TM), (unsigned)S);
    float* part = S > 1 ? ws : nullptr;
#define YK_SGEMM(T, A_, B_) \
    hipLaunchKernelGGL((k_sgemm<T, A_, B_>), grid, dim3(256), 0, s, M, N, K, kc, A, lda, B, ldb, C, ldc, beta, part)
    if (TM == 64) {
        if (ta) { if (tb) YK_SGEMM(64, true, true); else YK_SGEMM(64, true, false); }
        else { if (tb) YK_SGEMM(64, false, true); else YK_SGEMM(64, false, false); }
    } else {
        if (ta) { if (tb) YK_SGEMM(32, true, true); else YK_SGEMM(32, true, false); }
        else { if (tb) YK_SGEMM(32, false, true); else YK_SGEMM(32, false, false); }
    }
#undef YK_SGEMM
    if (S > 1)
        hipLaunchKernelGGL(k_sgemm_reduce, dim3((unsigned)(((long)M * N + 255) / 256)), dim3(256), 0, s, M, N, S, ws, C,
                           ldc, beta);
    return hipGetLastError() == hipSuccess ? YK_OK : YK_ERR_HIP;
}

template <int VPL>
int step_impl(yk_trainer* t, const yk_state_t* states, const int32_t* targets, const float* values, const int32_t* idx,
              int B, hipStream_t s) {
    constexpr int H = VPL * 64;
    const int NB = t->NB, A = ASIZE;
    const float p = t->cfg.dropout;
    const uint64_t seed = t->cfg.seed, step = t->step;
    auto Pt = [&](int k) { return t->P + t->off[k]; };
    auto Gt = [&](int k) { return t->G + t->off[k]; };
    const dim3 rows((B + 3) / 4), wave4(256);
    int rc;
    hipLaunchKernelGGL(k_gather, dim3((B * 64 + 255) / 256), dim3(256), 0, s, states, targets, values, idx, t->X, t->tgt,
                       t->vt, B);
    YK_LAUNCHED();
    // ---- forward
    if ((rc = gemm_rm(s, t->gws, false, true, B, H, FEAT, t->X, FEAT, Pt(T_WIN), FEAT, t->Z0, H, 0.f))) return rc;
    hipLaunchKernelGGL(k_inp_fwd<VPL>, rows, wave4, 0, s, t->Z0, Pt(T_BIN), Pt(T_GIN), Pt(T_BEIN), t->mu0, t->rs0,
                       t->mask0, t->Hs[0], B, p, seed, step, t->row_base);
    YK_LAUNCHED();
    for (int b = 0; b < NB; b++) {
        if ((rc = gemm_rm(s, t->gws, false, true, B, H, H, t->Hs[b], H, Pt(t_blk(b, 0)), H, t->U1[b], H, 0.f))) return rc;
        hipLaunchKernelGGL(k_blk_fwd<VPL>, rows, wave4, 0, s, t->U1[b], Pt(t_blk(b, 1)), Pt(t_blk(b, 2)), Pt(t_blk(b, 3)),
                           t->mu1[b], t->rs1[b], t->mask1[b], t->R1[b], (const float*)nullptr, B, p, seed, step, 1 + b,
                           t->row_base);
        YK_LAUNCHED();
        if ((rc = gemm_rm(s, t->gws, false, true, B, H, H, t->R1[b], H, Pt(t_blk(b, 4)), H, t->U2[b], H, 0.f))) return rc;
        hipLaunchKernelGGL(k_blk_fwd<VPL>, rows, wave4, 0, s, t->U2[b], Pt(t_blk(b, 5)), Pt(t_blk(b, 6)), Pt(t_blk(b, 7)),
                           t->mu2[b], t->rs2[b], (uint8_t*)nullptr, t->Hs[b + 1], t->Hs[b], B, p, seed, step, -1,
                           t->row_base);
        YK_LAUNCHED();
    }
    const float* Hh = t->Hs[NB];
    hipLaunchKernelGGL(k_heads_fwd<VPL>, rows, wave4, 0, s, Hh, Pt(t_head(NB, 0)), Pt(t_head(NB, 1)), Pt(t_head(NB, 4)),
                       Pt(t_head(NB, 5)), t->Api, t->Av, t->mup, t->rsp, t->muv, t->rsv, B);
    YK_LAUNCHED();
    if ((rc = gemm_rm(s, t->gws, false, true, B, A, H, t->Api, H, Pt(t_head(NB, 2)), H, t->logits, A, 0.f))) return rc;
    if ((rc = gemm_rm(s, t->gws, false, true, B, 128, H, t->Av, H, Pt(t_head(NB, 6)), H, t->Zv1, 128, 0.f))) return rc;
    hipLaunchKernelGGL(k_loss, dim3(B), dim3(LOSS_T), 0, s, t->logits, Pt(t_head(NB, 3)), t->Zv1, Pt(t_head(NB, 7)),
                       Pt(t_head(NB, 8)), Pt(t_head(NB, 9)), t->tgt, t->vt, t->dlogits, t->dZv1, t->dzv2, t->v2prod,
                       t->vout, t->lrow, B, A, t->cfg.vloss_weight);
    YK_LAUNCHED();
    // ---- backward: heads (bias / LayerNorm gradients are column sums, taken at the end)
    if ((rc = gemm_rm(s, t->gws, true, false, A, H, B, t->dlogits, A, t->Api, H, Gt(t_head(NB, 2)), H, 0.f))) return rc;
    if ((rc = gemm_rm(s, t->gws, true, false, 128, H, B, t->dZv1, 128, t->Av, H, Gt(t_head(NB, 6)), H, 0.f))) return rc;
    if ((rc = gemm_rm(s, t->gws, false, false, B, H, A, t->dlogits, A, Pt(t_head(NB, 2)), H, t->dA, H, 0.f))) return rc;
    if ((rc = gemm_rm(s, t->gws, false, false, B, H, 128, t->dZv1, 128, Pt(t_head(NB, 6)), H, t->dAv, H, 0.f))) return rc;
    hipLaunchKernelGGL(k_heads_bwd<VPL>, rows, wave4, 0, s, Hh, Pt(t_head(NB, 0)), Pt(t_head(NB, 1)), Pt(t_head(NB, 4)),
                       Pt(t_head(NB, 5)), t->mup, t->rsp, t->muv, t->rsv, t->dA, t->dAv, t->dH, t->rgp, t->rbp, t->rgv,
                       t->rbv, B);
    YK_LAUNCHED();
    // ---- blocks, last to first; t->dH holds dL/dH_{b+1}
    for (int b = NB - 1; b >= 0; b--) {
        hipLaunchKernelGGL(k_blk_bwd<VPL>, rows, wave4, 0, s, t->dH, (const uint8_t*)nullptr, 0.f, t->U2[b],
                           Pt(t_blk(b, 6)), t->mu2[b], t->rs2[b], t->dU2[b], t->rg2[b], t->rb2[b], B);
        YK_LAUNCHED();
            if ((rc = gemm_rm(s, t->gws, true, false, H, H, B, t->dU2[b], H, t->R1[b], H, Gt(t_blk(b, 4)), H, 0.f))) return rc;
        if ((rc = gemm_rm(s, t->gws, false, false, B, H, H, t->dU2[b], H, Pt(t_blk(b, 4)), H, t->dT, H, 0.f))) return rc;  // dR1
        hipLaunchKernelGGL(k_blk_bwd<VPL>, rows, wave4, 0, s, t->dT, t->mask1[b], p, t->U1[b], Pt(t_blk(b, 2)), t->mu1[b],
                           t->rs1[b], t->dU1[b], t->rg1[b], t->rb1[b], B);
        YK_LAUNCHED();
            if ((rc = gemm_rm(s, t->gws, true, false, H, H, B, t->dU1[b], H, t->Hs[b], H, Gt(t_blk(b, 0)), H, 0.f))) return rc;
        // dH_b = dH_{b+1} (residual) + dU1 . W1
        if ((rc = gemm_rm(s, t->gws, false, false, B, H, H, t->dU1[b], H, Pt(t_blk(b, 0)), H, t->dH, H, 1.f))) return rc;
    }
    // ---- input layer
    hipLaunchKernelGGL(k_inp_bwd<VPL>, rows, wave4, 0, s, t->dH, t->mask0, p, t->Z0, Pt(T_GIN), Pt(T_BEIN), t->mu0,
                       t->rs0, t->dZ0, t->rg0, t->rb0, B);
    YK_LAUNCHED();
    if ((rc = gemm_rm(s, t->gws, true, false, H, FEAT, B, t->dZ0, H, t->X, FEAT, Gt(T_WIN), FEAT, 0.f))) return rc;
    // ---- every bias / LayerNorm gradient: one launch of column sums
    hipLaunchKernelGGL(k_colsums, dim3(t->ntiles), dim3(256), 0, s, t->jobs, t->tiles, B);
    YK_LAUNCHED();
    return YK_OK;
}
}  // namespace

extern "C" {

int yk_trainer_create(yk_trainer_t** out, int H, int NB, const float* const* params, int nparams,
                      const yk_train_config_t* cfg) {
    if (!out || !params || !cfg) return YK_ERR_ARG;
    if (!(H == 64 || H == 128 || H == 256 || H == 512) || NB < 0 || NB > 64) return YK_ERR_ARG;
    if (nparams != 14 + 8 * NB || cfg->max_batch <= 0) return YK_ERR_ARG;
    if (!(cfg->dropout >= 0.0f && cfg->dropout < 1.0f)) return YK_ERR_ARG;
    if (cfg->amp) {
        // the mixed-precision step casts the Linear weights to fp16 (autocast): a finite weight with
        // |w| >= 65520 becomes inf there - every step's loss non-finite, every GradScaler step skipped
        // (torch's autocast path stalls the same way, silently); refused up front instead
        auto out_of_range = [](const float* w, long len) {
            for (long i = 0; i < len; i++)
                if (std::isfinite(w[i]) && std::fabs(w[i]) >= 65520.f) return true;
            return false;
        };
        if (out_of_range(params[0], (long)H * FEAT) || out_of_range(params[6 + 8 * NB], (long)ASIZE * H) ||
            out_of_range(params[10 + 8 * NB], 128L * H))
            return YK_ERR_RANGE;
        for (int b = 0; b < NB; b++)
            if (out_of_range(params[4 + 8 * b], (long)H * H) || out_of_range(params[8 + 8 * b], (long)H * H))
                return YK_ERR_RANGE;
    }
    yk_trainer* t = new yk_trainer();
    t->H = H;
    t->NB = NB;
    t->Bmax = cfg->max_batch;
    t->cfg = *cfg;
    // tensor sizes in state_dict order
    std::vector<long> n = {(long)H * FEAT, H, H, H};
    for (int b = 0; b < NB; b++)
        for (long x : {(long)H * H, (long)H, (long)H, (long)H, (long)H * H, (long)H, (long)H, (long)H}) n.push_back(x);
    for (long x : {(long)H, (long)H, (long)ASIZE * H, (long)ASIZE, (long)H, (long)H, (long)128 * H, 128L, 128L, 1L})
        n.push_back(x);
    long o = 0;
    for (long x : n) {
        t->off.push_back(o);
        t->len.push_back(x);
        o += x;
    }
    t->nparams = o;
    const size_t Bm = (size_t)t->Bmax, HH = (size_t)H;
    int rc = YK_OK;
#define TA(p, c) \
    if (rc == YK_OK) rc = talloc(t, &(p), (c))
    TA(t->P, o);
    TA(t->G, o);
    TA(t->M, o);
    TA(t->V, o);
    TA(t->X, Bm * FEAT);
    if (!cfg->amp) TA(t->gws, GEMM_WS);
    TA(t->tgt, Bm);
    TA(t->vt, Bm);
    TA(t->vout, Bm);
    TA(t->Z0, Bm * HH);
    TA(t->mu0, Bm);
    TA(t->rs0, Bm);
    TA(t->mask0, Bm * HH);
    t->Hs.assign(NB + 1, nullptr);
    for (int b = 0; b <= NB; b++) TA(t->Hs[b], Bm * HH);
    t->U1.assign(NB, nullptr); t->U2.assign(NB, nullptr); t->R1.assign(NB, nullptr);
    t->mu1.assign(NB, nullptr); t->rs1.assign(NB, nullptr); t->mu2.assign(NB, nullptr); t->rs2.assign(NB, nullptr);
    t->mask1.assign(NB, nullptr);
    for (int b = 0; b < NB; b++) {
        TA(t->U1[b], Bm * HH);
        TA(t->U2[b], Bm * HH);
        TA(t->R1[b], Bm * HH);
        TA(t->mu1[b], Bm);
        TA(t->rs1[b], Bm);
        TA(t->mu2[b], Bm);
        TA(t->rs2[b], Bm);
        TA(t->mask1[b], Bm * HH);
    }
    TA(t->Api, Bm * HH);
    TA(t->Av, Bm * HH);
    TA(t->mup, Bm); TA(t->rsp, Bm); TA(t->muv, Bm); TA(t->rsv, Bm);
    TA(t->logits, Bm * ASIZE);
    TA(t->dlogits, Bm * ASIZE);
    TA(t->Zv1, Bm * 128);
    TA(t->dZv1, Bm * 128);
    TA(t->dzv2, Bm);
    TA(t->dA, Bm * HH); TA(t->dAv, Bm * HH); TA(t->dH, Bm * HH); TA(t->dT, Bm * HH);
    TA(t->v2prod, Bm * 128);
    TA(t->rgp, Bm * HH); TA(t->rbp, Bm * HH); TA(t->rgv, Bm * HH); TA(t->rbv, Bm * HH);
    TA(t->dZ0, Bm * HH); TA(t->rg0, Bm * HH); TA(t->rb0, Bm * HH);
    t->dU1.assign(NB, nullptr); t->dU2.assign(NB, nullptr); t->rg1.assign(NB, nullptr); t->rb1.assign(NB, nullptr);
    t->rg2.assign(NB, nullptr); t->rb2.assign(NB, nullptr);
    for (int b = 0; b < NB; b++) {
        TA(t->dU1[b], Bm * HH); TA(t->dU2[b], Bm * HH); TA(t->rg1[b], Bm * HH); TA(t->rb1[b], Bm * HH);
        TA(t->rg2[b], Bm * HH); TA(t->rb2[b], Bm * HH);
    }
    TA(t->acc, 3);
    TA(t->sqpart, SQ_BLOCKS);
    TA(t->lrow, Bm);
    TA(t->lsum, 2);
    TA(t->eloss, 2);
    // the column-sum jobs: (row buffer, gradient tensor, width)
    std::vector<ColJob> jobs;
    if (rc == YK_OK) {
        auto G = [&](int k) { return t->G + t->off[k]; };
        jobs.push_back({t->dlogits, G(t_head(NB, 3)), ASIZE});
        jobs.push_back({t->dZv1, G(t_head(NB, 7)), 128});
        jobs.push_back({t->v2prod, G(t_head(NB, 8)), 128});
        jobs.push_back({t->dzv2, G(t_head(NB, 9)), 1});
        jobs.push_back({t->rgp, G(t_head(NB, 0)), H});
        jobs.push_back({t->rbp, G(t_head(NB, 1)), H});
        jobs.push_back({t->rgv, G(t_head(NB, 4)), H});
        jobs.push_back({t->rbv, G(t_head(NB, 5)), H});
        for (int b = 0; b < NB; b++) {
            jobs.push_back({t->dU1[b], G(t_blk(b, 1)), H});
            jobs.push_back({t->rg1[b], G(t_blk(b, 2)), H});
            jobs.push_back({t->rb1[b], G(t_blk(b, 3)), H});
            jobs.push_back({t->dU2[b], G(t_blk(b, 5)), H});
            jobs.push_back({t->rg2[b], G(t_blk(b, 6)), H});
            jobs.push_back({t->rb2[b], G(t_blk(b, 7)), H});
        }
        jobs.push_back({t->dZ0, G(T_BIN), H});
        jobs.push_back({reinterpret_cast<const float*>(t->lrow), t->lsum, 2});  // the batch's two loss sums
        jobs.push_back({t->rg0, G(T_GIN), H});
        jobs.push_back({t->rb0, G(T_BEIN), H});
    }
    std::vector<int2> tiles;
    for (size_t j = 0; j < jobs.size(); j++)
        for (int c = 0; c < jobs[j].N; c += 16) tiles.push_back(make_int2((int)j, c));
    t->ntiles = (int)tiles.size();
    TA(t->jobs, jobs.size());
    TA(t->tiles, tiles.size());
    if (rc == YK_OK) {
        (void)hipMemcpy(t->jobs, jobs.data(), sizeof(ColJob) * jobs.size(), hipMemcpyHostToDevice);
        (void)hipMemcpy(t->tiles, tiles.data(), sizeof(int2) * tiles.size(), hipMemcpyHostToDevice);
    }
#undef TA
    if (rc != YK_OK) {
        yk_trainer_destroy(t);
        return rc;
    }
    for (size_t k = 0; k < n.size(); k++)
        if (hipMemcpy(t->P + t->off[k], params[k], sizeof(float) * t->len[k], hipMemcpyHostToDevice) != hipSuccess) {
            yk_trainer_destroy(t);
            return YK_ERR_HIP;
        }
    (void)hipMemset(t->M, 0, sizeof(float) * o);
    (void)hipMemset(t->V, 0, sizeof(float) * o);
    (void)hipMemset(t->G, 0, sizeof(float) * o);
    (void)hipMemset(t->acc, 0, sizeof(double) * 3);
    (void)hipMemset(t->lsum, 0, sizeof(float) * 2);
    if (cfg->amp) {
        if ((rc = yk::amp_create(&t->amp, H, NB, t->Bmax, t->P, t->G, t->off.data(), cfg->init_scale,
                                 cfg->growth_interval)) != YK_OK ||
            (rc = yk::amp_pack(t->amp, 0)) != YK_OK) {
            yk_trainer_destroy(t);
            return rc;
        }
    }
    if (hipDeviceSynchronize() != hipSuccess) {
        yk_trainer_destroy(t);
        return YK_ERR_HIP;
    }
    *out = t;
    return YK_OK;
}

int yk_trainer_destroy(yk_trainer_t* t) {
    if (!t) return YK_OK;
    yk::amp_destroy(t->amp);
    for (void* p : t->allocs) (void)hipFree(p);
    delete t;
    return YK_OK;
}

int yk_trainer_buffers(yk_trainer_t* t, float** params, float** grads, int64_t* nparams) {
    if (!t) return YK_ERR_ARG;
    if (params) *params = t->P;
    if (grads) *grads = t->G;
    if (nparams) *nparams = t->nparams;
    return YK_OK;
}

static int backward_impl(yk_trainer_t* t, const yk_state_t* states, const int32_t* targets, const float* values,
                         const int32_t* batch_idx, int batch, bool fuse_norm, hipStream_t s) {
    if (t->amp)
        return yk::amp_backward(t->amp, states, targets, values, batch_idx, batch, t->cfg.dropout, t->cfg.seed, t->step,
                                t->row_base, t->cfg.vloss_weight, t->lrow, t->lsum, fuse_norm, s);
    switch (t->H) {
        case 64: return step_impl<1>(t, states, targets, values, batch_idx, batch, s);
        case 128: return step_impl<2>(t, states, targets, values, batch_idx, batch, s);
        case 256: return step_impl<4>(t, states, targets, values, batch_idx, batch, s);
        case 512: return step_impl<8>(t, states, targets, values, batch_idx, batch, s);
    }
    return YK_ERR_ARG;
}

// one report epoch's running loss, kept on the device so a reporting epoch takes no host
// round trip per minibatch: += ce/b + vw*se/b, in the order NNet.py:150-152's float sum takes
__global__ void k_epoch_loss(const float* lsum, double* eloss, double b, double vw) {
    if (threadIdx.x == 0) {
        eloss[0] += (double)lsum[0] / b + vw * (double)lsum[1] / b;
        eloss[1] += 1.0;
    }
}

static int backward_call(yk_trainer_t* t, const yk_state_t* states, const int32_t* targets, const float* values,
                         const int32_t* batch_idx, int batch, bool fuse_norm, void* stream) {
    if (!t || !states || !targets || !values) return YK_ERR_ARG;
    if (batch <= 0 || batch > t->Bmax) return YK_ERR_ARG;
    hipStream_t s = as_stream(stream);
    int rc = backward_impl(t, states, targets, values, batch_idx, batch, fuse_norm, s);
    t->row_base = 0;  // the offset applies to the one backward it was set for (yk_trainer_set_row_offset)
    if (rc == YK_OK && t->eloss_on) {
        hipLaunchKernelGGL(k_epoch_loss, dim3(1), dim3(64), 0, s, t->lsum, t->eloss, (double)batch, t->eloss_vw);
        YK_LAUNCHED();
    }
    return rc;
}

int yk_trainer_backward(yk_trainer_t* t, const yk_state_t* states, const int32_t* targets, const float* values,
                        const int32_t* batch_idx, int batch, void* stream) {
    return backward_call(t, states, targets, values, batch_idx, batch, false, stream);
}

int yk_trainer_epoch_loss_begin(yk_trainer_t* t, double vloss_weight) {
    if (!t) return YK_ERR_ARG;
    YK_HIP(hipMemset(t->eloss, 0, sizeof(double) * 2));
    t->eloss_on = true;
    t->eloss_vw = vloss_weight;
    return YK_OK;
}

int yk_trainer_epoch_loss_end(yk_trainer_t* t, double* out) {
    if (!t || !out) return YK_ERR_ARG;
    t->eloss_on = false;
    YK_HIP(hipDeviceSynchronize());
    YK_HIP(hipMemcpy(out, t->eloss, sizeof(double) * 2, hipMemcpyDeviceToHost));
    return YK_OK;
}

int yk_trainer_apply(yk_trainer_t* t, void* stream) {
    if (!t) return YK_ERR_ARG;
    hipStream_t s = as_stream(stream);
    t->step += 1;  // (amp: the dropout stream's step; the optimiser's count of steps taken is on the device)
    if (t->amp)
        return yk::amp_apply(t->amp, t->nparams, t->M, t->V, t->acc + 2, t->cfg.max_grad_norm, t->cfg.lr,
                             t->cfg.weight_decay, t->cfg.beta1, t->cfg.beta2, t->cfg.eps, t->cfg.dropout, t->cfg.seed,
                             t->step, s);
    const double b1 = t->cfg.beta1, b2 = t->cfg.beta2, st = (double)t->step;
    const double bc1 = 1.0 - std::pow(b1, st), bc2 = 1.0 - std::pow(b2, st);
    const float step_size = (float)(t->cfg.lr / bc1), bc2_sqrt = (float)std::sqrt(bc2);
    hipLaunchKernelGGL(k_sqnorm, dim3(SQ_BLOCKS), dim3(TPB), 0, s, t->G, t->nparams, t->sqpart);
    YK_LAUNCHED();
    hipLaunchKernelGGL(k_adamw, dim3(2048), dim3(TPB), 0, s, t->P, t->G, t->M, t->V, t->nparams, t->sqpart, t->acc + 2,
                       t->cfg.max_grad_norm, t->cfg.lr, t->cfg.weight_decay, t->cfg.beta1, t->cfg.beta2, t->cfg.eps,
                       step_size, bc2_sqrt);
    YK_LAUNCHED();
    return YK_OK;
}

int yk_trainer_step(yk_trainer_t* t, const yk_state_t* states, const int32_t* targets, const float* values,
                    const int32_t* batch_idx, int batch, void* stream) {
    // (one call, nothing between backward and apply: the gradient launches sum the norm themselves)
    int rc = backward_call(t, states, targets, values, batch_idx, batch, true, stream);
    if (rc) return rc;
    return yk_trainer_apply(t, stream);
}

int yk_trainer_losses(yk_trainer_t* t, double* out) {
    if (!t || !out) return YK_ERR_ARG;
    YK_HIP(hipDeviceSynchronize());
    YK_HIP(hipMemcpy(out, t->acc, sizeof(double) * 3, hipMemcpyDeviceToHost));
    float ls[2];
    YK_HIP(hipMemcpy(ls, t->lsum, sizeof(ls), hipMemcpyDeviceToHost));
    out[0] = ls[0];
    out[1] = ls[1];
    return YK_OK;
}

int yk_trainer_get(yk_trainer_t* t, int which, float* const* out) {
    if (!t || !out || which < 0 || which > 3) return YK_ERR_ARG;
    const float* src = which == 0 ? t->P : which == 1 ? t->G : which == 2 ? t->M : t->V;
    YK_HIP(hipDeviceSynchronize());
    for (size_t k = 0; k < t->off.size(); k++)
        if (out[k]) YK_HIP(hipMemcpy(out[k], src + t->off[k], sizeof(float) * t->len[k], hipMemcpyDeviceToHost));
    return YK_OK;
}

int yk_trainer_set(yk_trainer_t* t, int which, const float* const* in, int64_t step) {
    if (!t || !in || which < 0 || which > 3) return YK_ERR_ARG;
    float* dst = which == 0 ? t->P : which == 1 ? t->G : which == 2 ? t->M : t->V;
    for (size_t k = 0; k < t->off.size(); k++)
        if (in[k]) YK_HIP(hipMemcpy(dst + t->off[k], in[k], sizeof(float) * t->len[k], hipMemcpyHostToDevice));
    if (step >= 0) t->step = (uint64_t)step;
    if (t->amp) {
        if (step >= 0) {
            const int rc = yk::amp_set_steps(t->amp, step);
            if (rc) return rc;
        }
        if (which == 0) {  // new parameters: new fp16 copies
            const int rc = yk::amp_pack(t->amp, 0);
            if (rc) return rc;
        }
    }
    YK_HIP(hipDeviceSynchronize());
    return YK_OK;
}

int64_t yk_trainer_step_count(yk_trainer_t* t) {
    if (!t) return YK_ERR_ARG;
    return t->amp ? yk::amp_steps(t->amp) : (int64_t)t->step;
}

int yk_trainer_set_row_offset(yk_trainer_t* t, int64_t row0) {
    if (!t || row0 < 0) return YK_ERR_ARG;
    t->row_base = row0;
    return YK_OK;
}

int yk_trainer_amp_state(yk_trainer_t* t, double* out) {
    if (!t || !out || !t->amp) return YK_ERR_ARG;
    return yk::amp_state(t->amp, out);
}

}  // extern "C"
