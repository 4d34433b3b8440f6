// yk_net.hip - NNetWrapper.predict (yacht/NNet.py:177-195) over YachtNNet
// (yacht/pytorch/YachtNNet.py:8-70), batched over all pending leaves, float32.
//
// Two kernels carry the FLOPs (3,320,576 per row at H=256, 6 blocks):
//  * k_trunk: one 256-thread workgroup per 16 rows keeps the whole activation tile in
//    LDS across all 13 dense layers (featurize -> Linear/LN/SiLU -> 6 x ResidualBlock ->
//    head LayerNorms -> value head).  Each dense layer is [16 x K] x [K x N] on
//    v_mfma_f32_16x16x4_f32; the four waves split N; weights stream from L2.
//  * k_pihead: logits = a_pi @ W_pi^T + b over 64 x 64 output tiles (f32 MFMA).
// f32-in MFMA is exact f32 (fmaf chain), so results track torch's float32 CPU path
// within the 1e-5 tolerance of the north star (tests/test_gpu_net.py).
#include <vector>

#include "yk_api.h"
#include "yk_common.h"
#include "yk_net.h"

using namespace yk;

typedef float floatx4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int ROWS = 16;  // rows per trunk workgroup
constexpr int FPAD = 68;  // feature tile row stride (64 + 4)

__device__ __forceinline__ float silu(float x) { return x / (1.0f + expf(-x)); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// acc[t] += A[16 x K] (LDS, row stride lda) x W[n0 + 16t .. +16][K]^T (global, row stride ldw)
// Lane l supplies A[l&15][k0 + 4(l>>4) + i] and W[.][k0 + 4(l>>4) + i] to MFMA i of each
// 16-deep k-block, so each lane's operands are one float4 from each source.
template <int K, int NT>
__device__ __forceinline__ void gemm16(const float* A, int lda, const float* __restrict__ W, int ldw, int n0,
                                       floatx4 (&acc)[NT]) {
    const int lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
#pragma unroll
    for (int t = 0; t < NT; t++) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    const float* wrow[NT];
#pragma unroll
    for (int t = 0; t < NT; t++) wrow[t] = W + (long)(n0 + 16 * t + r) * ldw + 4 * q;
#pragma unroll 2
    for (int k0 = 0; k0 < K; k0 += 16) {
        const float4 a = *reinterpret_cast<const float4*>(A + r * lda + k0 + 4 * q);
        float4 b[NT];
#pragma unroll
        for (int t = 0; t < NT; t++) b[t] = *reinterpret_cast<const float4*>(wrow[t] + k0);
#pragma unroll
        for (int t = 0; t < NT; t++) {
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b[t].x, acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b[t].y, acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b[t].z, acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b[t].w, acc[t], 0, 0, 0);
        }
    }
}

// D[16 x 16] tile t of the wave: lane holds rows 4(l>>4)+j, column n0 + 16t + (l&15)
template <int NT>
__device__ __forceinline__ void store_acc(float* D, int ldd, int n0, const floatx4 (&acc)[NT],
                                          const float* __restrict__ bias) {
    const int lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
#pragma unroll
    for (int t = 0; t < NT; t++) {
        const int c = n0 + 16 * t + r;
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

template <int H>
__global__ __launch_bounds__(256) void k_trunk(NetDev net, const yk_state_t* __restrict__ states,
                                              const float* __restrict__ xin, const int32_t* __restrict__ rows,
                                              const int32_t* __restrict__ count, int n, float* __restrict__ a_pi,
                                              float* __restrict__ vout) {
    constexpr int LD = (H > 128 ? H : 128) + 4;  // X also holds the 128-wide v_head hidden
    constexpr int NT = H / 64;  // 16-col tiles per wave (4 waves split H)
    constexpr int VPL = H / 64; // values per lane in row passes
    __shared__ __attribute__((aligned(16))) float X[ROWS * LD];
    __shared__ __attribute__((aligned(16))) float T[ROWS * LD];
    __shared__ __attribute__((aligned(16))) float F[ROWS * FPAD];

    if (count) n = min(n, *count);
    const int row0 = blockIdx.x * ROWS;
    if (row0 >= n) return;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;

    // featurize (state_to_vec, NNet.py:65-86), zero padded to K = 64
    for (int idx = tid; idx < ROWS * 64; idx += 256) {
        const int r = idx >> 6, f = idx & 63;
        const int row = row0 + r;
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
        F[r * FPAD + f] = val;
    }
    __syncthreads();

    const int n0 = wave * (H / 4);
    floatx4 acc[NT];
    // inp: Linear -> LayerNorm -> SiLU (-> Dropout, identity in eval)  YachtNNet.py:30-35
    gemm16<64, NT>(F, FPAD, net.w_in, 64, n0, acc);
    store_acc<NT>(T, LD, n0, acc, net.b_in);
    __syncthreads();
    for (int rr = 0; rr < 4; rr++) {
        const int r = wave * 4 + rr;
        float x[VPL];
#pragma unroll
        for (int i = 0; i < VPL; i++) x[i] = T[r * LD + lane * VPL + i];
        layernorm<VPL>(x, net.g_in, net.be_in, lane * VPL, H);
#pragma unroll
        for (int i = 0; i < VPL; i++) X[r * LD + lane * VPL + i] = silu(x[i]);
    }
    __syncthreads();

    // ResidualBlock x NB: h = LN1(SiLU(fc1 x)); h = LN2(SiLU(fc2 h)); x + h  YachtNNet.py:17-21
    for (int b = 0; b < net.NB; b++) {
        const long wo = (long)b * H * H, bo = (long)b * H;
        gemm16<H, NT>(X, LD, net.w1 + wo, H, n0, acc);
        store_acc<NT>(T, LD, n0, acc, net.b1 + bo);
        __syncthreads();
        for (int rr = 0; rr < 4; rr++) {
            const int r = wave * 4 + rr;
            float x[VPL];
#pragma unroll
            for (int i = 0; i < VPL; i++) x[i] = silu(T[r * LD + lane * VPL + i]);
            layernorm<VPL>(x, net.g1 + bo, net.be1 + bo, lane * VPL, H);
#pragma unroll
            for (int i = 0; i < VPL; i++) T[r * LD + lane * VPL + i] = x[i];
        }
        __syncthreads();
        gemm16<H, NT>(T, LD, net.w2 + wo, H, n0, acc);
        __syncthreads();
        store_acc<NT>(T, LD, n0, acc, net.b2 + bo);
        __syncthreads();
        for (int rr = 0; rr < 4; rr++) {
            const int r = wave * 4 + rr;
            float x[VPL];
#pragma unroll
            for (int i = 0; i < VPL; i++) x[i] = silu(T[r * LD + lane * VPL + i]);
            layernorm<VPL>(x, net.g2 + bo, net.be2 + bo, lane * VPL, H);
#pragma unroll
            for (int i = 0; i < VPL; i++) X[r * LD + lane * VPL + i] += x[i];
        }
        __syncthreads();
    }

    // heads: pi_head = LN -> SiLU -> (Linear in k_pihead); v_head = LN -> SiLU -> ...
    for (int rr = 0; rr < 4; rr++) {
        const int r = wave * 4 + rr;
        const int row = row0 + r;
        float x[VPL], y[VPL];
#pragma unroll
        for (int i = 0; i < VPL; i++) x[i] = y[i] = X[r * LD + lane * VPL + i];
        layernorm<VPL>(x, net.g_pi, net.be_pi, lane * VPL, H);
        layernorm<VPL>(y, net.g_v, net.be_v, lane * VPL, H);
        if (row < n) {
#pragma unroll
            for (int i = 0; i < VPL; i++) a_pi[(long)row * H + lane * VPL + i] = silu(x[i]);
        }
#pragma unroll
        for (int i = 0; i < VPL; i++) T[r * LD + lane * VPL + i] = silu(y[i]);
    }
    __syncthreads();
    {  // v_head.2: Linear(H, 128), 4 waves x 32 columns
        floatx4 av[2];
        gemm16<H, 2>(T, LD, net.w_v1, H, wave * 32, av);
        store_acc<2>(X, LD, wave * 32, av, net.b_v1);
    }
    __syncthreads();
    for (int rr = 0; rr < 4; rr++) {  // SiLU -> Linear(128, 1) -> tanh  YachtNNet.py:49-52,69
        const int r = wave * 4 + rr;
        const int row = row0 + r;
        float s = silu(X[r * LD + 2 * lane]) * net.w_v2[2 * lane] + silu(X[r * LD + 2 * lane + 1]) * net.w_v2[2 * lane + 1];
        s = wave_sum(s);
        if (lane == 0 && row < n) vout[row] = tanhf(s + net.b_v2[0]);
    }
}

// logits tile 64 x 64 per workgroup; wave w owns rows 16w..16w+15, four 16-col tiles
template <int H>
__global__ __launch_bounds__(256) void k_pihead(NetDev net, const float* __restrict__ a_pi,
                                               const int32_t* __restrict__ count, int n, float* __restrict__ logits) {
    if (count) n = min(n, *count);
    const int rb = blockIdx.y * 64;
    if (rb >= n) return;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
    const int c0 = blockIdx.x * 64;
    const int row_a = min(rb + wave * 16 + r, n - 1);
    const float* arow = a_pi + (long)row_a * H + 4 * q;
    const float* wrow[4];
#pragma unroll
    for (int t = 0; t < 4; t++) wrow[t] = net.w_pi + (long)(c0 + 16 * t + r) * H + 4 * q;
    floatx4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; t++) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
    for (int k0 = 0; k0 < H; k0 += 16) {
        const float4 a = *reinterpret_cast<const float4*>(arow + k0);
        float4 b[4];
#pragma unroll
        for (int t = 0; t < 4; t++) b[t] = *reinterpret_cast<const float4*>(wrow[t] + k0);
#pragma unroll
        for (int t = 0; t < 4; t++) {
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b[t].x, acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b[t].y, acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b[t].z, acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b[t].w, acc[t], 0, 0, 0);
        }
    }
#pragma unroll
    for (int t = 0; t < 4; t++) {
        const int c = c0 + 16 * t + r;
        const float b = net.b_pi[c];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int row = rb + wave * 16 + 4 * q + j;
            if (row < n) logits[(long)row * PI_LD + c] = acc[t][j] + b;
        }
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

int launch_trunk(const NetDev& net, const yk_state_t* states, const float* x, const int32_t* rows,
                 const int32_t* count, int n, float* a_pi, float* v, hipStream_t stream) {
    if (n <= 0) return YK_OK;
    const dim3 grid((n + ROWS - 1) / ROWS), block(256);
    switch (net.H) {
        case 64: hipLaunchKernelGGL(k_trunk<64>, grid, block, 0, stream, net, states, x, rows, count, n, a_pi, v); break;
        case 128: hipLaunchKernelGGL(k_trunk<128>, grid, block, 0, stream, net, states, x, rows, count, n, a_pi, v); break;
        case 256: hipLaunchKernelGGL(k_trunk<256>, grid, block, 0, stream, net, states, x, rows, count, n, a_pi, v); break;
        case 512: hipLaunchKernelGGL(k_trunk<512>, grid, block, 0, stream, net, states, x, rows, count, n, a_pi, v); break;
        default: return YK_ERR_ARG;
    }
    YK_LAUNCHED();
    return YK_OK;
}

int launch_pihead(const NetDev& net, const float* a_pi, const int32_t* count, int n, float* logits,
                  hipStream_t stream) {
    if (n <= 0) return YK_OK;
    const dim3 grid(PI_LD / 64, (n + 63) / 64), block(256);
    switch (net.H) {
        case 64: hipLaunchKernelGGL(k_pihead<64>, grid, block, 0, stream, net, a_pi, count, n, logits); break;
        case 128: hipLaunchKernelGGL(k_pihead<128>, grid, block, 0, stream, net, a_pi, count, n, logits); break;
        case 256: hipLaunchKernelGGL(k_pihead<256>, grid, block, 0, stream, net, a_pi, count, n, logits); break;
        case 512: hipLaunchKernelGGL(k_pihead<512>, grid, block, 0, stream, net, a_pi, count, n, logits); break;
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
    // host staging of the device layout
    std::vector<float> h;
    auto put = [&](size_t n) { size_t o = h.size(); h.resize(o + ((n + 63) / 64) * 64, 0.f); return o; };
    const size_t o_win = put((size_t)H * 64), o_bin = put(H), o_gin = put(H), o_bein = put(H);
    const size_t o_w1 = put((size_t)NB * H * H), o_b1 = put((size_t)NB * H), o_g1 = put((size_t)NB * H),
                 o_be1 = put((size_t)NB * H);
    const size_t o_w2 = put((size_t)NB * H * H), o_b2 = put((size_t)NB * H), o_g2 = put((size_t)NB * H),
                 o_be2 = put((size_t)NB * H);
    const size_t o_gpi = put(H), o_bepi = put(H), o_wpi = put((size_t)PI_LD * H), o_bpi = put(PI_LD);
    const size_t o_gv = put(H), o_bev = put(H), o_wv1 = put((size_t)128 * H), o_bv1 = put(128), o_wv2 = put(128),
                 o_bv2 = put(1);
    int k = 0;
    for (int o = 0; o < H; o++)
        for (int i = 0; i < FEAT; i++) h[o_win + (size_t)o * 64 + i] = p[k][(size_t)o * FEAT + i];
    k++;
    auto cp = [&](size_t off, size_t n) { std::copy(p[k], p[k] + n, h.begin() + off); k++; };
    cp(o_bin, H); cp(o_gin, H); cp(o_bein, H);
    for (int b = 0; b < NB; b++) {
        cp(o_w1 + (size_t)b * H * H, (size_t)H * H); cp(o_b1 + (size_t)b * H, H);
        cp(o_g1 + (size_t)b * H, H); cp(o_be1 + (size_t)b * H, H);
        cp(o_w2 + (size_t)b * H * H, (size_t)H * H); cp(o_b2 + (size_t)b * H, H);
        cp(o_g2 + (size_t)b * H, H); cp(o_be2 + (size_t)b * H, H);
    }
    cp(o_gpi, H); cp(o_bepi, H); cp(o_wpi, (size_t)ASIZE * H); cp(o_bpi, ASIZE);
    cp(o_gv, H); cp(o_bev, H); cp(o_wv1, (size_t)128 * H); cp(o_bv1, 128); cp(o_wv2, 128); cp(o_bv2, 1);

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
    float *a_pi = nullptr, *logits = nullptr;
    YK_HIP(hipMallocAsync((void**)&a_pi, sizeof(float) * (size_t)n * net->dev.H, s));
    YK_HIP(hipMallocAsync((void**)&logits, sizeof(float) * (size_t)n * PI_LD, s));
    int rc = launch_trunk(net->dev, states, x, nullptr, nullptr, n, a_pi, v, s);
    if (rc == YK_OK) rc = launch_pihead(net->dev, a_pi, nullptr, n, logits, s);
    if (rc == YK_OK) rc = launch_softmax(logits, pi, n, s);
    (void)hipFreeAsync(a_pi, s);
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
