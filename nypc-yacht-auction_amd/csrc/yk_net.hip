// yk_net.hip - NNetWrapper.predict (yacht/NNet.py:177-195) over YachtNNet
// (yacht/pytorch/YachtNNet.py:8-70), batched over all pending leaves, f32-equivalent.
//
// One kernel, k_forward, carries all 3,320,576 FLOP per row (hidden 256, 6 blocks): a
// 512-thread workgroup (8 waves, 2 per SIMD, up to 256 VGPRs each) owns 16 rows and keeps
// their activations in LDS through featurize -> Linear/LN/SiLU -> 6 x ResidualBlock -> head
// LayerNorms -> value head and policy logits (204 x 16 columns).  Every dense product is
// f32-equivalent: weights and GEMM inputs are held as fp16 planes hi = fp16(x) and
// lo = fp16((x - hi) 2^11), and a 16x16x32 tile is hi*hi + 2^-11 (hi*lo + lo*hi + (lo 2^-11)*lo) -
// four v_mfma_f32_16x16x32_f16 with exact products and f32 accumulation (the lo*lo term, 2^-22
// relative, enters the cross-term accumulator through an fp16 operand lo * 2^-11; dropping it
// doubled the prior's error against float64, tools/prior_error_emulation.py).  Results track
// torch's float32 path within the north star's 1e-5 (tests/test_gpu_net.py) at 1/4 of the MFMA
// cycles of v_mfma_f32_16x16x4_f32.
//
// The kernel is latency-bound per workgroup (one per CU), and on this chip a CU does not
// overlap MFMA execution with its vector-memory stream (tools/stream_bench.hip), so the weight
// stream must never stop and the MFMA time must be small: weights are pre-packed in MFMA
// fragment order (yk_net.h), each wave keeps a ring of W slices of its fragments in registers,
// and as soon as a slice is consumed its registers are refilled with the slice W ahead - across
// layer boundaries, so the
// next layer streams in under the current GEMM and the LayerNorm phase.  Nothing the kernel
// waits on is ever issued behind that stream (vmcnt retires in order): biases and LayerNorm
// vectors live in LDS, and the kernel must not spill (scratch also counts in vmcnt).
#include <algorithm>
#include <cmath>
#include <vector>

#include "yk_api.h"
#include "yk_common.h"
#include "yk_net.h"

using namespace yk;

#include "yk_fwd.h"

using namespace ykf;

namespace {

template <int H, int PL, bool NB0 = false>
__global__ __launch_bounds__(NTHR) void k_forward(NetDev net, const yk_state_t* __restrict__ states,
                                                 const float* __restrict__ xin, const int32_t* __restrict__ rows,
                                                 const int32_t* __restrict__ count, int n,
                                                 float* __restrict__ logits, float* __restrict__ vout,
                                                 const uint8_t* __restrict__ active, float2* __restrict__ mlse,
                                                 int valid_only, uint32_t want, int parts, int mstride) {
    // head split (parts > 1): `parts` workgroups share a 16-row tile; each runs the trunk and the
    // value head and the policy head over its slice of the tile list, and writes its raw partial
    // (max, sum exp) to mlse[part * mstride + row] (the consumer merges them); part 0 writes v
    if (count) n = min(n, *count);
    const int part = (int)(blockIdx.x % (unsigned)parts);
    const int row0 = (int)(blockIdx.x / (unsigned)parts) * ROWS;
    forward_tile<H, PL, WAVES, NB0>(net, states, xin, rows, nullptr, n, logits, vout, active, mlse, valid_only, want,
                               parts, mstride, row0, part);
}

// exp(log_softmax(x)) over the first 3226 columns from the forward's per-row (max, log sum
// exp): one wavefront per row
__global__ void k_softmax(const float* __restrict__ logits, const float2* __restrict__ mlse, float* __restrict__ pi,
                          int n) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= n) return;
    const float* x = logits + (long)row * PI_LD;
    const float2 ml = mlse[row];
    for (int a = lane; a < ASIZE; a += 64) pi[(long)row * ASIZE + a] = expf(x[a] - ml.x - ml.y);
}

// The engine's leaf prior before renormalisation (yk_selfplay's expand, MCTS.py:86-88): at the
// row's valid actions (player 1 of the canonical state) exp(x - m - l) from the forward's row
// statistics, with the expand's hardware exp, 0 elsewhere.  One wavefront per row.
__global__ void k_leaf_prior(const float* __restrict__ logits, const float2* __restrict__ mlse,
                             const yk_state_t* __restrict__ states, float* __restrict__ pi, int n) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= n) return;
    YkS s;
#pragma unroll
    for (int k = 0; k < 8; k++) s.w[k] = states[row].w[k];
    const float* x = logits + (long)row * PI_LD;
    const float2 ml = mlse[row];
    for (int a = lane; a < ASIZE; a += 64)
        pi[(long)row * ASIZE + a] = action_valid(s, 1, a) ? exp_acc(x[a] - ml.x - ml.y) : 0.f;  // the expand's exp
}

// The submission bot's move (agent.py:248-280): softmax over all 3226 logits in f32, then the
// most probable *decodable* action (agent.py:150-187 == getValidMoves for the mover p1,
// YachtGame.py:375-400), the lowest index among equal probabilities (its stable descending
// sort).  One wavefront per row; -1 when the row has no valid action.
__global__ void k_policy_pick(const float* __restrict__ logits, const yk_state_t* __restrict__ states,
                              int32_t* __restrict__ actions, float* __restrict__ probs, int n) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= n) return;
    const float* x = logits + (long)row * PI_LD;
    YkS s;
#pragma unroll
    for (int k = 0; k < 8; k++) s.w[k] = states[row].w[k];
    float m = -INFINITY;
    for (int a = lane; a < ASIZE; a += 64) m = fmaxf(m, x[a]);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    float sum = 0.f;
    for (int a = lane; a < ASIZE; a += 64) sum += expf(x[a] - m);
    sum = wave_sum(sum);
    float bp = -1.f;
    int ba = INT_MAX;
    for (int a = lane; a < ASIZE; a += 64) {  // ascending per lane: strict > keeps the first
        if (!action_valid(s, 1, a)) continue;
        const float p = expf(x[a] - m) / sum;
        if (p > bp) { bp = p; ba = a; }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const float op = __shfl_xor(bp, o, 64);
        const int oa = __shfl_xor(ba, o, 64);
        if (op > bp || (op == bp && oa < ba)) { bp = op; ba = oa; }
    }
    if (lane == 0) {
        actions[row] = ba == INT_MAX ? -1 : ba;
        if (probs) probs[row] = ba == INT_MAX ? 0.f : bp;
    }
}

}  // namespace

namespace yk {

int launch_forward(const NetDev& net, const yk_state_t* states, const float* x, const int32_t* rows,
                   const int32_t* count, int n, float* logits, float* v, hipStream_t stream, const uint8_t* active,
                   float2* mlse, bool valid_only, uint8_t want, int parts, int mstride) {
    if (n <= 0) return YK_OK;
    if (parts < 1 || parts > 4 || (parts > 1 && (!mlse || mstride < n))) return YK_ERR_ARG;
    const dim3 grid((unsigned)((n + ROWS - 1) / ROWS * parts)), block(NTHR);
    const int vo = valid_only ? 1 : 0;
#define YK_FWD1(HH, PP, Z) hipLaunchKernelGGL((k_forward<HH, PP, Z>), grid, block, 0, stream, net, states, x, rows, count, \
                                               n, logits, v, active, mlse, vo, (uint32_t)want, parts, mstride)
#define YK_FWD(HH, PP) \
    if (net.NB == 0) YK_FWD1(HH, PP, true); else YK_FWD1(HH, PP, false)
    const bool f16 = net.planes == 1;
    switch (net.H) {
        case 64: if (f16) { YK_FWD(64, 1); } else { YK_FWD(64, 2); } break;
        case 128: if (f16) { YK_FWD(128, 1); } else { YK_FWD(128, 2); } break;
        case 256: if (f16) { YK_FWD(256, 1); } else { YK_FWD(256, 2); } break;
        case 512: if (f16) { YK_FWD(512, 1); } else { YK_FWD(512, 2); } break;
        default: return YK_ERR_ARG;
    }
#undef YK_FWD
#undef YK_FWD1
    YK_LAUNCHED();
    return YK_OK;
}

int launch_softmax(const float* logits, const float2* mlse, float* pi, int n, hipStream_t stream) {
    if (n <= 0) return YK_OK;
    hipLaunchKernelGGL(k_softmax, dim3((n + 3) / 4), dim3(256), 0, stream, logits, mlse, pi, n);
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
    // torch [N][K] row-major (K valid columns) -> fp16 hi / lo planes in MFMA fragment order
    // (yk_net.h), N padded to Np, K to Kp; same footprint as the f32 matrix
    auto pack = [&](size_t dst, const float* W, int N, int K, int Np, int Kp) {
        const int KSp = Kp / 32;
        _Float16* o = reinterpret_cast<_Float16*>(h.data() + dst);
        for (int nt = 0; nt < Np / 16; nt++)
            for (int ks = 0; ks < KSp; ks++)
                for (int l = 0; l < 64; l++)
                    for (int j = 0; j < 8; j++) {
                        const int nn = 16 * nt + (l & 15), kk = 32 * ks + 8 * (l >> 4) + j;
                        const float x = (nn < N && kk < K) ? W[(size_t)nn * K + kk] : 0.f;
                        const _Float16 hi = (_Float16)x;
                        const _Float16 lo = (_Float16)((x - (float)hi) * SPLIT);
                        const size_t base = (((size_t)nt * KSp + ks) * 2 * 64 + l) * 8 + j;
                        o[base] = hi;
                        o[base + 64 * 8] = lo;
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
    const size_t o_vs = put(vstat_size(H)), o_vb = put((size_t)NB * 6 * H);
    const size_t o_err = put(1);  // the forwards' check flags (a uint32 word, zeroed below)
    // the f32-equivalent split's range: hi = fp16(w) must be finite for every finite weight of the
    // packed (MFMA) matrices - |w| >= 65520 rounds to inf, where torch's float32 holds a number
    {
        const int mats[4] = {0, 6 + 8 * NB, 10 + 8 * NB, -1};
        const size_t mlen[3] = {(size_t)H * FEAT, (size_t)ASIZE * H, (size_t)128 * H};
        auto out_of_range = [](const float* w, size_t n) {
            for (size_t i = 0; i < n; i++)
                if (std::isfinite(w[i]) && std::fabs(w[i]) >= 65520.f) return true;
            return false;
        };
        for (int m = 0; mats[m] >= 0; m++)
            if (out_of_range(p[mats[m]], mlen[m])) return YK_ERR_RANGE;
        for (int b = 0; b < NB; b++)
            if (out_of_range(p[4 + 8 * b], (size_t)H * H) || out_of_range(p[8 + 8 * b], (size_t)H * H))
                return YK_ERR_RANGE;
    }
    // pi_head.2 bounds for the valid-only softmax (k_forward): bias spread, largest weight-row norm
    float pi_bmin = INFINITY, pi_bmax = -INFINITY, pi_wmax = 0.f;
    {
        const float* wpi = p[6 + 8 * NB];
        const float* bpi = p[7 + 8 * NB];
        for (int a = 0; a < ASIZE; a++) {
            pi_bmin = std::min(pi_bmin, bpi[a]);
            pi_bmax = std::max(pi_bmax, bpi[a]);
            double n2 = 0.0;
            for (int i = 0; i < H; i++) n2 += (double)wpi[(size_t)a * H + i] * wpi[(size_t)a * H + i];
            pi_wmax = std::max(pi_wmax, (float)std::sqrt(n2));
        }
    }
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
    // LDS-staged copies of the vectors (yk_net.h): static set, then per block b1 g1 be1 b2 g2 be2
    auto dup = [&](size_t dst, size_t src, size_t n) { std::copy(h.begin() + src, h.begin() + src + n, h.begin() + dst); };
    dup(o_vs + VS_BIN * H, o_bin, H); dup(o_vs + VS_GIN * H, o_gin, H); dup(o_vs + VS_BEIN * H, o_bein, H);
    dup(o_vs + VS_GPI * H, o_gpi, H); dup(o_vs + VS_BEPI * H, o_bepi, H);
    dup(o_vs + VS_GV * H, o_gv, H); dup(o_vs + VS_BEV * H, o_bev, H);
    dup(o_vs + VS_BV1 * H, o_bv1, 128); dup(o_vs + VS_BV1 * H + 128, o_wv2, 128);
    dup(o_vs + vs_bpi(H), o_bpi, PI_LD);
    for (int b = 0; b < NB; b++) {
        const size_t d0 = o_vb + (size_t)b * 6 * H, v0 = (size_t)b * H;
        dup(d0, o_b1 + v0, H); dup(d0 + H, o_g1 + v0, H); dup(d0 + 2 * H, o_be1 + v0, H);
        dup(d0 + 3 * H, o_b2 + v0, H); dup(d0 + 4 * H, o_g2 + v0, H); dup(d0 + 5 * H, o_be2 + v0, H);
    }

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
    d.planes = 2;  // f32-equivalent (yk_net_set_precision switches to the fp16 mode)
    d.w_in = B + o_win; d.b_in = B + o_bin; d.g_in = B + o_gin; d.be_in = B + o_bein;
    d.w1 = B + o_w1; d.b1 = B + o_b1; d.g1 = B + o_g1; d.be1 = B + o_be1;
    d.w2 = B + o_w2; d.b2 = B + o_b2; d.g2 = B + o_g2; d.be2 = B + o_be2;
    d.g_pi = B + o_gpi; d.be_pi = B + o_bepi; d.w_pi = B + o_wpi; d.b_pi = B + o_bpi;
    d.g_v = B + o_gv; d.be_v = B + o_bev; d.w_v1 = B + o_wv1; d.b_v1 = B + o_bv1; d.w_v2 = B + o_wv2; d.b_v2 = B + o_bv2;
    d.vstat = B + o_vs; d.vblk = B + o_vb;
    d.err = reinterpret_cast<uint32_t*>(net->blob + o_err);
    // rounded up so the device-side bound stays an upper bound (and non-finite weights force the
    // full softmax)
    d.pi_bspread = std::isfinite(pi_bmax - pi_bmin) ? (pi_bmax - pi_bmin) * 1.001f + 1e-3f : INFINITY;
    d.pi_wmax = std::isfinite(pi_wmax) ? pi_wmax * 1.001f + 1e-3f : INFINITY;
    *out = net;
    return YK_OK;
}


int yk_net_set_precision(yk_net_t* net, int mode) {
    if (!net || (mode != YK_PREDICT_F32 && mode != YK_PREDICT_F16)) return YK_ERR_ARG;
    net->dev.planes = mode == YK_PREDICT_F16 ? 1 : 2;
    return YK_OK;
}

int yk_net_errors(yk_net_t* net, uint32_t* flags) {
    if (!net || !flags) return YK_ERR_ARG;
    YK_HIP(hipDeviceSynchronize());
    YK_HIP(hipMemcpy(flags, net->dev.err, sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (*flags) YK_HIP(hipMemset(net->dev.err, 0, sizeof(uint32_t)));
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
    YK_HIP(hipMallocAsync((void**)&logits, sizeof(float) * ((size_t)n * PI_LD + 2 * (size_t)n), s));
    float2* mlse = reinterpret_cast<float2*>(logits + (size_t)n * PI_LD);
    int rc = launch_forward(net->dev, states, x, nullptr, nullptr, n, logits, v, s, nullptr, mlse);
    if (rc == YK_OK) rc = launch_softmax(logits, mlse, pi, n, s);
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

int yk_net_leaf_prior(yk_net_t* net, const yk_state_t* states, float* pi, float* v, int n, void* stream) {
    if (!net || !states || !pi || !v || n < 0) return YK_ERR_ARG;
    if (n == 0) return YK_OK;
    hipStream_t s = as_stream(stream);
    float* logits = nullptr;
    YK_HIP(hipMallocAsync((void**)&logits, sizeof(float) * ((size_t)n * PI_LD + 2 * (size_t)n), s));
    float2* mlse = reinterpret_cast<float2*>(logits + (size_t)n * PI_LD);
    int rc = launch_forward(net->dev, states, nullptr, nullptr, nullptr, n, logits, v, s, nullptr, mlse, true);
    if (rc == YK_OK) {
        hipLaunchKernelGGL(k_leaf_prior, dim3((n + 3) / 4), dim3(256), 0, s, logits, mlse, states, pi, n);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) {
            yk::set_hip_error(e);
            rc = YK_ERR_HIP;
        }
    }
    (void)hipFreeAsync(logits, s);
    return rc;
}

int yk_net_policy_action(yk_net_t* net, const yk_state_t* states, int32_t* actions, float* probs, int n,
                         void* stream) {
    if (!net || !states || !actions || n < 0) return YK_ERR_ARG;
    if (n == 0) return YK_OK;
    hipStream_t s = as_stream(stream);
    float *logits = nullptr, *v = nullptr;
    YK_HIP(hipMallocAsync((void**)&logits, sizeof(float) * ((size_t)n * PI_LD + n), s));
    v = logits + (size_t)n * PI_LD;
    int rc = launch_forward(net->dev, states, nullptr, nullptr, nullptr, n, logits, v, s);
    if (rc == YK_OK) {
        hipLaunchKernelGGL(k_policy_pick, dim3((n + 3) / 4), dim3(256), 0, s, logits, states, actions, probs, n);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) {
            yk::set_hip_error(e);
            rc = YK_ERR_HIP;
        }
    }
    (void)hipFreeAsync(logits, s);
    return rc;
}

}  // extern "C"
