// yk_net.h - batched YachtNNet forward (yacht/pytorch/YachtNNet.py:8-70) on gfx950.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "yacht_hip.h"

namespace yk {

constexpr int PI_LD = 3264;         // logits row stride: 3226 padded to 204 tiles of 16 columns
constexpr int PI_TILES = PI_LD / 16;

// Dense weights are stored as two fp16 planes (hi = fp16(w), lo = fp16((w - hi) * 2^11)) in
// v_mfma_f32_16x16x32_f16 fragment order ("packed"): for a [N][K] matrix,
//   P[nt][ks][plane][lane][j] = plane(W[16 nt + (lane & 15)][32 ks + 8 (lane >> 4) + j]),  j < 8
// so one wave loads one plane of a 16-column x 32-deep slice as one contiguous 1 KB access;
// a packed matrix takes the bytes of the f32 one.
struct NetDev {
    int H, NB;
    const float *w_in, *b_in, *g_in, *be_in;  // w_in packed [H/16][2][2][64][8 fp16] (K 59 padded to 64)
    const float *w1, *b1, *g1, *be1;          // per block: packed [H/16][H/32][2][64][8 fp16], vectors [H]
    const float *w2, *b2, *g2, *be2;
    const float *g_pi, *be_pi, *w_pi, *b_pi;  // w_pi packed [204][H/32][2][64][8] (rows >= 3226 zero), b_pi [3264]
    const float *g_v, *be_v, *w_v1, *b_v1, *w_v2, *b_v2;  // w_v1 packed [8][H/32][2][64][8], w_v2 [128], b_v2 [1]
    const float* vstat;  // copies staged to LDS once: [VS_* x H] + b_v1[128] w_v2[128] + b_pi[3264]
    const float* vblk;   // per block b: b1 g1 be1 b2 g2 be2 ([6][H]), staged to LDS per block
    float pi_bspread;    // max - min of pi_head.2's bias over the 3226 actions
    float pi_wmax;       // max over actions of |pi_head.2 weight row|_2
    int planes;          // 2: f32-equivalent hi/lo products (default); 1: fp16 mode (hi planes only)
    uint32_t* err;       // device check flags (FWD_ERR_SYNC), a word of the net's blob; read by yk_net_errors
};
constexpr uint32_t FWD_ERR_SYNC = 1u;  // = YK_NET_ERR_SYNC: the value head's wait for v_head.2 timed out
// vstat offsets in units of H (b_v1 at VS_BV1*H, w_v2 right after it, b_pi at vs_bpi(H))
enum { VS_BIN = 0, VS_GIN = 1, VS_BEIN = 2, VS_GPI = 3, VS_BEPI = 4, VS_GV = 5, VS_BEV = 6, VS_BV1 = 7 };
constexpr int vs_bpi(int H) { return 7 * H + 256; }
constexpr int vstat_size(int H) { return vs_bpi(H) + PI_LD; }

// Full forward: features (from packed states, or explicit rows x[n][59]) ->
// logits[n][PI_LD] (pi_head before softmax) and v[n] = tanh(v_head).  `rows` (optional) maps
// output row i to input index rows[i]; `count` (optional, device) overrides n; `active`
// (optional, device, [n]) lets a workgroup whose 16 rows are all inactive exit at once.
// `mlse` (optional, device, [n]) gets each row's (max, log sum exp(x - max)) over the 3226
// logits, so that exp(log_softmax(x))[a] = exp(x[a] - m - l) needs only the logits it is asked for.
int launch_forward(const NetDev& net, const yk_state_t* states, const float* x, const int32_t* rows,
                   const int32_t* count, int n, float* logits, float* v, hipStream_t stream,
                   const uint8_t* active = nullptr, float2* mlse = nullptr, bool valid_only = false,
                   uint8_t want = 0xFF,  // a row is predicted iff !active || (active[row] & want)
                   int parts = 1, int mstride = 0);
// parts > 1 (1, 2 or 4): `parts` workgroups per 16-row tile split the policy head's tile list
// (each runs the trunk), for launches with fewer tiles than CUs; mlse[p * mstride + row] then holds
// part p's raw (max, sum exp) of the row, which the consumer merges (max, then log of the sum).
// pi[n][3226] = exp(log_softmax(logits[:, :3226])) = exp(logits - m - l), (m, l) = mlse[row]
int launch_softmax(const float* logits, const float2* mlse, float* pi, int n, hipStream_t stream);

}  // namespace yk

struct yk_net {
    yk::NetDev dev;
    float* blob;  // single device allocation holding every tensor
    size_t bytes;
};
