// yk_net.h - batched YachtNNet forward (yacht/pytorch/YachtNNet.py:8-70) on gfx950.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "yacht_hip.h"

namespace yk {

constexpr int PI_LD = 3264;  // logits row stride: 3226 padded to 51 tiles of 64 columns

struct NetDev {
    int H, NB;
    const float *w_in, *b_in, *g_in, *be_in;  // w_in [H][64] (59 used)
    const float *w1, *b1, *g1, *be1;          // [NB][H][H], [NB][H] ...
    const float *w2, *b2, *g2, *be2;
    const float *g_pi, *be_pi, *w_pi, *b_pi;  // w_pi [PI_LD][H] (rows >= 3226 zero)
    const float *g_v, *be_v, *w_v1, *b_v1, *w_v2, *b_v2;  // w_v1 [128][H], w_v2 [128], b_v2 [1]
};

// Trunk: features (from packed states, or explicit rows x[n][59]) -> a_pi[n][H] =
// SiLU(LN_pi(h)) and v[n] = tanh(v_head(h)).  `rows` (optional) maps output row i to
// input state index rows[i]; `count` (optional, device) overrides n.
int launch_trunk(const NetDev& net, const yk_state_t* states, const float* x, const int32_t* rows,
                 const int32_t* count, int n, float* a_pi, float* v, hipStream_t stream);
// logits[n][PI_LD] = a_pi @ w_pi^T + b_pi  (f32 MFMA)
int launch_pihead(const NetDev& net, const float* a_pi, const int32_t* count, int n, float* logits,
                  hipStream_t stream);
// pi[n][3226] = exp(log_softmax(logits[:, :3226]))
int launch_softmax(const float* logits, float* pi, int n, hipStream_t stream);

}  // namespace yk

struct yk_net {
    yk::NetDev dev;
    float* blob;  // single device allocation holding every tensor
    size_t bytes;
};
