// yk_env.hip - batched Game plugin kernels (YachtGame, yacht/YachtGame.py:210-467) and
// their C-ABI entry points (include/yacht_hip.h).
//
// These are HBM-bound integer kernels: one lane per game for the transition-type
// functions (64 B in, 64 B out, coalesced as 4 x 16-B loads per lane), one wavefront per
// game where the output is action-shaped (valid mask via wave ballots, score table).
#include <atomic>

#include "yk_api.h"
#include "yk_common.h"

using namespace yk;

namespace yk {
static std::atomic<int> g_last_hip_error{0};
void set_hip_error(hipError_t e) { g_last_hip_error.store((int)e); }
}  // namespace yk

__device__ __forceinline__ YkS load_state(const yk_state_t* p, long i) {
    const uint4* q = reinterpret_cast<const uint4*>(p + i);
    YkS s;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        uint4 v = q[k];
        s.w[2 * k] = (uint64_t)v.x | ((uint64_t)v.y << 32);
        s.w[2 * k + 1] = (uint64_t)v.z | ((uint64_t)v.w << 32);
    }
    return s;
}
__device__ __forceinline__ void store_state(yk_state_t* p, long i, const YkS& s) {
    uint4* q = reinterpret_cast<uint4*>(p + i);
#pragma unroll
    for (int k = 0; k < 4; k++)
        q[k] = make_uint4((uint32_t)s.w[2 * k], (uint32_t)(s.w[2 * k] >> 32), (uint32_t)s.w[2 * k + 1],
                          (uint32_t)(s.w[2 * k + 1] >> 32));
}

__global__ void k_init_board(yk_state_t* out, uint64_t* ctr, const uint32_t* env, uint64_t seed, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Stream rs{seed, env[i], ctr[i]};
    YkS s;
#pragma unroll
    for (int k = 0; k < 8; k++) s.w[k] = 0;
    s.w[0] = 1ull | NO_BIDS;  // round 1, BID, no bids  (YachtState defaults, :133-147)
    new_round_rolls(s, rs);    // rollA, rollB  (getInitBoard :235-236)
    store_state(out, i, s);
    ctr[i] = rs.ctr;
}

__global__ void k_step(const yk_state_t* in, const int32_t* players, const int32_t* actions, uint64_t seed,
                       const uint32_t* env, uint64_t* ctr, yk_state_t* out, int32_t* next_players, int8_t* status,
                       int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    YkS s = load_state(in, i);
    Stream rs{seed, env[i], ctr[i]};
    int np = 0;
    const int st = step_state(s, players[i], actions[i], rs, np);
    status[i] = (int8_t)st;
    if (st == YK_ST_OK) {
        store_state(out, i, s);
        next_players[i] = np;
        ctr[i] = rs.ctr;
    }
}

// one wavefront per state; ballot builds 64 action bits per iteration
__global__ void k_valid_mask(const yk_state_t* in, const int32_t* players, uint32_t* mask, int32_t* counts, int n) {
    const int lane = threadIdx.x & 63;
    const int i = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (i >= n) return;
    const YkS s = load_state(in, i);
    const int pl = players[i];
    int total = 0;
    for (int base = 0; base < 64 * ((ASIZE + 63) / 64); base += 64) {
        const int a = base + lane;
        const bool v = a < ASIZE && action_valid(s, pl, a);
        const uint64_t b = __ballot(v);
        total += __popcll(b);
        const int word = base / 32;
        if (lane == 0 && word < MASK_WORDS) mask[(long)i * MASK_WORDS + word] = (uint32_t)b;
        if (lane == 1 && word + 1 < MASK_WORDS) mask[(long)i * MASK_WORDS + word + 1] = (uint32_t)(b >> 32);
    }
    if (counts && lane == 0) counts[i] = total;
}

__global__ void k_ended(const yk_state_t* in, const int32_t* players, double* r, int32_t* totals, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const YkS s = load_state(in, i);
    r[i] = game_ended(s, players[i]);
    if (totals) {
        totals[2 * i] = total_with_bonus(s, 0);
        totals[2 * i + 1] = total_with_bonus(s, 1);
    }
}

__global__ void k_canonical(const yk_state_t* in, const int32_t* players, yk_state_t* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    store_state(out, i, canonical(load_state(in, i), players[i]));
}

// one wavefront per state: lanes over the 252 combos, loop over the 12 categories
__global__ void k_score_table(const yk_state_t* in, const int32_t* players, int32_t* out, int n) {
    const int lane = threadIdx.x & 63;
    const int i = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (i >= n) return;
    const YkS s = load_state(in, i);
    const uint64_t wa = s_pw(s, players[i] == 1 ? 0 : 1, 0);
    const int nc = wa_n(wa);
    for (int ci = lane; ci < NCOMB; ci += 64) {
        const bool ok = c_tab.comb_max[ci] < nc;
        uint32_t chosen = 0;
        const uint32_t pos = c_tab.comb_pos[ci];
#pragma unroll
        for (int t = 0; t < 5; t++) chosen |= (uint32_t)((wa >> (4 * ((pos >> (4 * t)) & 0xF))) & 0xF) << (4 * t);
        for (int c = 0; c < NCAT; c++)
            out[((long)i * NCAT + c) * NCOMB + ci] = ok ? 1000 * score_k(c, chosen) : -1;
    }
}

__global__ void k_score_dice(const int8_t* dice, int32_t* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n * NCAT) return;
    const int r = i / NCAT, c = i % NCAT;
    uint32_t d = 0;
    for (int t = 0; t < 5; t++) d |= (uint32_t)(dice[5 * r + t] & 0xF) << (4 * t);
    out[i] = 1000 * score_k(c, d);
}

__global__ void k_featurize(const yk_state_t* in, float* x, int n) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long)n * FEAT) return;
    const int i = (int)(t / FEAT), f = (int)(t % FEAT);
    x[t] = feature(load_state(in, i), f);
}

__global__ void k_key_hash(const yk_state_t* in, uint64_t* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = key_hash(load_state(in, i));
}

__global__ void k_hash_prior(const yk_state_t* in, float* pi, float* v, int n) {
    const int i = blockIdx.y;
    const uint64_t h = key_hash(load_state(in, i));
    for (int a = blockIdx.x * blockDim.x + threadIdx.x; a < ASIZE; a += gridDim.x * blockDim.x)
        pi[(long)i * ASIZE + a] = hash_prior_pi(h, a);
    if (blockIdx.x == 0 && threadIdx.x == 0) v[i] = hash_prior_v(h);
}

// ------------------------------------------------------------------ C ABI
// GreedyYachtPlayer's heuristic, one wave per state
__global__ __launch_bounds__(256) void k_greedy(const yk_state_t* in, int32_t* out, int n) {
    const int lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    const YkS s = load_state(in, i);
    const int a = greedy_heuristic_wave(s, lane);
    if (lane == 0) out[i] = a;
}

extern "C" {

const char* yk_version(void) { return "yacht_hip 0.1 (gfx950)"; }
int yk_last_hip_error(void) { return yk::g_last_hip_error.load(); }
uint64_t yk_rng_draw64(uint64_t seed, uint32_t env, uint64_t ctr) { return philox_draw(seed, env, ctr); }

#define YK_CHECK_N(n) \
    if ((n) < 0) return YK_ERR_ARG; \
    if ((n) == 0) return YK_OK

int yk_init_board(yk_state_t* out, uint64_t* rng_ctr, const uint32_t* env_ids, uint64_t seed, int n, void* stream) {
    YK_CHECK_N(n);
    if (!out || !rng_ctr || !env_ids) return YK_ERR_ARG;
    hipLaunchKernelGGL(k_init_board, dim3(grid_for(n, 256)), dim3(256), 0, as_stream(stream), out, rng_ctr, env_ids,
                       seed, n);
    YK_LAUNCHED();
    return YK_OK;
}

int yk_step(const yk_state_t* in, const int32_t* players, const int32_t* actions, uint64_t seed,
            const uint32_t* env_ids, uint64_t* rng_ctr, yk_state_t* out, int32_t* next_players, int8_t* status, int n,
            void* stream) {
    YK_CHECK_N(n);
    if (!in || !players || !actions || !env_ids || !rng_ctr || !out || !next_players || !status) return YK_ERR_ARG;
    hipLaunchKernelGGL(k_step, dim3(grid_for(n, 256)), dim3(256), 0, as_stream(stream), in, players, actions, seed,
                       env_ids, rng_ctr, out, next_players, status, n);
    YK_LAUNCHED();
    return YK_OK;
}

int yk_valid_mask(const yk_state_t* in, const int32_t* players, uint32_t* mask, int32_t* counts, int n,
                  void* stream) {
    YK_CHECK_N(n);
    if (!in || !players || !mask) return YK_ERR_ARG;
    hipLaunchKernelGGL(k_valid_mask, dim3(grid_for(n, 4)), dim3(256), 0, as_stream(stream), in, players, mask, counts,
                       n);
    YK_LAUNCHED();
    return YK_OK;
}

int yk_ended(const yk_state_t* in, const int32_t* players, double* result, int32_t* totals, int n, void* stream) {
    YK_CHECK_N(n);
    if (!in || !players || !result) return YK_ERR_ARG;
    hipLaunchKernelGGL(k_ended, dim3(grid_for(n, 256)), dim3(256), 0, as_stream(stream), in, players, result, totals,
                       n);
    YK_LAUNCHED();
    return YK_OK;
}

int yk_canonical(const yk_state_t* in, const int32_t* players, yk_state_t* out, int n, void* stream) {
    YK_CHECK_N(n);
    if (!in || !players || !out) return YK_ERR_ARG;
    hipLaunchKernelGGL(k_canonical, dim3(grid_for(n, 256)), dim3(256), 0, as_stream(stream), in, players, out, n);
    YK_LAUNCHED();
    return YK_OK;
}

int yk_score_table(const yk_state_t* in, const int32_t* players, int32_t* out, int n, void* stream) {
    YK_CHECK_N(n);
    if (!in || !players || !out) return YK_ERR_ARG;
    hipLaunchKernelGGL(k_score_table, dim3(grid_for(n, 4)), dim3(256), 0, as_stream(stream), in, players, out, n);
    YK_LAUNCHED();
    return YK_OK;
}

int yk_score_dice(const int8_t* dice, int32_t* out, int n, void* stream) {
    YK_CHECK_N(n);
    if (!dice || !out) return YK_ERR_ARG;
    hipLaunchKernelGGL(k_score_dice, dim3(grid_for((long)n * NCAT, 256)), dim3(256), 0, as_stream(stream), dice, out,
                       n);
    YK_LAUNCHED();
    return YK_OK;
}

int yk_featurize(const yk_state_t* in, float* x, int n, void* stream) {
    YK_CHECK_N(n);
    if (!in || !x) return YK_ERR_ARG;
    hipLaunchKernelGGL(k_featurize, dim3(grid_for((long)n * FEAT, 256)), dim3(256), 0, as_stream(stream), in, x, n);
    YK_LAUNCHED();
    return YK_OK;
}

int yk_key_hash(const yk_state_t* in, uint64_t* out, int n, void* stream) {
    YK_CHECK_N(n);
    if (!in || !out) return YK_ERR_ARG;
    hipLaunchKernelGGL(k_key_hash, dim3(grid_for(n, 256)), dim3(256), 0, as_stream(stream), in, out, n);
    YK_LAUNCHED();
    return YK_OK;
}

int yk_hash_prior(const yk_state_t* in, float* pi, float* v, int n, void* stream) {
    YK_CHECK_N(n);
    if (!in || !pi || !v) return YK_ERR_ARG;
    if (n > 65535) return YK_ERR_ARG;
    hipLaunchKernelGGL(k_hash_prior, dim3(4, n), dim3(256), 0, as_stream(stream), in, pi, v, n);
    YK_LAUNCHED();
    return YK_OK;
}

int yk_greedy_action(const yk_state_t* states, int32_t* actions, int n, void* stream) {
    YK_CHECK_N(n);
    if (!states || !actions) return YK_ERR_ARG;
    hipLaunchKernelGGL(k_greedy, dim3((n + 3) / 4), dim3(256), 0, as_stream(stream), states, actions, n);
    YK_LAUNCHED();
    return YK_OK;
}

}  // extern "C"
