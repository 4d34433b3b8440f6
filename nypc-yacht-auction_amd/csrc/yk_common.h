// yk_common.h - device-side Yacht Auction rules on the 64-byte packed state.
//
// Everything here is a __device__ restatement of yacht/YachtGame.py (reference paths) on
// the packed layout of include/yacht_hip.h / DESIGN.md s3:
//   w0 : round[0:4] phase[4] hasA[5] hasB[6] bid1[8:16] bid2[16:24] rollA[24:44] rollB[44:64]
//   w1..w3 (p1), w4..w6 (p2):
//     wa : carry nibbles[0:40] ncarry[40:44] used[44:56]
//     wb : cat[0..7] bytes (points / 1000)
//     wc : cat[8..11] bytes [0:32], bid_score int32 [32:64]
//   w7 : 0
// Dice are nibbles 1..6; a bid byte is 0xFF (None) or target<<7 | amount/500.
// Only constant indices into w[] are used so states live in registers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <climits>

#include "yacht_hip.h"

namespace yk {

constexpr int NCAT = 12, NBID = 202, NCOMB = 252, ASIZE = 3226, FEAT = 59, BID_LEVELS = 101;
constexpr int MASK_WORDS = 101;

struct YkS {
    uint64_t w[8];
};

// ------------------------------------------------------------------ constant tables
struct Tables {
    uint16_t comb_mask[NCOMB];  // COMB_5_OF_10[i] as a position bitmask (YachtGame.py:35)
    uint32_t comb_pos[NCOMB];   // the 5 positions as nibbles
    uint8_t comb_max[NCOMB];    // max(comb)
    uint16_t vcnt[16];          // number of combos with max < n  (= C(n,5))
    uint16_t voff[16];          // offset into vids
    uint8_t vids[512];          // those combo ids, ascending, for n = 5..10
    uint8_t vrank[6][NCOMB];    // rank of combo i among those with max < n (n = 5..10; valid ones only)
    float die_scale[16];        // _scale_die(d) = (d - 3.5) / 3.5  (NNet.py:50-51), f32
    float round_feat[16];       // round / 13.0 as f32 (NNet.py:69)
};
constexpr Tables make_tables() {
    Tables t{};
    int k = 0;
    for (int a = 0; a < 10; a++)
        for (int b = a + 1; b < 10; b++)
            for (int c = b + 1; c < 10; c++)
                for (int d = c + 1; d < 10; d++)
                    for (int e = d + 1; e < 10; e++) {
                        t.comb_mask[k] = (uint16_t)((1 << a) | (1 << b) | (1 << c) | (1 << d) | (1 << e));
                        t.comb_pos[k] = (uint32_t)(a | (b << 4) | (c << 8) | (d << 12) | (e << 16));
                        t.comb_max[k] = (uint8_t)e;
                        k++;
                    }
    int off = 0;
    for (int n = 0; n < 16; n++) {
        t.voff[n] = (uint16_t)off;
        int cnt = 0;
        if (n >= 5 && n <= 10)
            for (int i = 0; i < NCOMB; i++)
                if (t.comb_max[i] < n) t.vids[off + cnt++] = (uint8_t)i;
        t.vcnt[n] = (uint16_t)cnt;
        if (n >= 5 && n <= 10)
            for (int r = 0; r < cnt; r++) t.vrank[n - 5][t.vids[off + r]] = (uint8_t)r;
        off += cnt;
    }
    for (int d = 0; d < 16; d++) t.die_scale[d] = (float)(((double)d - 3.5) / 3.5);
    for (int r = 0; r < 16; r++) t.round_feat[r] = (float)((double)r / 13.0);
    return t;
}
static __constant__ Tables c_tab = make_tables();
static constexpr Tables h_tab = make_tables();

// ------------------------------------------------------------------ field access
__device__ __host__ inline int s_round(const YkS& s) { return (int)(s.w[0] & 0xF); }
__device__ __host__ inline int s_phase(const YkS& s) { return (int)((s.w[0] >> 4) & 1); }
__device__ __host__ inline int s_bid(const YkS& s, int b) { return (int)((s.w[0] >> (8 + 8 * b)) & 0xFF); }
__device__ __host__ inline uint64_t s_pw(const YkS& s, int p, int k) {  // player word k of player p
    return p ? (k == 0 ? s.w[4] : k == 1 ? s.w[5] : s.w[6]) : (k == 0 ? s.w[1] : k == 1 ? s.w[2] : s.w[3]);
}
__device__ __host__ inline void s_set_pw(YkS& s, int p, int k, uint64_t v) {
    if (p) {
        if (k == 0) s.w[4] = v; else if (k == 1) s.w[5] = v; else s.w[6] = v;
    } else {
        if (k == 0) s.w[1] = v; else if (k == 1) s.w[2] = v; else s.w[3] = v;
    }
}
__device__ __host__ inline int wa_n(uint64_t wa) { return (int)((wa >> 40) & 0xF); }
__device__ __host__ inline int wa_used(uint64_t wa) { return (int)((wa >> 44) & 0xFFF); }
__device__ __host__ inline int32_t wc_bid(uint64_t wc) { return (int32_t)(uint32_t)(wc >> 32); }

// sum of category bytes (points/1000) and of the six basic ones
__device__ __host__ inline int cat_sum(uint64_t wb, uint64_t wc, int* basic) {
    int b = 0, all = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        int v = (int)((wb >> (8 * i)) & 0xFF);
        all += v;
        if (i < 6) b += v;
    }
#pragma unroll
    for (int i = 0; i < 4; i++) all += (int)((wc >> (8 * i)) & 0xFF);
    *basic = b;
    return all;
}
// PlayerState.total_with_bonus  YachtGame.py:125-130
__device__ __host__ inline int total_with_bonus(const YkS& s, int p) {
    int basic;
    int all = cat_sum(s_pw(s, p, 1), s_pw(s, p, 2), &basic);
    return 1000 * all + (1000 * basic >= 63000 ? 35000 : 0) + wc_bid(s_pw(s, p, 2));
}
__device__ __host__ inline bool all_used(const YkS& s, int p) {  // both_scored_all  YachtGame.py:189-190
    return wa_used(s_pw(s, p, 0)) == 0xFFF;
}

// ------------------------------------------------------------------ RNG contract (oracle/spec.py)
__device__ __host__ inline uint64_t philox_draw(uint64_t seed, uint32_t env, uint64_t ctr) {
    uint32_t c0 = (uint32_t)ctr, c1 = (uint32_t)(ctr >> 32), c2 = env, c3 = 0;
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int r = 0; r < 10; r++) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c0 = n0;
        c1 = (uint32_t)p1;
        c2 = n2;
        c3 = (uint32_t)p0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return (uint64_t)c0 | ((uint64_t)c1 << 32);
}
// Dropout keep masks of the trainers (yk_train.hip, yk_train_amp.hip): element e (= global row x H
// + column) of layer `layer` at optimiser step `step` is kept iff its 16-bit uniform - bits
// 16 (e % 4) .. of the Philox draw of its group of four - is >= p (one draw per 4 elements).
// The cache is keyed by (layer, group): one cache may serve every layer of a kernel, and a row
// whose last group of layer l is its first of layer l + 1 (a wave holding a single row at H <= 256)
// must not reuse layer l's mask.
struct KeepCache {
    long g = -1;
    int layer = -1;
    uint32_t m = 0;
};
// the keep bits of elements 4 g .. 4 g + 3 of a dropout layer: one Philox draw, four 16-bit uniforms
__device__ inline uint32_t dropout_bits(uint64_t seed, int layer, uint64_t step, long g, float p) {
    const uint64_t d = philox_draw(seed, 0x44524F50u + (uint32_t)layer, (step << 32) ^ (uint64_t)g);
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < 4; k++)  // (a 32-bit value into the conversion: a 64-bit one is a long sequence)
        m |= ((float)(uint32_t)((d >> (16 * k)) & 0xFFFFu) * (1.0f / 65536.0f) >= p ? 1u : 0u) << k;
    return m;
}
__device__ inline bool dropout_keep(KeepCache& kc, uint64_t seed, int layer, uint64_t step, long e, float p) {
    if (p <= 0.0f) return true;
    const long g = e >> 2;
    if (g != kc.g || layer != kc.layer) {
        kc.g = g;
        kc.layer = layer;
        kc.m = dropout_bits(seed, layer, step, g, p);
    }
    return (kc.m >> (e & 3)) & 1u;
}
struct Stream {
    uint64_t seed;
    uint32_t env;
    uint64_t ctr;
    __device__ __host__ uint64_t next() { return philox_draw(seed, env, ctr++); }
    __device__ __host__ int below(int n) { return (int)(((next() >> 32) * (uint64_t)n) >> 32); }
    __device__ __host__ int die() { return 1 + below(6); }
    __device__ __host__ double uniform53() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
    // roll_five  YachtGame.py:154-155 -> 5 nibbles
    __device__ __host__ uint64_t roll5() {
        uint64_t r = 0;
        for (int i = 0; i < 5; i++) r |= (uint64_t)die() << (4 * i);
        return r;
    }
};

// ------------------------------------------------------------------ hashing
__device__ __host__ inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __host__ inline uint64_t key_hash(const YkS& s) {
    uint64_t h = 0x243F6A8885A308D3ull;
#pragma unroll
    for (int i = 0; i < 8; i++) h = mix64(h ^ (s.w[i] + 0x9E3779B97F4A7C15ull * (uint64_t)(i + 1)));
    return h;
}
__device__ __host__ inline float hash_prior_pi(uint64_t h, int a) {
    uint64_t z = mix64(h ^ (0xD1B54A32D192ED03ull * (uint64_t)(a + 1)));
    return ((float)((z >> 40) & 0xFFFF) + 1.0f) * (1.0f / 65536.0f);
}
__device__ __host__ inline float hash_prior_v(uint64_t h) {
    uint64_t zv = mix64(h ^ 0x8CB92BA72F3D8DD7ull);
    return (float)((double)((int64_t)((zv >> 40) & 0xFFFF) - 32768) / 32768.0);
}

// ------------------------------------------------------------------ scoring
// score_category  YachtGame.py:57-108 on 5 dice given as nibbles; returns points / 1000
__device__ __host__ inline int score_k(int cat, uint32_t dice) {
    uint32_t cnt = 0;
    int sum = 0;
#pragma unroll
    for (int i = 0; i < 5; i++) {
        int d = (int)((dice >> (4 * i)) & 0xF);
        cnt += 1u << (4 * (d - 1));
        sum += d;
    }
    auto c = [&](int v) { return (int)((cnt >> (4 * (v - 1))) & 0xF); };
    if (cat <= 5) return (cat + 1) * c(cat + 1);
    if (cat == 6) return sum;
    if (cat == 7) {
        bool ok = false;
        for (int v = 1; v <= 6; v++) ok |= c(v) >= 4;
        return ok ? sum : 0;
    }
    if (cat == 8) {
        bool pair = false, triple = false;
        for (int v = 1; v <= 6; v++) {
            pair |= (c(v) == 2 || c(v) == 5);
            triple |= (c(v) == 3 || c(v) == 5);
        }
        return (pair && triple) ? sum : 0;
    }
    uint32_t e = 0;  // presence bits of faces 1..6
    for (int v = 1; v <= 6; v++) e |= (c(v) > 0 ? 1u : 0u) << v;
    if (cat == 9) return ((e & 0x1E) == 0x1E || (e & 0x3C) == 0x3C || (e & 0x78) == 0x78) ? 15 : 0;
    if (cat == 10) return ((e & 0x3E) == 0x3E || (e & 0x7C) == 0x7C) ? 30 : 0;
    if (cat == 11) {
        bool ok = false;
        for (int v = 1; v <= 6; v++) ok |= c(v) == 5;
        return ok ? 50 : 0;
    }
    return -1;
}

// ------------------------------------------------------------------ transitions
constexpr uint64_t NO_BIDS = (0xFFull << 8) | (0xFFull << 16);

// _resolve_bids_and_assign  YachtGame.py:502-542
__device__ __host__ inline int resolve_bids(YkS& s, Stream& rs) {
    int b1 = s_bid(s, 0), b2 = s_bid(s, 1);
    if (b1 == 0xFF || b2 == 0xFF) return YK_ST_ASSERT;
    int t1 = b1 >> 7, a1 = 500 * (b1 & 0x7F), t2 = b2 >> 7, a2 = 500 * (b2 & 0x7F);
    int g0 = t1, g1 = t2;
    if (g0 == g1) {
        int winner;
        if (a1 > a2) winner = 0;
        else if (a2 > a1) winner = 1;
        else winner = rs.below(2);  // tiebreak_uniform  YachtGame.py:158-159
        if (winner == 0) g1 = 1 - g0;
        else g0 = 1 - g1;
    }
    const uint64_t w0 = s.w[0];
    const int hasA = (int)((w0 >> 5) & 1), hasB = (int)((w0 >> 6) & 1);
    const uint64_t rA = (w0 >> 24) & 0xFFFFF, rB = (w0 >> 44) & 0xFFFFF;
    for (int p = 0; p < 2; p++) {
        const int g = p ? g1 : g0, t = p ? t2 : t1, a = p ? a2 : a1;
        uint64_t wa = s_pw(s, p, 0), wc = s_pw(s, p, 2);
        int32_t bid = wc_bid(wc) + ((g == t) ? -a : a);
        wc = (wc & 0xFFFFFFFFull) | ((uint64_t)(uint32_t)bid << 32);
        const int has = g == 0 ? hasA : hasB;
        if (has) {
            int n = wa_n(wa);
            if (n + 5 > 10) return YK_ST_CAPACITY;
            uint64_t carry = (wa & ((1ull << 40) - 1)) | ((g == 0 ? rA : rB) << (4 * n));
            wa = carry | ((uint64_t)(n + 5) << 40) | (wa & (0xFFFull << 44));
        }
        s_set_pw(s, p, 0, wa);
        s_set_pw(s, p, 2, wc);
    }
    return YK_ST_OK;
}

// WAVE: called by all 64 lanes of a wave together (wave-per-game kernels): lanes 0-9 draw
// the ten dice (counters ctr .. ctr + 9) at once and three ballots assemble them - the same
// values, in the same stream order, as the sequential path.
template <bool WAVE = false>
__device__ __host__ inline void new_round_rolls(YkS& s, Stream& rs) {
    uint64_t ra = 0, rb = 0;
#ifdef __HIP_DEVICE_COMPILE__
    if constexpr (WAVE) {
        const int lane = threadIdx.x & 63;
        int die = 0;
        if (lane < 10) die = 1 + (int)(((philox_draw(rs.seed, rs.env, rs.ctr + (uint64_t)lane) >> 32) * 6ull) >> 32);
        const uint64_t b0 = __ballot(die & 1), b1 = __ballot(die & 2), b2 = __ballot(die & 4);
#pragma unroll
        for (int i = 0; i < 10; i++) {
            const uint64_t dv = ((b0 >> i) & 1) | (((b1 >> i) & 1) << 1) | (((b2 >> i) & 1) << 2);
            if (i < 5) ra |= dv << (4 * i);
            else rb |= dv << (4 * (i - 5));
        }
        rs.ctr += 10;
    } else
#endif
    {
        ra = rs.roll5();
        rb = rs.roll5();
    }
    s.w[0] = (s.w[0] & ((1ull << 24) - 1)) | (1ull << 5) | (1ull << 6) | (ra << 24) | (rb << 44);
}

// getNextState  YachtGame.py:260-372, in place on a register copy (the reference copies,
// :264).  Returns YK_ST_*.
template <bool WAVE = false>
__device__ __host__ inline int step_state(YkS& s, int player, int action, Stream& rs, int& next_player) {
    const int round = s_round(s), phase = s_phase(s);
    if (phase == 0 && round != 13) {
        if (!(action >= 0 && action < NBID)) return YK_ST_VALUE_BID;
        const uint64_t code = ((uint64_t)(action / BID_LEVELS) << 7) | (uint64_t)(action % BID_LEVELS);
        const int sh = (player == 1) ? 8 : 16;
        const bool first = s_bid(s, 0) == 0xFF && s_bid(s, 1) == 0xFF;
        s.w[0] = (s.w[0] & ~(0xFFull << sh)) | (code << sh);
        if (first) {
            next_player = -player;
            return YK_ST_OK;
        }
        int r = resolve_bids(s, rs);
        if (r) return r;
        if (round != 1) {
            s.w[0] |= 1ull << 4;  // PHASE_SCORE, bids and stale rolls kept (:290-293)
        } else {
            s.w[0] = (s.w[0] & ~0xFull & ~(1ull << 4)) | 2ull | NO_BIDS;  // round 2, BID
            new_round_rolls<WAVE>(s, rs);
        }
        next_player = 1;
        return YK_ST_OK;
    }
    if (phase == 1) {
        if (!(action >= NBID && action < ASIZE)) return YK_ST_VALUE_SCORE;
        const int base = action - NBID, cat = base / NCOMB, ci = base % NCOMB;
        const int p = (player == 1) ? 0 : 1;
        uint64_t wa = s_pw(s, p, 0);
        const int n = wa_n(wa);
        if ((wa_used(wa) >> cat) & 1) {  // category reuse -> unchanged copy (:312-314)
            next_player = -player;
            return YK_ST_OK;
        }
#ifdef __HIP_DEVICE_COMPILE__
        const Tables& T = c_tab;
#else
        const Tables& T = h_tab;
#endif
        if (T.comb_max[ci] >= n) {  // combo past the carry -> unchanged copy (:322-324)
            next_player = -player;
            return YK_ST_OK;
        }
        const uint32_t pos = T.comb_pos[ci];
        const uint32_t mask = T.comb_mask[ci];
        uint32_t chosen = 0;
#pragma unroll
        for (int t = 0; t < 5; t++) chosen |= (uint32_t)((wa >> (4 * ((pos >> (4 * t)) & 0xF))) & 0xF) << (4 * t);
        const int sc = score_k(cat, chosen);
        uint64_t nc = 0;
        int k = 0;
#pragma unroll
        for (int i = 0; i < 10; i++) {
            if (i < n && !((mask >> i) & 1)) {
                nc |= ((wa >> (4 * i)) & 0xF) << (4 * k);
                k++;
            }
        }
        const int used = wa_used(wa) | (1 << cat);
        wa = nc | ((uint64_t)k << 40) | ((uint64_t)used << 44);
        s_set_pw(s, p, 0, wa);
        if (cat < 8) {
            uint64_t wb = s_pw(s, p, 1);
            wb = (wb & ~(0xFFull << (8 * cat))) | ((uint64_t)sc << (8 * cat));
            s_set_pw(s, p, 1, wb);
        } else {
            uint64_t wc = s_pw(s, p, 2);
            wc = (wc & ~(0xFFull << (8 * (cat - 8)))) | ((uint64_t)sc << (8 * (cat - 8)));
            s_set_pw(s, p, 2, wc);
        }
        if (round == 13) {
            next_player = (all_used(s, 0) && all_used(s, 1)) ? 1 : -player;
            return YK_ST_OK;
        }
        if (player == -1) {
            const int nr = round + 1;
            s.w[0] = (s.w[0] & ~0xFull) | (uint64_t)nr | NO_BIDS;
            if (nr != 13) {
                new_round_rolls<WAVE>(s, rs);
                s.w[0] &= ~(1ull << 4);
            } else {
                s.w[0] |= 1ull << 4;
            }
            next_player = 1;
            return YK_ST_OK;
        }
        next_player = -player;
        return YK_ST_OK;
    }
    return YK_ST_RUNTIME;
}

// getCanonicalForm  YachtGame.py:430-442
__device__ __host__ inline YkS canonical(const YkS& s, int player) {
    if (player == 1) return s;
    YkS o;
    o.w[0] = (s.w[0] & ~((0xFFull << 8) | (0xFFull << 16))) | (((s.w[0] >> 8) & 0xFF) << 16) |
             (((s.w[0] >> 16) & 0xFF) << 8);
    o.w[1] = s.w[4]; o.w[2] = s.w[5]; o.w[3] = s.w[6];
    o.w[4] = s.w[1]; o.w[5] = s.w[2]; o.w[6] = s.w[3];
    o.w[7] = s.w[7];
    return o;
}

// getGameEnded  YachtGame.py:408-428
__device__ __host__ inline double game_ended(const YkS& s, int player) {
    if (!(all_used(s, 0) && all_used(s, 1))) return 0.0;
    const int t1 = total_with_bonus(s, 0), t2 = total_with_bonus(s, 1);
    if (t1 == t2) return 1e-4;
    const int winner = t1 > t2 ? 1 : -1;
    return (double)(player == 1 ? winner : -winner);
}

// ------------------------------------------------------------------ valid actions
// getValidMoves  YachtGame.py:374-406, in compact form: the valid set is either the 202
// bids, or {unused categories (ascending)} x {combos with max < n (ascending)}.
struct VInfo {
    int V;          // number of valid actions
    int W;          // combos per category (score) ; 0 for bids
    int n;          // carry length
    uint64_t cats;  // unused categories as nibbles, ascending
    int k;          // number of unused categories
};
__device__ __host__ inline VInfo valid_info(const YkS& s, int player) {
    VInfo v{0, 0, 0, 0, 0};
    const int round = s_round(s), phase = s_phase(s);
    if (phase == 0 && round != 13) {
        v.V = NBID;
        return v;
    }
    if (phase == 1) {
        const uint64_t wa = s_pw(s, player == 1 ? 0 : 1, 0);
        const int n = wa_n(wa);
        if (n < 5) return v;
#ifdef __HIP_DEVICE_COMPILE__
        const Tables& T = c_tab;
#else
        const Tables& T = h_tab;
#endif
        const int used = wa_used(wa);
        int k = 0;
        uint64_t cats = 0;
        for (int c = 0; c < NCAT; c++)
            if (!((used >> c) & 1)) {
                cats |= (uint64_t)c << (4 * k);
                k++;
            }
        v.n = n;
        v.W = T.vcnt[n > 15 ? 15 : n];
        v.k = k;
        v.cats = cats;
        v.V = k * v.W;
    }
    return v;
}
__device__ __host__ inline int compact_to_action(const VInfo& v, int j) {
    if (v.W == 0) return j;
    // the two carry sizes of real play need no table and no runtime division: 10 dice -> all
    // 252 combos valid (ids = ranks); 5 dice -> only combo 0
    if (v.n >= 10) {
        const int ci = j / NCOMB, r = j - ci * NCOMB;
        return NBID + NCOMB * (int)((v.cats >> (4 * ci)) & 0xF) + r;
    }
    if (v.n == 5) return NBID + NCOMB * (int)((v.cats >> (4 * j)) & 0xF);
#ifdef __HIP_DEVICE_COMPILE__
    const Tables& T = c_tab;
#else
    const Tables& T = h_tab;
#endif
    const int ci = j / v.W, r = j - ci * v.W;
    const int cat = (int)((v.cats >> (4 * ci)) & 0xF);
    return NBID + NCOMB * cat + (int)T.vids[T.voff[v.n] + r];
}
// dense validity of one action (for bitmask kernels)
__device__ __host__ inline bool action_valid(const YkS& s, int player, int a) {
    const int round = s_round(s), phase = s_phase(s);
    if (phase == 0 && round != 13) return a < NBID;
    if (phase != 1 || a < NBID) return false;
    const uint64_t wa = s_pw(s, player == 1 ? 0 : 1, 0);
    const int n = wa_n(wa);
    if (n < 5) return false;
    const int base = a - NBID, cat = base / NCOMB, ci = base - cat * NCOMB;
#ifdef __HIP_DEVICE_COMPILE__
    const Tables& T = c_tab;
#else
    const Tables& T = h_tab;
#endif
    return !((wa_used(wa) >> cat) & 1) && T.comb_max[ci] < n;
}

// ------------------------------------------------------------------ cross-lane exchange
// xlane<O>(x): the value lane l ^ O holds, without __shfl_xor's LDS round trip (ds_bpermute,
// ~100+ cycles, on the LDS pipe every wave of the CU shares): DPP quad permutes for O = 1, 2,
// the quad reversal then the half-row mirror for O = 4, a row rotation by 8 for O = 8, and
// gfx950's permlane swaps for O = 16, 32.  Exact for any contents of the wave, so a butterfly
// on it gives __shfl_xor's results bit for bit (tools/xlane_check.hip checks every O).
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, 0xF, 0xF, false);
}
template <int O>
__device__ __forceinline__ uint32_t xlane_u(uint32_t v) {
    static_assert(O == 1 || O == 2 || O == 4 || O == 8 || O == 16 || O == 32, "xor offsets 1 .. 32");
    if constexpr (O == 1) return dpp_mov<0xB1>(v);                   // quad_perm [1,0,3,2]
    else if constexpr (O == 2) return dpp_mov<0x4E>(v);              // quad_perm [2,3,0,1]
    else if constexpr (O == 4) return dpp_mov<0x141>(dpp_mov<0x1B>(v));  // quad_perm [3,2,1,0], row_half_mirror
    else if constexpr (O == 8) return dpp_mov<0x128>(v);             // row_ror:8
    else {
        // v_permlane{16,32}_swap(v, v): the first result holds the lower row / half in both
        // positions, the second the upper
        // (threadIdx.x & O is the lane's bit O for the 1-D workgroups of multiples of 64 threads every
        // launch of this library uses; __lane_id()'s mbcnt pair cost the expand 0.8 us, r06d A/B)
        const bool upper = (threadIdx.x & O) != 0;
        if constexpr (O == 16) {
            const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
            return upper ? r[0] : r[1];
        } else {
            const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
            return upper ? r[0] : r[1];
        }
    }
}
template <int O>
__device__ __forceinline__ float xlane(float v) { return __builtin_bit_cast(float, xlane_u<O>(__builtin_bit_cast(uint32_t, v))); }
template <int O>
__device__ __forceinline__ int xlane(int v) { return (int)xlane_u<O>((uint32_t)v); }
template <int O>
__device__ __forceinline__ double xlane(double v) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    return __builtin_bit_cast(double, (uint64_t)xlane_u<O>((uint32_t)b) | (uint64_t)xlane_u<O>((uint32_t)(b >> 32)) << 32);
}
// the sum over the wave in __shfl_xor's butterfly order (o = 32 .. 1), bit for bit
template <typename T>
__device__ __forceinline__ T xlane_sum(T v) {
    v += xlane<32>(v);
    v += xlane<16>(v);
    v += xlane<8>(v);
    v += xlane<4>(v);
    v += xlane<2>(v);
    return v + xlane<1>(v);
}
// lane f's value (f wave-uniform): v_readlane instead of a ds_bpermute
__device__ __forceinline__ float lane_val(float v, int f) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), f));
}
// argmax butterfly over the wave: the largest value, the lowest index among equals, on every lane
// (the same pairs as a __shfl_xor butterfly, so the same result)
template <int O = 32>
__device__ __forceinline__ void wave_argmax_step(float& best, int& bj) {
    const float ob = xlane<O>(best);
    const int oj = xlane<O>(bj);
    if (ob > best || (ob == best && oj < bj)) {
        best = ob;
        bj = oj;
    }
    if constexpr (O > 1) wave_argmax_step<O / 2>(best, bj);
}
template <int O = 32>
__device__ __forceinline__ void wave_argmax_step(int& best, int& bj) {
    const int ob = xlane<O>(best);
    const int oj = xlane<O>(bj);
    if (ob > best || (ob == best && oj < bj)) {
        best = ob;
        bj = oj;
    }
    if constexpr (O > 1) wave_argmax_step<O / 2>(best, bj);
}

// ------------------------------------------------------------------ GreedyYachtPlayer
// Best immediate gain (score + the basic bonus when it crosses 63,000) over unused categories x
// combos of `dice` (nibbles, n of them), all 64 lanes together; *best_t = the first maximum in
// (category, combo) order.  stop_first_invalid: the scorer's walk stops at the first combo
// reaching past the carry (YachtPlayers.py:151-153); otherwise combos with max(comb) < n
// (the bid potential, :67).  INT_MIN when nothing is eligible.
__device__ inline int greedy_best_wave(uint64_t dice, int n, uint32_t used, int basic_before, bool stop_first_invalid,
                                       int lane, int* best_t) {
    const int lim = n >= 10 ? NCOMB : (n >= 5 ? n - 4 : 0);
    int best = INT_MIN, bt = 0x7FFFFFFF;
    for (int t = lane; t < NCAT * NCOMB; t += 64) {
        const int cat = t / NCOMB, ci = t - cat * NCOMB;
        if ((used >> cat) & 1u) continue;
        if (stop_first_invalid ? ci >= lim : c_tab.comb_max[ci] >= n) continue;
        const uint32_t pos = c_tab.comb_pos[ci];
        uint32_t chosen = 0;
#pragma unroll
        for (int k = 0; k < 5; k++) chosen |= (uint32_t)((dice >> (4 * ((pos >> (4 * k)) & 0xF))) & 0xF) << (4 * k);
        const int sc = 1000 * score_k(cat, chosen);
        const int gain = sc + ((cat < 6 && basic_before < 63000 && 63000 <= basic_before + sc) ? 35000 : 0);
        if (gain > best) {
            best = gain;
            bt = t;
        }
    }
    wave_argmax_step(best, bt);
    *best_t = bt;
    return best;
}
// _score_potential_after_bid  YachtPlayers.py:38-87 (bundle: 5 nibbles, or absent)
__device__ inline int greedy_potential_wave(const YkS& s, uint64_t bundle, bool has_bundle, int lane) {
    const uint64_t wa = s_pw(s, 0, 0);
    const int nc = wa_n(wa);
    const uint64_t dice = (wa & ((1ull << 40) - 1)) | (has_bundle ? bundle << (4 * nc) : 0ull);
    const int n = nc + (has_bundle ? 5 : 0);
    if (s_round(s) == 1) {
        int sum = 0, cnt[7] = {0, 0, 0, 0, 0, 0, 0};
        for (int i = 0; i < n; i++) {
            const int d = (int)((dice >> (4 * i)) & 0xF);
            sum += d;
            cnt[d] += 1;
        }
        int v = 1000 * sum, mx = 0;
        for (int f = 1; f <= 6; f++) mx = cnt[f] > mx ? cnt[f] : mx;
        if (mx >= 4) v += 6000;
        else if (mx == 3) v += 3000;
        const bool e1 = cnt[1] > 0, e2 = cnt[2] > 0, e3 = cnt[3] > 0, e4 = cnt[4] > 0, e5 = cnt[5] > 0, e6 = cnt[6] > 0;
        if ((e1 && e2 && e3 && e4) || (e2 && e3 && e4 && e5) || (e3 && e4 && e5 && e6)) v += 5000;
        return v;
    }
    if (n < 5) return 0;
    int basic;
    cat_sum(s_pw(s, 0, 1), s_pw(s, 0, 2), &basic);
    int t;
    const int best = greedy_best_wave(dice, n, (uint32_t)wa_used(wa), 1000 * basic, false, lane, &t);
    return best == INT_MIN ? 0 : best;
}
// GreedyYachtPlayer.play's heuristic (YachtPlayers.py:90-171, 199-214) on a canonical board,
// all 64 lanes together: the chosen action if it is valid, else -1 (the player then draws a
// random legal action).  The bid may encode past index 100 (bids up to 100,000, :124-127).
__device__ inline int greedy_heuristic_wave(const YkS& s, int lane) {
    const int round = s_round(s), phase = s_phase(s);
    if (phase == 0 && round != 13) {
        const uint64_t w0 = s.w[0];
        const int valA = greedy_potential_wave(s, (w0 >> 24) & 0xFFFFF, (w0 >> 5) & 1, lane);
        const int valB = greedy_potential_wave(s, (w0 >> 44) & 0xFFFFF, (w0 >> 6) & 1, lane);
        int target, gap;
        if (valA >= valB) {
            target = 0;
            gap = valA - valB > 0 ? valA - valB : 0;
        } else {
            target = 1;
            gap = valB - valA > 0 ? valB - valA : 0;
        }
        const int diff = total_with_bonus(s, 0) - total_with_bonus(s, 1);
        const double bid_k = 0.5 * ((double)gap / 1000.0) - 0.15 * ((double)diff / 1000.0);
        long bid = (long)rint(1000.0 * bid_k);  // python round(): half to even
        bid = bid > 100000 ? 100000 : (bid < 0 ? 0 : bid);
        bid = (bid / 500) * 500;
        const int a = target * BID_LEVELS + (int)(bid / 500);
        return a < NBID ? a : -1;
    }
    const uint64_t wa = s_pw(s, 0, 0);
    const int n = wa_n(wa);
    if (n < 5) return -1;  // the scorer returns 0, never valid in the score phase
    int basic;
    cat_sum(s_pw(s, 0, 1), s_pw(s, 0, 2), &basic);
    int t;
    const int best = greedy_best_wave(wa & ((1ull << 40) - 1), n, (uint32_t)wa_used(wa), 1000 * basic, true, lane, &t);
    if (best == INT_MIN) return -1;
    const int a = NBID + t;
    return phase == 1 ? a : -1;  // valid only in the score phase
}

// ------------------------------------------------------------------ softmax exp
// exp(x) for the policy softmax (x <= ~0): 2^t (1 + r ln 2) with t = x * log2e rounded and r its
// residual (the product's exact error by fma, plus x times log2e's f32 tail), so the result stays
// within about 1 ulp of exp(x) like the library expf / torch's CPU exp, where __expf's product
// rounding costs up to |x| * 2^-24 relative.  Six instructions (one v_exp_f32) against the
// library form's thirteen; results below 2^-126 are not needed (priors of that size are zeros to
// MCTS.py's renormalisation at f32) and follow v_exp_f32; exp_acc(-inf) = 0, NaN stays NaN.
__device__ __forceinline__ float exp_acc(float x) {
    constexpr float L2E = 1.44269504088896340736f, L2E_LO = 1.9259629890910904e-08f, LN2 = 0.693147180559945309f;
    const float t = x * L2E;
    const float r = t > -150.f ? fmaf(x, L2E_LO, fmaf(x, L2E, -t)) : 0.f;  // (x = -inf: fma gives NaN)
    const float e = __builtin_amdgcn_exp2f(t);
    return fmaf(e, r * LN2, e);
}
// ------------------------------------------------------------------ features
// c_tab.die_scale / round_feat recomputed in registers: a per-lane table index would be a vector
// load, and in k_forward that would retire only after the weight ring's first fill.  numpy computes
// them in float64 and rounds to float32; the correctly rounded f32 division of the same (exact)
// operands gives the same bits for every d in 0..15 and round in 0..13 (checked on the host: a
// float64 quotient of these operands never lies on an f32 rounding midpoint), at a third of the cost
__device__ __forceinline__ float die_scale(uint32_t d) { return ((float)d - 3.5f) / 3.5f; }
constexpr bool f32_feature_quotients_exact() {
    for (int d = 0; d < 16; d++)
        if (((float)d - 3.5f) / 3.5f != (float)(((double)d - 3.5) / 3.5)) return false;
    for (int r = 0; r < 16; r++)
        if ((float)r / 13.0f != (float)((double)r / 13.0)) return false;
    return true;
}
static_assert(f32_feature_quotients_exact(), "f32 feature quotients == numpy's float64-then-float32");
// state_to_vec  yacht/NNet.py:65-86 (bit-exact f32).  f(i) for i in [0, 59).  Branch-free: the lanes
// of a wave compute different features, and divergent branches would run every region's code for
// every lane; each region's value is computed from per-lane selects instead, with one die-value
// quotient for the carry and roll regions
__device__ inline float feature(const YkS& s, int i) {
    const int round = s_round(s), phase = s_phase(s);
    const bool carry = i >= 3 && i < 23, rolls = i >= 23 && i < 33, used = i >= 33 && i < 57;
    // the player and position within the region (carry: 10 dice, rolls: 5 per roll, used: 12)
    // (every shift below stays in 0 .. 63 for every lane, also where its value is not selected)
    const int rel = carry ? i - 3 : rolls ? i - 23 : used ? i - 33 : i >= 57 ? i - 57 : 0;
    const int per = carry ? 10 : rolls ? 5 : 12;
    const int p = (i >= 57) ? (rel & 1) : rel / per, k = (i >= 57) ? 0 : rel - p * per;
    const uint64_t wa = p ? s_pw(s, 1, 0) : s_pw(s, 0, 0);
    // the die of a carry / roll slot, and whether the slot holds one (else -1)
    const uint64_t src = rolls ? s.w[0] >> (24 + 20 * (p & 1)) : wa;
    const uint32_t die = (uint32_t)(src >> (4 * k)) & 0xFu;
    const bool has = rolls ? (phase == 0 && round != 13 && ((s.w[0] >> (5 + (p & 1))) & 1)) : k < wa_n(wa);
    const float dv = has ? die_scale(die) : -1.0f;
    const float uv = (float)((wa_used(wa) >> k) & 1);
    const float bv = (float)((double)wc_bid(p ? s_pw(s, 1, 2) : s_pw(s, 0, 2)) * 1e-5);
    const float r0 = (float)round / 13.0f;  // (= float32(round / 13.0), die_scale above)
    return i == 0 ? r0 : i == 1 ? (phase == 0 ? 1.0f : 0.0f) : i == 2 ? (phase == 1 ? 1.0f : 0.0f)
         : (carry || rolls) ? dv : used ? uv : bv;
}

}  // namespace yk
