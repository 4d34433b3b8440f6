// yk_engine.hip - batched self-play: Coach.executeEpisode (Coach.py:34-72) driving
// MCTS.getActionProb / MCTS.search (MCTS.py:28-164) for thousands of games in lock-step.
//
// Lock-step semantics.  Every game runs simulation k of move m at the same time:
//   k_select         one wavefront per game walks its own tree from the root (UCB argmax
//                    over the compact valid set, transitions with the game's own RNG
//                    stream) to the first unexpanded state, a terminal, or a dead node;
//   k_forward        one batched f32-MFMA forward over all pending leaves (yk_net.hip);
//   k_expand_backup  one wavefront per game: exp(log_softmax), mask, numpy-pairwise
//                    renormalise, insert the node, back the value up the path.
// Within a game the simulations stay strictly sequential, so each game reproduces the
// reference's recursive search exactly (no virtual loss); only different games overlap.
//
// Data layout (per game): open-addressing index of node ids keyed by the
// 64-byte packed state; 96-byte node records; one arena holding, per expanded node, its
// prior P over the compact valid set (f32) and a u16 edge slot per valid action; 16-byte
// edges {Q (f64 value + python-type tag), N}.  Node/edge pools are double-buffered; at a
// real round change the survivors (round >= the root's round - the only nodes a game can
// ever reach again, since round_no never decreases) are compacted into the other buffer.
#include <math.h>

#include <algorithm>
#include <vector>

#include "yk_api.h"
#include "yk_common.h"
#include "yk_net.h"

#define YK_MAX_GROUPS 8

using namespace yk;

namespace {

constexpr int MAXD = 64;          // max search depth (path entries)
constexpr int LUT_N = 1 << 16;    // f32(sqrt(Ns)), f32(sqrt(Ns + 1e-8)) table size
constexpr int GAMES_PER_BLOCK = 4;
constexpr int GROUP_ALIGN = 16;   // group boundaries on forward row tiles
constexpr int YK_EXPAND_WPE = 4;  // waves per SIMD the expand kernel is register-budgeted for
// The root's incremental UCB scan: per tree, the root's compact set sorted by P
// (descending, ascending index on ties) and the list of its visited edges, valid for one move
constexpr int RO_CAP = 3072;      // >= the largest compact valid set (3024)
constexpr int RO_K = 512;         // entries of the order kept: the top RO_K by (P, -j); the walk needs
                                  // about (visited edges + 1) of them, and past them falls back to a full scan
constexpr int RV_CAP = 1024;      // visited root edges kept; more -> the move falls back to full scans
constexpr uint32_t RV_OFF = 0xFFFFFFFFu;

// python value kinds on the search path (MCTS.py:82, 115, 147)
enum : uint32_t { T_INT = 0, T_F64 = 1, T_F32 = 2 };

struct NodeRec {          // 96 bytes
    uint64_t key[8];      // packed canonical state
    uint64_t hash;
    uint64_t vinfo;       // cats nibbles [0:48] | k [48:52] | n [52:56] | W [56:64]
    uint32_t p_off;       // arena offset (entries) of P / slots
    uint32_t nvalid;
    uint32_t Ns;
    uint32_t pad;
};
struct Edge {             // 16 bytes
    double Q;
    uint32_t N;
    uint32_t tag;         // [0:2) python value kind of Q; [2:32) child node id + 1 when the edge's
                          // transition draws no dice (0: not known) - a revisit then skips the
                          // step, the canonical form and the index probe (section 6)
};
__device__ __forceinline__ uint32_t edge_kind(uint32_t tag) { return tag & 3u; }
constexpr uint32_t PATH_DET = 0x80000000u;  // path entry low word: node id | PATH_DET when the
                                            // level's transition consumed no random draw

constexpr int GST = 16;  // per-game counters (gstats)
struct EngDev {
    int E, NCAP, HCAP, ECAP, M, VCAP;
    int e_lo, e_hi;        // the game group a per-game launch covers ([0, E) unless pipelined)
    int T, dual;           // trees: T = E, or 2E with dual trees (one per arena seat: tree e is the
                           // agent's, tree E + e the opponent's - two MCTS objects, Coach.py:120-125)
    int64_t AE;
    int sims, temp_threshold;
    float c32;
    int prior;  // 0 net, 1 hash
    int fparts; // forward head split: workgroups per 16-row tile (mlse holds fparts partials [p][E])
    int rec_pred, max_exp, rec_stride;  // record_predictions: games e % rec_stride == 0, slot e / rec_stride
    int arena;             // 1 while yk_arena runs
    int arena_agent, arena_opp;  // YK_PLAYER_* of the seat-agent_seat player and of the other seat
    uint64_t seed;
    NodeRec* nodes[2];
    uint32_t* hidx[2];
    Edge* edges[2];
    uint32_t* node_count;  // [2][E]
    uint32_t* edge_count;  // [2][E]
    float* arenaP;
    uint16_t* arenaS;
    uint32_t* arena_top;   // [E]
    uint8_t* gen;          // [T]
    uint8_t* cur_round;    // [T]
    uint4* root_c;         // [T][2] the move's root once a descent found it: {id + 1 (0: not yet), p_off,
                           //        nvalid, entries of its P order}, {vinfo lo, hi, visited root edges in
                           //        rv (RV_OFF: no P order this move), walk start: the order's entries
                           //        before it are all visited}; one 32-byte read for root_scan
    int ro_k;              // entries of the root's order k_root_sort keeps (RO_K; YK_ROOT_K for the tests)
    uint32_t* rv;          // [T][RV_CAP] j | slot << 12 of each visited root edge
    uint16_t* ro_j;        // [T][RO_K] the root's top compact indices by descending P (ascending j on ties)
    float* ro_p;           // [T][RO_K] their P
    // game state
    yk_state_t* board;
    int32_t* cur;
    uint64_t* ctr;
    uint32_t* env_id;
    uint8_t* done;
    int32_t* nmoves;
    yk_state_t* root;
    int32_t* seat;         // [E] arena: the agent's seat (1 / -1)
    uint8_t* idle;         // [E] arena: a non-MCTS player is to move (no search this move)
    // per-sim
    yk_state_t* leaf_state;
    uint64_t* leaf_hash;
    uint8_t* leaf_flag;
    uint64_t* path;        // [E][MAXD]: (p_off + j) << 32 | node id
    uint8_t* path_len;
    uint32_t* end_node;    // [E] id + 1 of the node the descent stopped at (no valid action), else 0
    double* res_v;
    uint32_t* res_t;
    const float* logits;   // [E][PI_LD]
    const float* vpred;    // [E]
    const float2* mlse;    // [E] per-row (max, log sum exp) of the logits, from the forward; with
                           // fparts > 1, [fparts][E] raw partials (max, sum exp) merged by the expand
    const float* lut_sq;
    const float* lut_sqe;
    // records
    yk_state_t* rec_state; // [E][M]
    int32_t* rec_info;     // [E][M][8]
    uint64_t* rec_ctr;     // [E][M][2]
    double* rec_val;       // [E][M]
    uint32_t* rec_visits;  // [E][VCAP]: action << 16 | N
    int32_t* rec_voff;     // [E][M+1]
    double* final_r;       // [E]
    int32_t* final_cur;    // [E]
    int32_t* final_tot;    // [E][2] score totals with bonus (getGameEnded, YachtGame.py:408-428)
    float* rec_pi;         // [R][max_exp][3226]  (record_predictions; R = ceil(E / rec_stride))
    float* rec_v;          // [R][max_exp]
    yk_state_t* rec_leaf;  // [R][max_exp] the expanded leaf (canonical state)
    // stats
    uint64_t* gstats;      // [E][GST]: expansions, scanned, path edges, vnew, max nodes, max edges, max arena, sims,
                           // edge gathers of the UCB scans
    uint32_t* err;         // [1] error bits
};

enum : uint32_t {
    ERR_NODES = 1u, ERR_EDGES = 2u, ERR_ARENA = 4u, ERR_DEPTH = 8u, ERR_STEP = 16u, ERR_ROUND = 32u,
    ERR_VISITS = 64u, ERR_MOVES = 128u, ERR_ZERO_COUNTS = 256u, ERR_ROOT = 512u, ERR_HASH = 1024u,
    ERR_FWD_SYNC = 2048u  // a forward's value head timed out on its v_head.2 hand-off (the net's flag word)
};

// numpy float32 pairwise-sum plan for n = 3226 (loops_utils.h.src @TYPE@_pairwise_sum)
struct PwPlan {
    int nleaf, nop, root;
    uint16_t start[64], len[64];
    uint8_t a[64], b[64];
};
constexpr int pw_build(PwPlan& p, int start, int n) {
    if (n <= 128) {
        p.start[p.nleaf] = (uint16_t)start;
        p.len[p.nleaf] = (uint16_t)n;
        return p.nleaf++;
    }
    int n2 = n / 2;
    n2 -= n2 % 8;
    const int l = pw_build(p, start, n2);
    const int r = pw_build(p, start + n2, n - n2);
    p.a[p.nop] = (uint8_t)l;
    p.b[p.nop] = (uint8_t)r;
    return 64 + p.nop++;
}
constexpr PwPlan make_plan() {
    PwPlan p{};
    p.root = pw_build(p, 0, ASIZE);
    return p;
}
static __constant__ PwPlan c_pw = make_plan();
static_assert(make_plan().nleaf <= 64 && make_plan().nop <= 64, "pairwise plan too large");
// The expand kernel evaluates the plan as a register butterfly: that is exact iff the tree is
// perfect over 32 in-order leaves, every leaf 8-aligned with 8 <= len <= 128.
constexpr bool plan_is_butterfly() {
    const PwPlan p = make_plan();
    if (p.nleaf != 32 || p.nop != 31) return false;
    int first[128] = {}, cnt[128] = {};
    for (int i = 0; i < p.nleaf; i++) {
        if (p.start[i] % 8 != 0 || p.len[i] < 8 || p.len[i] > 128) return false;
        if (i > 0 && p.start[i] != p.start[i - 1] + p.len[i - 1]) return false;
        first[i] = i;
        cnt[i] = 1;
    }
    for (int o = 0; o < p.nop; o++) {
        const int a = p.a[o], b = p.b[o];
        if (cnt[a] != cnt[b] || first[a] + cnt[a] != first[b] || first[a] % (2 * cnt[a]) != 0) return false;
        first[64 + o] = first[a];
        cnt[64 + o] = 2 * cnt[a];
    }
    return p.root == 64 + p.nop - 1 && cnt[p.root] == 32;
}
static_assert(plan_is_butterfly(), "numpy's pairwise tree for 3226 is no longer a perfect 32-leaf tree");
constexpr int pw_gmax() {
    const PwPlan p = make_plan();
    int g = 0;
    for (int i = 0; i < p.nleaf; i++) g = p.len[i] / 8 > g ? p.len[i] / 8 : g;
    return g;
}
constexpr int pw_tmax() {
    const PwPlan p = make_plan();
    int t = 0;
    for (int i = 0; i < p.nleaf; i++) t = p.len[i] % 8 > t ? p.len[i] % 8 : t;
    return t;
}
constexpr int PW_GMAX = pw_gmax();  // 8-element groups in the longest leaf
constexpr int PW_TMAX = pw_tmax() > 0 ? pw_tmax() : 1;  // longest n % 8 tail

// getValidMoves of player 1 as wave-uniform scalars (the same test as action_valid)
struct ValidQ {
    int mode;       // 1: bid phase (a < 202), 0: score phase, -1: nothing valid
    int n;          // carry length
    uint32_t used;  // used categories
    __device__ __forceinline__ bool operator()(int a) const {
        if (mode == 1) return a < NBID;
        if (mode != 0 || a < NBID) return false;
        const int base = a - NBID, cat = base / NCOMB, ci = base - cat * NCOMB;
        if ((used >> cat) & 1u) return false;
        // the two carry sizes of real play need no table: 10 dice -> every combo, 5 -> combo 0
        if (n >= 10) return true;
        if (n == 5) return ci == 0;
        return c_tab.comb_max[ci] < n;
    }
};
__device__ __forceinline__ ValidQ valid_q(const YkS& s) {
    ValidQ q;
    const int round = s_round(s), phase = s_phase(s);
    const uint64_t wa = s_pw(s, 0, 0);
    q.n = __builtin_amdgcn_readfirstlane(wa_n(wa));
    q.used = __builtin_amdgcn_readfirstlane((uint32_t)wa_used(wa));
    q.mode = __builtin_amdgcn_readfirstlane((phase == 0 && round != 13) ? 1 : (phase == 1 && q.n >= 5) ? 0 : -1);
    return q;
}

__device__ __forceinline__ YkS ld_state(const yk_state_t* p) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    YkS s;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        uint4 v = q[k];
        s.w[2 * k] = (uint64_t)v.x | ((uint64_t)v.y << 32);
        s.w[2 * k + 1] = (uint64_t)v.z | ((uint64_t)v.w << 32);
    }
    return s;
}
__device__ __forceinline__ void st_state(yk_state_t* p, const YkS& s) {
    uint4* q = reinterpret_cast<uint4*>(p);
#pragma unroll
    for (int k = 0; k < 4; k++)
        q[k] = make_uint4((uint32_t)s.w[2 * k], (uint32_t)(s.w[2 * k] >> 32), (uint32_t)s.w[2 * k + 1],
                          (uint32_t)(s.w[2 * k + 1] >> 32));
}
__device__ __forceinline__ bool key_eq(const NodeRec& r, const YkS& s) {
    bool eq = true;
#pragma unroll
    for (int i = 0; i < 8; i++) eq &= r.key[i] == s.w[i];
    return eq;
}
__device__ __forceinline__ uint64_t pack_vinfo(const VInfo& v) {
    return (v.cats & 0xFFFFFFFFFFFFull) | ((uint64_t)v.k << 48) | ((uint64_t)v.n << 52) | ((uint64_t)v.W << 56);
}
__device__ __forceinline__ VInfo unpack_vinfo(uint64_t x, uint32_t V) {
    VInfo v;
    v.cats = x & 0xFFFFFFFFFFFFull;
    v.k = (int)((x >> 48) & 0xF);
    v.n = (int)((x >> 52) & 0xF);
    v.W = (int)(x >> 56);
    v.V = (int)V;
    return v;
}
__device__ __forceinline__ int pad4(int v) { return (v + 3) & ~3; }

// The transposition index's hash of a packed state: 32-bit multiply-rotate over the 16 words
// (the index only needs spread; a key compare settles every probe).  key_hash (yk_common.h, the
// spec's) is computed only where the hash prior needs it.
__device__ __forceinline__ uint64_t index_hash(const YkS& s) {
    uint32_t a = 0x9E3779B9u, b = 0x85EBCA6Bu;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        a = (a ^ (uint32_t)s.w[i]) * 0xCC9E2D51u;
        a = (a << 15) | (a >> 17);
        b = (b ^ (uint32_t)(s.w[i] >> 32)) * 0x1B873593u;
        b = (b << 13) | (b >> 19);
    }
    a ^= b * 0x85EBCA6Bu;
    a ^= a >> 16;
    a *= 0xC2B2AE35u;
    a ^= a >> 13;
    return ((uint64_t)b << 32) | a;
}

// open-addressing lookup; returns node id or -1.  Uniform across the wave.
__device__ __forceinline__ int lookup(const EngDev& d, int g, int t, const YkS& s, uint64_t h) {  // t: tree
    const uint32_t* hx = d.hidx[g] + (long)t * d.HCAP;
    const NodeRec* nodes = d.nodes[g] + (long)t * d.NCAP;
    const uint32_t mask = (uint32_t)d.HCAP - 1;
    uint32_t slot = (uint32_t)h & mask;
    for (int probe = 0; probe < d.HCAP; probe++) {
        const uint32_t v = hx[slot];
        if (v == 0) return -1;
        const NodeRec& r = nodes[v - 1];
        if (r.hash == h && key_eq(r, s)) return (int)(v - 1);
        slot = (slot + 1) & mask;
    }
    return -1;
}
__device__ __forceinline__ bool insert_index(const EngDev& d, int g, int t, uint64_t h, uint32_t id) {
    uint32_t* hx = d.hidx[g] + (long)t * d.HCAP;
    const uint32_t mask = (uint32_t)d.HCAP - 1;
    uint32_t slot = (uint32_t)h & mask;
    for (int probe = 0; probe < d.HCAP; probe++) {
        if (hx[slot] == 0) {
            hx[slot] = id + 1;
            return true;
        }
        slot = (slot + 1) & mask;
    }
    return false;
}

// the tree game e searches with at its current move: its own, or with dual trees the one of the
// seat to move (the agent's tree e, the opponent's tree E + e)
__device__ __forceinline__ int tree_of(const EngDev& d, int e) {
    return (d.dual && d.cur[e] != d.seat[e]) ? e + d.E : e;
}

// orders this wave's LDS / global accesses across lanes (waves of a block diverge, so no
// __syncthreads in per-game code)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ float wave_max(float v) {
    v = fmaxf(v, xlane<32>(v));
    v = fmaxf(v, xlane<16>(v));
    v = fmaxf(v, xlane<8>(v));
    v = fmaxf(v, xlane<4>(v));
    v = fmaxf(v, xlane<2>(v));
    return fmaxf(v, xlane<1>(v));
}
__device__ __forceinline__ float softmax_p(float x, float m, float lse) { return exp_acc(x - m - lse); }  // yk_common.h
__device__ __forceinline__ float wave_sumf(float v) {  // __shfl_xor's butterfly, bit for bit
    v += xlane<32>(v);
    v += xlane<16>(v);
    v += xlane<8>(v);
    v += xlane<4>(v);
    v += xlane<2>(v);
    return v + xlane<1>(v);
}
__device__ __forceinline__ int wave_min_i(int v) {
    v = min(v, xlane<32>(v));
    v = min(v, xlane<16>(v));
    v = min(v, xlane<8>(v));
    v = min(v, xlane<4>(v));
    v = min(v, xlane<2>(v));
    return min(v, xlane<1>(v));
}

// ------------------------------------------------------------------ python-typed arithmetic
// NEP 50 weak-scalar rules of numpy 2 (verified bitwise): any float32
// operand makes the result float32 (python ints/floats are cast to f32 first); python
// float with int -> float64; int / int -> float64 (true division).
struct PyV {
    double v;
    uint32_t t;
};
__device__ __forceinline__ PyV pv_update(PyV q, uint32_t n, PyV v) {  // (n*q + v) / (n+1)  MCTS.py:155-156
    PyV prod, sum, out;
    if (q.t == T_F32) prod = PyV{(double)((float)n * (float)q.v), T_F32};
    else prod = PyV{(double)n * q.v, q.t};
    if (prod.t == T_F32 || v.t == T_F32) sum = PyV{(double)((float)prod.v + (float)v.v), T_F32};
    else if (prod.t == T_F64 || v.t == T_F64) sum = PyV{prod.v + v.v, T_F64};
    else sum = PyV{prod.v + v.v, T_INT};
    if (sum.t == T_F32) out = PyV{(double)((float)sum.v / (float)(n + 1)), T_F32};
    else out = PyV{sum.v / (double)(n + 1), T_F64};
    return out;
}

// ------------------------------------------------------------------ kernels
__global__ void k_lut(float* sq, float* sqe) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= LUT_N) return;
    sq[i] = (float)sqrt((double)i);
    sqe[i] = (float)sqrt((double)i + 1e-8);
}

// reset every tree (MCTS() per episode, Coach.py:93) and, for self-play, start the games
__global__ void k_reset(EngDev d, int start_games, uint32_t env_base) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= d.E) return;
    for (int t = e; t < d.T; t += d.E) {  // the game's tree(s)
        d.node_count[t] = d.node_count[d.T + t] = 0;
        d.edge_count[t] = d.edge_count[d.T + t] = 0;
        d.arena_top[t] = 0;
        d.gen[t] = 0;
        d.cur_round[t] = 0;
        d.root_c[2 * t] = make_uint4(0, 0, 0, 0);
        d.root_c[2 * t + 1] = make_uint4(0, 0, RV_OFF, 0);
    }
#pragma unroll
    for (int k = 0; k < GST; k++) d.gstats[(long)e * GST + k] = 0;
    if (!start_games) return;
    d.env_id[e] = env_base + (uint32_t)e;
    Stream rs{d.seed, d.env_id[e], 0};
    YkS s;
#pragma unroll
    for (int k = 0; k < 8; k++) s.w[k] = 0;
    s.w[0] = 1ull | NO_BIDS;  // getInitBoard  YachtGame.py:232-237
    new_round_rolls(s, rs);
    st_state(d.board + e, s);
    d.cur[e] = 1;
    d.ctr[e] = rs.ctr;
    d.done[e] = 0;
    d.nmoves[e] = 0;
    d.rec_voff[(long)e * (d.M + 1)] = 0;
}

// Per move: root = canonical(board, cur)  (Coach.py:57); on a real round change compact the
// game's tree into the other buffer, keeping nodes whose round >= the root's.  One wave per game.
__global__ __launch_bounds__(256) void k_move_begin(EngDev d, int move, int external_root) {
    const int lane = threadIdx.x & 63;
    const int e = d.e_lo + blockIdx.x * GAMES_PER_BLOCK + (threadIdx.x >> 6);
    if (e >= d.e_hi) return;
    const int t = tree_of(d, e);
    if (lane == 0) {
        d.root_c[2 * t] = make_uint4(0, 0, 0, 0);  // ids move at a compaction: look the root up afresh
        d.root_c[2 * t + 1] = make_uint4(0, 0, RV_OFF, 0);  // the sorted root: rebuilt after the first expansion
    }
    if (!external_root) {
        if (d.done[e]) return;
        const YkS b = ld_state(d.board + e);
        const YkS r = canonical(b, d.cur[e]);
        const bool idle = d.arena && (d.cur[e] == d.seat[e] ? d.arena_agent : d.arena_opp) != YK_PLAYER_MCTS;
        if (lane == 0) {
            st_state(d.root + e, r);
            d.rec_ctr[((long)e * d.M + move) * 2] = d.ctr[e];
            d.idle[e] = idle ? 1 : 0;
        }
        if (idle) return;  // Arena: the random / greedy players do not search (YachtPlayers.py:174-214)
    } else if (lane == 0) {
        d.idle[e] = 0;
    }
    const YkS r = ld_state(d.root + e);
    const int rr = s_round(r);
    const int cr = d.cur_round[t];
    if (rr == cr) return;
    if (rr < cr) {
        if (lane == 0) atomicOr(d.err, ERR_ROUND);
        return;
    }
    // ---- compaction g -> g ^ 1 (in-place for the arena: survivors only move down)
    const int g = d.gen[t], h = g ^ 1;
    uint32_t* hx = d.hidx[h] + (long)t * d.HCAP;
    for (int i = lane; i < d.HCAP; i += 64) hx[i] = 0;
    const NodeRec* src = d.nodes[g] + (long)t * d.NCAP;
    NodeRec* dst = d.nodes[h] + (long)t * d.NCAP;
    const Edge* esrc = d.edges[g] + (long)t * d.ECAP;
    Edge* edst = d.edges[h] + (long)t * d.ECAP;
    float* P = d.arenaP + (long)t * d.AE;
    uint16_t* S = d.arenaS + (long)t * d.AE;
    const uint32_t cnt = d.node_count[g * d.T + t];
    uint32_t nn = 0, ne = 0, top = 0;
    wave_sync();
    // 64 records' rounds at a time (one load per lane), then the survivors in id order: the
    // records of earlier rounds cost no serial round trip
    for (uint32_t b0 = 0; b0 < cnt; b0 += 64) {
    const uint32_t il = b0 + (uint32_t)lane;
    uint64_t live = __ballot(il < cnt && (int)(src[il < cnt ? il : 0].key[0] & 0xF) >= rr);
    while (live) {
        const uint32_t id = b0 + (uint32_t)__builtin_ctzll(live);
        live &= live - 1;
        NodeRec rec = src[id];
        const int V = (int)rec.nvalid, VP = pad4(V);
        const uint32_t so = rec.p_off;
        for (int j0 = 0; j0 < VP; j0 += 64) {
            const int j = j0 + lane;
            float p = 0.f;
            uint16_t sl = 0;
            if (j < VP) {
                p = P[so + j];
                sl = S[so + j];
            }
            const bool vis = j < V && sl != 0;
            const uint64_t bal = __ballot(vis);
            const uint32_t before = __popcll(bal & ((1ull << lane) - 1));
            uint16_t nsl = 0;
            if (vis) {
                Edge x = esrc[sl - 1];
                x.tag = edge_kind(x.tag);  // node ids change: the cached child is dropped
                edst[ne + before] = x;
                nsl = (uint16_t)(ne + before + 1);
            }
            ne += (uint32_t)__popcll(bal);
            if (j < VP) {
                P[top + j] = p;
                S[top + j] = nsl;
            }
        }
        rec.p_off = top;
        top += (uint32_t)VP;
        if (lane == 0) {
            dst[nn] = rec;
            insert_index(d, h, t, rec.hash, nn);
        }
        nn++;
    }
    }
    if (lane == 0) {
        d.node_count[h * d.T + t] = nn;
        d.edge_count[h * d.T + t] = ne;
        d.arena_top[t] = top;
        d.gen[t] = (uint8_t)h;
        d.cur_round[t] = (uint8_t)rr;
    }
}


// The root's UCB argmax (MCTS.py:117-135) without scanning its whole compact set: the root is the
// same node for all of a move's simulations, and between two of them only one of its edges changes.
// An unvisited edge's u = (c P) sqrt(Ns + 1e-8) is monotone in P, so the best unvisited edge is the
// first unvisited entry of the root's P order (k_root_sort), and entries of equal u - the band that
// follows it in that order - go to the lowest index (strict '>' in ascending action order).  The
// visited edges (the list the backups append to) are scanned as before.  Same f32 operations as the
// full scan, so the same winner, bit for bit.  Returns the winner's compact index (0x7FFFFFFF: none)
// and its edge tag (0: unvisited), or -1 when the order's nk stored entries end before the walk does
// (the caller then scans the whole set); `scanned` counts the entries read.
__device__ __forceinline__ int root_scan(const EngDev& d, int t, int lane, uint32_t nv, const float* P,
                                         const uint16_t* S, const Edge* edges, int V, int nk, int ws, float sq,
                                         float sqe, uint32_t& wtag, uint64_t& scanned, uint64_t& gathered) {
    const uint16_t* oj = d.ro_j + (long)t * RO_K;
    const float* op = d.ro_p + (long)t * RO_K;
    const uint32_t* rv = d.rv + (long)t * RV_CAP;
    // the walk starts at ws (every entry before it is visited: a visit is never undone within a
    // move); its first piece is loaded beside the visited list
    int jj = ws + lane < nk ? (int)oj[ws + lane] : 0;
    float pp = ws + lane < nk ? op[ws + lane] : 0.f;
    float best = -INFINITY;
    int bj = 0x7FFFFFFF;
    uint32_t btag = 0;
    for (uint32_t i = (uint32_t)lane; i < nv; i += 64) {
        const uint32_t w = rv[i];
        const int j = (int)(w & 0xFFFu);
        const float p = P[j];
        const Edge ev = edges[(w >> 12) - 1];
        const float u = (float)ev.Q + ((d.c32 * p) * sq) / (float)(ev.N + 1);
        if (u > best || (u == best && j < bj)) {
            best = u;
            bj = j;
            btag = ev.tag;
        }
    }
    float ub = -INFINITY;
    int uj = 0x7FFFFFFF;
    bool found = false, done = false;
    int walked = 0;  // entries of the order read
    int first = nk;   // the order's first unvisited entry: the next walk's start
    for (int k0 = ws; k0 < nk; k0 += 64) {
        const int k = k0 + lane;
        if (k0 != ws) {
            jj = k < nk ? (int)oj[k] : 0;
            pp = k < nk ? op[k] : 0.f;
        }
        walked = min(k0 + 64, nk) - ws;
        const bool in = k < nk;
        const bool unv = in && S[jj] == 0;
        const float u = (d.c32 * pp) * sqe;
        bool cand;
        if (!found) {
            const uint64_t bal = __ballot(unv);
            if (!bal) continue;  // every entry of this piece is visited
            const int f = __builtin_ctzll(bal);
            ub = lane_val(u, f);
            found = true;
            first = k0 + f;
            cand = unv && lane >= f && u == ub;
        } else {
            cand = unv && u == ub;
        }
        uj = min(uj, wave_min_i(cand ? jj : 0x7FFFFFFF));
        // u is non-increasing along the order: the band goes on into the next piece only if the
        // piece's last entry still has u == ub
        if (!(k0 + 64 < nk && lane_val(u, 63) == ub)) {
            done = k0 + 64 < nk || nk == V || lane_val(u, (nk - 1 - k0) & 63) != ub;
            break;
        }
    }
    if (lane == 0 && first != ws) d.root_c[2 * t + 1].w = (uint32_t)first;
    if (!done && nk < V) {  // the stored order ended first: no unvisited entry among the top nk, or
        scanned += (uint64_t)nv + (uint64_t)walked;  // a band of equal u that may go on past them
        gathered += (uint64_t)nv;                     // (one edge per visited-list entry)
        return -1;
    }
    if (lane == 0 && found && (ub > best || (ub == best && uj < bj))) {
        best = ub;
        bj = uj;
        btag = 0;
    }
    const int mine = bj;
    wave_argmax_step(best, bj);
    const uint64_t own = __ballot(mine == bj);  // the lane whose own candidate won holds its tag
    wtag = own ? __builtin_amdgcn_readlane(btag, (int)__builtin_ctzll(own)) : 0u;
    scanned += (uint64_t)nv + (uint64_t)walked;
    gathered += (uint64_t)nv;
    return bj;
}

// One simulation's descent (MCTS.search, MCTS.py:56-152 up to the recursion).
// All 64 lanes of the game's wave call it together.
__device__ __forceinline__ void select_game(const EngDev& d, int e, int lane, const uint32_t* env_ids, uint64_t* ctr_arr) {
    if (d.done[e] || d.idle[e]) {
        if (lane == 0) {
            d.leaf_flag[e] = 0;
            d.path_len[e] = 0;
            d.end_node[e] = 0;
        }
        return;
    }
    const int t = tree_of(d, e);
    const int g = d.gen[t];
    YkS s = ld_state(d.root + e);
    Stream rs{d.seed, env_ids[e], ctr_arr[e]};
    const NodeRec* nodes = d.nodes[g] + (long)t * d.NCAP;
    const Edge* edges = d.edges[g] + (long)t * d.ECAP;
    const float* Pbase = d.arenaP + (long)t * d.AE;
    const uint16_t* Sbase = d.arenaS + (long)t * d.AE;
    uint64_t* path = d.path + (long)e * MAXD;
    int depth = 0;
    uint64_t scanned = 0, gathered = 0;  // UCB entries read; their edges gathered (visited entries)
    int ngl = 0;                          // this lane's edge gathers in full scans
    int leaf = 0;
    int known = -1;        // the node this level's state is, when the edge taken to it cached it
    uint32_t end_id = 0;   // id + 1 of a node the descent stops at
    PyV res{0.0, T_INT};
    // the root's pick from its P order and visited list (root_scan), made before the walk, where
    // little else is live (inside the loop the second scan path would spill)
    bool pre = false;
    int pre_bj = 0x7FFFFFFF;
    uint32_t pre_tag = 0;
    {
        const uint4 rc = d.root_c[2 * t], rc1 = d.root_c[2 * t + 1];
        if (rc.x != 0 && rc1.z != RV_OFF) {  // k_root_sort ran this move: root_c holds the root
            const uint32_t Ns = nodes[rc.x - 1].Ns;
            const float sq = (float)sqrt((double)Ns), sqe = (float)sqrt((double)Ns + 1e-8);
            pre_bj = __builtin_amdgcn_readfirstlane(root_scan(d, t, lane, rc1.z, Pbase + rc.y, Sbase + rc.y, edges,
                                                              (int)rc.z, (int)rc.w, (int)rc1.w, sq, sqe, pre_tag, scanned,
                                                              gathered));
            pre_tag = __builtin_amdgcn_readfirstlane(pre_tag);
            pre = pre_bj != -1;
        }
    }
    while (true) {
        if (known >= 0) {  // the cached child: its key is the state step + canonical would give
            const uint64_t* kp = nodes[known].key;
#pragma unroll
            for (int i = 0; i < 8; i++) s.w[i] = kp[i];
        }
        const double es = game_ended(s, 1);  // Es (MCTS.py:78-82)
        if (es != 0.0) {
            res = PyV{-es, T_F64};
            break;
        }
        // the root (depth 0) is the same node for every simulation of a move: its id and the
        // record's fixed fields are kept after the first lookup, which saves the hash, the index
        // probe and the record's round trip before the prior / slot loads
        uint4 rc0 = make_uint4(0, 0, 0, 0), rc1 = rc0;
        if (depth == 0) {
            rc0 = d.root_c[2 * t];
            rc1 = d.root_c[2 * t + 1];
        }
        const bool cached = rc0.x != 0;
        const uint64_t hsh = (cached || known >= 0) ? 0ull : index_hash(s);
        const int nid = cached ? (int)rc0.x - 1 : known >= 0 ? known : lookup(d, g, t, s, hsh);
        if (nid < 0) {  // leaf: predict (MCTS.py:84-115)
            leaf = 1;
            if (lane == 0) {
                st_state(d.leaf_state + e, s);
                d.leaf_hash[e] = hsh;
            }
            break;
        }
        const NodeRec& nd = nodes[nid];
        const uint32_t p_off = cached ? rc0.y : nd.p_off;
        const int V = cached ? (int)rc0.z : (int)nd.nvalid;
        const uint64_t vinfo = cached ? ((uint64_t)rc1.x | ((uint64_t)rc1.y << 32)) : nd.vinfo;
        if (depth == 0 && !cached && lane == 0) {
            d.root_c[2 * t] = make_uint4((uint32_t)nid + 1, p_off, (uint32_t)V, 0);
            d.root_c[2 * t + 1] = make_uint4((uint32_t)vinfo, (uint32_t)(vinfo >> 32), RV_OFF, 0);
        }
        if (V == 0) {  // no valid action: MCTS.py:141-147 returns 0 (python int)
            res = PyV{0.0, T_INT};
            end_id = (uint32_t)nid + 1;
            break;
        }
        // UCB argmax, MCTS.py:117-135: float32 arithmetic, strict '>' => lowest action wins
        const uint32_t Ns = nd.Ns;
        // f32(sqrt(Ns)), f32(sqrt(Ns + 1e-8)) (MCTS.py:125-129 under NEP 50): f64 sqrt is correctly
        // rounded, so these are the bits numpy gets; computed here rather than read from a table,
        // which saves a dependent load per level (expand 53.35 -> 53.02 us, profiles/r03_expand_ab.log)
        const float sq = (float)sqrt((double)Ns);
        const float sqe = (float)sqrt((double)Ns + 1e-8);
        const float* P = Pbase + p_off;
        const uint16_t* S = Sbase + p_off;
        int bj_out;
        uint32_t wtag;
        if (depth == 0 && pre) {  // the root: picked above from its P order and visited list
            bj_out = pre_bj;
            wtag = pre_tag;
        } else {
            float best = -INFINITY;
            int bj = 0x7FFFFFFF;
            uint32_t btag = 0;  // the edge tag of the lane's best entry (0: unvisited)
            // software-pipelined scan: iteration it+1's P / slot loads fly while iteration it's
            // visited-edge gathers resolve
            float4 p4 = make_float4(0.f, 0.f, 0.f, 0.f);
            ushort4 s4 = make_ushort4(0, 0, 0, 0);
            if (lane * 4 < V) {
                p4 = *reinterpret_cast<const float4*>(P + lane * 4);
                s4 = *reinterpret_cast<const ushort4*>(S + lane * 4);
            }
            for (int j0 = lane * 4; j0 < V; j0 += 256) {
                const float pv[4] = {p4.x, p4.y, p4.z, p4.w};
                const uint16_t sv[4] = {s4.x, s4.y, s4.z, s4.w};
                Edge ev[4];
#pragma unroll
                for (int t = 0; t < 4; t++)
                    if (j0 + t < V && sv[t]) {
                        ev[t] = edges[sv[t] - 1];
                        ngl++;
                    }
                if (j0 + 256 < V) {
                    p4 = *reinterpret_cast<const float4*>(P + j0 + 256);
                    s4 = *reinterpret_cast<const ushort4*>(S + j0 + 256);
                }
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    const int j = j0 + t;
                    if (j < V) {
                        float u;
                        const float cp = d.c32 * pv[t];
                        if (sv[t]) {
                            u = (float)ev[t].Q + (cp * sq) / (float)(ev[t].N + 1);
                        } else {
                            u = cp * sqe;
                        }
                        if (u > best) {
                            best = u;
                            bj = j;
                            btag = sv[t] ? ev[t].tag : 0u;
                        }
                    }
                }
            }
            wave_argmax_step(best, bj);
            scanned += (uint64_t)V;
            bj_out = bj;
            // the winner's lane holds its tag: its own best is the wave's (lowest j among equals)
            wtag = __builtin_amdgcn_readlane(btag, __builtin_amdgcn_readfirstlane((bj & 255) >> 2));
        }
        const int bj = bj_out;
        int j = bj;
        if (j == 0x7FFFFFFF) j = 0;  // MCTS.py:138-143: first valid action
        if (depth >= MAXD) {
            if (lane == 0) atomicOr(d.err, ERR_DEPTH);
            res = PyV{0.0, T_INT};
            break;
        }
        const uint32_t child = bj == 0x7FFFFFFF ? 0u : (wtag >> 2);  // id + 1, 0: not cached
        if (child) {  // a deterministic transition taken before: the child node is known
            if (lane == 0) path[depth] = ((uint64_t)(p_off + (uint32_t)j) << 32) | (uint32_t)nid | PATH_DET;
            depth++;
            known = (int)child - 1;
            continue;
        }
        known = -1;
        const VInfo vi = unpack_vinfo(vinfo, (uint32_t)V);
        const int a = compact_to_action(vi, j);
        int np = 1;
        const uint64_t ctr0 = rs.ctr;
        const int st = step_state<true>(s, 1, a, rs, np);  // MCTS.py:149 (all lanes: wave-parallel dice)
        const uint32_t det = rs.ctr == ctr0 ? PATH_DET : 0u;  // no dice drawn: the child is a function of (s, a)
        if (lane == 0) path[depth] = ((uint64_t)(p_off + (uint32_t)j) << 32) | (uint32_t)nid | det;
        depth++;
        if (st != YK_ST_OK) {
            if (lane == 0) atomicOr(d.err, ERR_STEP);
            res = PyV{0.0, T_INT};
            break;
        }
        s = canonical(s, np);  // MCTS.py:150
    }
    gathered += (uint64_t)xlane_sum(ngl);
    if (lane == 0) {
        d.leaf_flag[e] = (uint8_t)(leaf ? (t < d.E ? 1 : 2) : 0);  // which net predicts it (dual trees)
        d.path_len[e] = (uint8_t)depth;
        d.end_node[e] = end_id;
        d.res_v[e] = res.v;
        d.res_t[e] = res.t;
        ctr_arr[e] = rs.ctr;
        d.gstats[(long)e * GST + 1] += scanned;
        d.gstats[(long)e * GST + 2] += (uint64_t)depth;
        d.gstats[(long)e * GST + 7] += 1;
        d.gstats[(long)e * GST + 8] += gathered;
    }
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_select(EngDev d, const uint32_t* env_ids, uint64_t* ctr_arr) {
    const int lane = threadIdx.x & 63;
    const int e = d.e_lo + blockIdx.x * GAMES_PER_BLOCK + (threadIdx.x >> 6);
    if (e >= d.e_hi) return;
    select_game(d, e, lane, env_ids, ctr_arr);
}

// Leaf expansion (MCTS.py:84-115) and backup (MCTS.py:154-164) of this simulation, then -
// when do_select - the next simulation's descent for the same game (one kernel boundary per
// simulation fewer).  One wave per game.
__device__ __forceinline__ void expand_backup_game(const EngDev& d, int e, int lane);
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(YK_EXPAND_WPE))) void k_expand_backup(
    EngDev d, int do_select, const uint32_t* env_ids, uint64_t* ctr_arr) {
    const int lane = threadIdx.x & 63;
    const int e = d.e_lo + blockIdx.x * GAMES_PER_BLOCK + (threadIdx.x >> 6);
    if (e >= d.e_hi) return;
    if (d.done[e]) return;
    expand_backup_game(d, e, lane);
    if (do_select) {
        wave_sync();  // this wave's backup writes (edges, slots, Ns) precede its descent's reads
        select_game(d, e, lane, env_ids, ctr_arr);
    }
}

__device__ __forceinline__ void expand_backup_game(const EngDev& d, int e, int lane) {
    const int t = tree_of(d, e);
    const int g = d.gen[t];
    PyV res{d.res_v[e], d.res_t[e]};
    uint32_t end_id = 0;  // id + 1 of the node the path's last edge leads to, if any
    if (d.leaf_flag[e]) {
        const YkS s = ld_state(d.leaf_state + e);
        const uint64_t ihsh = d.leaf_hash[e];                  // the index's hash
        const uint64_t hsh = d.prior == 1 ? key_hash(s) : 0ull;  // the hash prior's (spec) hash
        const VInfo vi = valid_info(s, 1);
        const ValidQ valid = valid_q(s);
        const int V = vi.V;
        // ---- prior, Ps * valids (MCTS.py:88) and np.sum(Ps) (MCTS.py:89), in registers.
        // Lane pair (2k, 2k+1) owns leaf k of numpy's float32 pairwise tree for n = 3226 (32
        // in-order leaves, 8-aligned): lane 2k+h holds elements 8j + 4h .. 8j + 4h + 3 of the
        // leaf (numpy's accumulators r[4h .. 4h+3]) and, for h = 0, its n % 8 tail.
        const int leaf = lane >> 1, h = lane & 1;
        const int st = c_pw.start[leaf], nl = c_pw.len[leaf], G = nl >> 3, R = nl & 7;
        float4 q[PW_GMAX];
        float qt[PW_TMAX];
        float v, mx = 0.f, lse = 0.f;
        const int pidx = (int)d.gstats[(long)e * GST + 0];
        // record_predictions samples games without changing the path: the production prior
        // below is what gets recorded (after masking, i.e. exactly what np.sum / P see)
        const bool rec = d.rec_pred && (e % d.rec_stride) == 0 && pidx < d.max_exp;
        const long rslot = rec ? (long)(e / d.rec_stride) * d.max_exp + pidx : 0;
        bool masked = false;  // q / qt already hold Ps * valids
        if (d.prior == 0) {
            // pi = exp(log_softmax(logits)) (NNet.py:193) at the valid actions only: the forward
            // supplies each row's (max, log sum exp), so the invalid logits are never read
            const float* x = d.logits + (long)e * PI_LD + st;
            const float2 ml = d.mlse[e];
            mx = ml.x;
            lse = ml.y;
            if (d.fparts > 1) {  // merge the head parts' (max, sum exp), in part order
                float ms = ml.y;
                for (int p = 1; p < d.fparts; p++) {
                    const float2 q = d.mlse[(long)p * d.E + e];
                    const float mm = fmaxf(mx, q.x);
                    if (mm != -INFINITY) {
                        ms = ms * exp_acc(mx - mm) + q.y * exp_acc(q.x - mm);
                        mx = mm;
                    }
                }
                lse = logf(ms);
            }
            // score actions at 10 dice (most leaves): a group a .. a + 3 (a = 0 mod 4) holds at
            // most two categories, a's and a + 2's (category starts are 202 + 252 c = 2 mod 4)
            static_assert(NBID % 4 == 2 && NCOMB % 4 == 0, "category starts are 2 mod 4");
            const bool score10 = valid.mode == 0 && valid.n >= 10;
#pragma unroll
            for (int j = 0; j < PW_GMAX; j++) {
                const int a = st + 8 * j + 4 * h;
                bool v0, v1, v2, v3;
                if (score10) {
                    const int b0 = a - NBID, b2 = a + 2 - NBID;
                    const bool lo = j < G && b0 >= 0 && !((valid.used >> ((unsigned)b0 / NCOMB)) & 1u);
                    const bool hi = j < G && b2 >= 0 && !((valid.used >> ((unsigned)b2 / NCOMB)) & 1u);
                    v0 = v1 = lo;
                    v2 = v3 = hi;
                } else {
                    v0 = j < G && valid(a);
                    v1 = j < G && valid(a + 1);
                    v2 = j < G && valid(a + 2);
                    v3 = j < G && valid(a + 3);
                }
                float4 x4 = make_float4(0.f, 0.f, 0.f, 0.f);
                if (v0 || v1 || v2 || v3) x4 = *reinterpret_cast<const float4*>(x + 8 * j + 4 * h);
                q[j] = make_float4(v0 ? softmax_p(x4.x, mx, lse) : 0.f, v1 ? softmax_p(x4.y, mx, lse) : 0.f,
                                   v2 ? softmax_p(x4.z, mx, lse) : 0.f, v3 ? softmax_p(x4.w, mx, lse) : 0.f);
            }
#pragma unroll
            for (int r = 0; r < PW_TMAX; r++)
                qt[r] = (h == 0 && r < R && valid(st + 8 * G + r)) ? softmax_p(x[8 * G + r], mx, lse) : 0.f;
            v = d.vpred[e];
            masked = true;
        } else {
#pragma unroll
            for (int j = 0; j < PW_GMAX; j++) {
                const int a = st + 8 * j + 4 * h;
                q[j] = j < G ? make_float4(hash_prior_pi(hsh, a), hash_prior_pi(hsh, a + 1), hash_prior_pi(hsh, a + 2),
                                           hash_prior_pi(hsh, a + 3))
                             : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int r = 0; r < PW_TMAX; r++) qt[r] = (h == 0 && r < R) ? hash_prior_pi(hsh, st + 8 * G + r) : 0.f;
            v = hash_prior_v(hsh);
        }
        // mask with the valid moves
#pragma unroll
        for (int j = 0; j < PW_GMAX; j++) {
            const int a = st + 8 * j + 4 * h;
            if (j < G && !masked) {
                if (!valid(a)) q[j].x = 0.f;
                if (!valid(a + 1)) q[j].y = 0.f;
                if (!valid(a + 2)) q[j].z = 0.f;
                if (!valid(a + 3)) q[j].w = 0.f;
            }
        }
#pragma unroll
        for (int r = 0; r < PW_TMAX; r++)
            if (h == 0 && r < R && !masked && !valid(st + 8 * G + r)) qt[r] = 0.f;
        if (rec) {  // Ps * valids (MCTS.py:88) of this expansion, the leaf and v
            float* rpi = d.rec_pi + rslot * ASIZE;
#pragma unroll
            for (int j = 0; j < PW_GMAX; j++)
                if (j < G) *reinterpret_cast<float4*>(rpi + st + 8 * j + 4 * h) = q[j];
#pragma unroll
            for (int r = 0; r < PW_TMAX; r++)
                if (h == 0 && r < R) rpi[st + 8 * G + r] = qt[r];
            if (lane == 0) {
                d.rec_v[rslot] = v;
                st_state(d.rec_leaf + rslot, s);
            }
        }
        // numpy pairwise_sum on the leaf: r_k = a[k] + a[8 + k] + ..., then
        // ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)), then the tail one by one
        float4 racc = q[0];
#pragma unroll
        for (int j = 1; j < PW_GMAX; j++)
            if (j < G) {
                racc.x += q[j].x;
                racc.y += q[j].y;
                racc.z += q[j].z;
                racc.w += q[j].w;
            }
        const float half = (racc.x + racc.y) + (racc.z + racc.w);
        const float other = xlane<1>(half);
        float lsum = h == 0 ? half + other : other + half;
#pragma unroll
        for (int r = 0; r < PW_TMAX; r++)
            if (r < R) lsum += qt[r];  // h = 0 holds the tail
        lsum = __builtin_bit_cast(float, dpp_mov<0xA0>(__builtin_bit_cast(uint32_t, lsum)));  // quad_perm [0,0,2,2]: the even lane's
        // the perfect tree over the 32 leaves, left + right at every level
        float y = xlane<2>(lsum);
        lsum = (lane & 2) ? y + lsum : lsum + y;
        y = xlane<4>(lsum);
        lsum = (lane & 4) ? y + lsum : lsum + y;
        y = xlane<8>(lsum);
        lsum = (lane & 8) ? y + lsum : lsum + y;
        y = xlane<16>(lsum);
        lsum = (lane & 16) ? y + lsum : lsum + y;
        y = xlane<32>(lsum);
        lsum = (lane & 32) ? y + lsum : lsum + y;
        const float sum = lsum;
        // ---- allocate + write P over the compact valid set, zero edge slots
        const int VP = pad4(V);
        const uint32_t off = d.arena_top[t];
        const uint32_t nid = d.node_count[g * d.T + t];
        bool ok = true;
        if ((int64_t)off + VP > d.AE) {
            if (lane == 0) atomicOr(d.err, ERR_ARENA);
            ok = false;
        }
        if (nid >= (uint32_t)d.NCAP) {
            if (lane == 0) atomicOr(d.err, ERR_NODES);
            ok = false;
        }
        if (ok) {
            float* P = d.arenaP + (long)t * d.AE + off;
            uint16_t* S = d.arenaS + (long)t * d.AE + off;
            const float inv_fallback = V > 0 ? 1.0f / (float)V : 0.0f;
            // P over the compact valid set (ascending action): Ps / sum, or the uniform fallback
            // (MCTS.py:90-107).  Written in compact order (coalesced), recomputing each prior
            // exactly as above from the L2-resident logits row (or the hash).
            const float* __restrict__ xr = d.logits + (long)e * PI_LD;
            for (int j0 = lane; j0 < VP; j0 += 256) {  // four gathers in flight per lane
                float xa[4];
                int aa[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int j = j0 + 64 * u;
                    aa[u] = j < V ? compact_to_action(vi, j) : 0;
                    xa[u] = (d.prior == 0 && j < V) ? xr[aa[u]] : 0.f;
                }
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int j = j0 + 64 * u;
                    if (j < VP) {
                        float p = 0.0f;
                        if (j < V) {
                            const float pa = d.prior == 0 ? softmax_p(xa[u], mx, lse) : hash_prior_pi(hsh, aa[u]);
                            p = sum > 0.0f ? pa / sum : inv_fallback;
                        }
                        P[j] = p;
                        S[j] = 0;
                    }
                }
            }
            if (lane == 0) {
                NodeRec r;
#pragma unroll
                for (int i = 0; i < 8; i++) r.key[i] = s.w[i];
                r.hash = ihsh;
                r.vinfo = pack_vinfo(vi);
                r.p_off = off;
                r.nvalid = (uint32_t)V;
                r.Ns = 0;
                r.pad = 0;
                d.nodes[g][(long)t * d.NCAP + nid] = r;
                if (!insert_index(d, g, t, ihsh, nid)) atomicOr(d.err, ERR_HASH);
            }
            end_id = nid + 1;
            if (lane == 0) {
                d.node_count[g * d.T + t] = nid + 1;
                d.arena_top[t] = off + (uint32_t)VP;
                uint64_t* gs = d.gstats + (long)e * GST;
                gs[0] += 1;
                gs[3] += (uint64_t)V;
                if (nid + 1 > gs[4]) gs[4] = nid + 1;
                if (off + VP > gs[6]) gs[6] = off + VP;
            }
        }
        res = PyV{-(double)v, T_F32};  // return -v  (MCTS.py:115)
    } else {
        end_id = d.end_node[e];
    }
    // ---- backup (MCTS.py:154-164): the path's nodes are distinct, so every level updates in
    // parallel; level k receives v * (-1)^(depth-1-k) ("return -v" per level).
    const int depth = d.path_len[e];
    if (depth > 0) {
        NodeRec* nodes = d.nodes[g] + (long)t * d.NCAP;
        Edge* edges = d.edges[g] + (long)t * d.ECAP;
        uint16_t* Sb = d.arenaS + (long)t * d.AE;
        const uint64_t* path = d.path + (long)e * MAXD;
        const uint32_t ne0 = d.edge_count[g * d.T + t];
        uint64_t pe = 0;
        uint16_t sl = 0;
        if (lane < depth) {
            pe = path[lane];
            sl = Sb[pe >> 32];
        }
        // the child each level's edge leads to: the next level's node, or for the last edge the
        // node the descent ended at (the new leaf, or a node without valid actions); cached in
        // the edge's tag when that transition drew no dice
        const uint32_t pnext = __shfl((uint32_t)pe, (lane + 1) & 63, 64);
        const uint32_t cnode = lane + 1 < depth ? (pnext & ~PATH_DET) + 1 : end_id;
        const uint32_t cbits = ((uint32_t)pe & PATH_DET) ? cnode << 2 : 0u;
        const bool is_new = lane < depth && sl == 0;
        const uint64_t bal = __ballot(is_new);
        const uint32_t eid = ne0 + (uint32_t)__popcll(bal & ((1ull << lane) - 1));
        const uint32_t ne1 = ne0 + (uint32_t)__popcll(bal);
        if (lane < depth) {
            PyV v = res;
            if ((depth - 1 - lane) & 1) v.v = -v.v;
            if (sl) {
                Edge& ed = edges[sl - 1];
                const PyV q = pv_update(PyV{ed.Q, edge_kind(ed.tag)}, ed.N, v);
                ed.Q = q.v;
                ed.tag = q.t | cbits;
                ed.N += 1;
            } else if (eid < (uint32_t)d.ECAP && eid < 65535u) {
                edges[eid] = Edge{v.v, 1u, v.t | cbits};
                Sb[pe >> 32] = (uint16_t)(eid + 1);
            } else {
                atomicOr(d.err, ERR_EDGES);
            }
            nodes[(uint32_t)pe & ~PATH_DET].Ns += 1;
        }
        if (lane == 0) {
            d.edge_count[g * d.T + t] = ne1;
            uint64_t* gs = d.gstats + (long)e * GST;
            if (ne1 > gs[5]) gs[5] = ne1;
            // a new edge at level 0 (the move's root): into the root's visited list (root_scan)
            if (is_new && eid < (uint32_t)d.ECAP && eid < 65535u) {
                const uint32_t n = d.root_c[2 * t + 1].z;
                if (n != RV_OFF) {
                    const uint32_t j = (uint32_t)(pe >> 32) - d.root_c[2 * t].y;
                    if (n < (uint32_t)RV_CAP) {
                        d.rv[(long)t * RV_CAP + n] = j | ((eid + 1) << 12);
                        d.root_c[2 * t + 1].z = n + 1;
                    } else {
                        d.root_c[2 * t + 1].z = RV_OFF;  // too many: full scans for the rest of the move
                    }
                }
            }
        }
    }
}

// The root's P order for root_scan, once per move after its first expansion (the root is expanded
// by then, by this move's first simulation or an earlier search): the compact set sorted by P
// descending, ascending index on ties (a bitonic sort of 64-bit keys P bits << 32 | 0xFFFF - j in
// LDS; P >= 0, so its bits order as unsigned), and the list of the edges already visited.  One
// workgroup per game.  Leaves the root in full-scan mode when c <= 0 (the order is then not the
// UCB order), when the root has at most 256 valid actions (every bid node), or when its visited
// list would overflow.
__global__ __launch_bounds__(256) void k_root_sort(EngDev d) {
    constexpr int PT = (RO_CAP + 255) / 256;  // keys per thread
    __shared__ uint64_t sk[RO_K];
    __shared__ uint32_t hist[256];
    __shared__ int s_nid, s_need;
    __shared__ uint32_t s_nv, s_cnt;
    __shared__ uint64_t s_prefix;
    const int e = d.e_lo + (int)blockIdx.x;
    if (e >= d.e_hi || d.done[e] || d.idle[e] || !(d.c32 > 0.f)) return;
    const int tid = threadIdx.x, lane = tid & 63;
    const int t = tree_of(d, e);
    const int g = d.gen[t];
    const uint4 rc0 = d.root_c[2 * t];
    if (tid < 64) {
        int nid = rc0.x ? (int)rc0.x - 1 : -1;
        if (nid < 0) {
            const YkS r = ld_state(d.root + e);
            nid = lookup(d, g, t, r, index_hash(r));
        }
        if (tid == 0) {
            s_nid = nid;
            s_nv = 0;
            s_cnt = 0;
        }
    }
    __syncthreads();
    const int nid = s_nid;
    if (nid < 0) return;
    const NodeRec& nd = d.nodes[g][(long)t * d.NCAP + nid];
    const int V = (int)nd.nvalid;
    const uint32_t p_off = nd.p_off;
    // (a root of <= 256 entries is one pass of the full scan, 4 entries per lane: no order pays)
    if (V <= 256 || V > RO_CAP) return;
    const float* P = d.arenaP + (long)t * d.AE + p_off;
    const uint16_t* S = d.arenaS + (long)t * d.AE + p_off;
    uint32_t* rv = d.rv + (long)t * RV_CAP;
    // keys P bits << 16 | (0xFFFF - j): unique, ordered as (P descending, j ascending); 0 = no entry
    uint64_t key[PT];
#pragma unroll
    for (int i = 0; i < PT; i++) {
        const int j = tid + 256 * i;
        key[i] = 0;
        if (j < V) {
            key[i] = ((uint64_t)__float_as_uint(P[j]) << 16) | (uint32_t)(0xFFFFu - (uint32_t)j);
            const uint16_t sl = S[j];
            if (sl) {
                const uint32_t pos = atomicAdd(&s_nv, 1u);
                if (pos < (uint32_t)RV_CAP) rv[pos] = (uint32_t)j | ((uint32_t)sl << 12);
            }
        }
    }
    const int K = V < d.ro_k ? V : d.ro_k;
    uint64_t thr = 1;  // the keys >= thr are the top K
    if (V > K) {  // radix select of the K-th largest key, 8 bits at a time from the top of 48
        uint64_t prefix = 0, mask = 0;
        int need = K;
        for (int sh = 40; sh >= 0; sh -= 8) {
            hist[tid] = 0;
            __syncthreads();
#pragma unroll
            for (int i = 0; i < PT; i++)
                if (key[i] && (key[i] & mask) == prefix) atomicAdd(&hist[(uint32_t)(key[i] >> sh) & 255u], 1u);
            __syncthreads();
            if (tid < 64) {  // the bin holding the need-th largest: suffix sums over lanes of 4 bins each
                const uint32_t h0 = hist[4 * lane], h1 = hist[4 * lane + 1], h2 = hist[4 * lane + 2], h3 = hist[4 * lane + 3];
                const uint32_t own = h0 + h1 + h2 + h3;
                uint32_t suf = own;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t x = __shfl_down(suf, o, 64);
                    if (lane + o < 64) suf += x;
                }
                const uint32_t above = suf - own;
                if (above < (uint32_t)need && (uint32_t)need <= suf) {
                    const uint32_t hb[4] = {h0, h1, h2, h3};
                    uint32_t c = above;
                    int b = 3;
                    for (; b > 0; b--) {
                        if (c + hb[b] >= (uint32_t)need) break;
                        c += hb[b];
                    }
                    s_prefix = prefix | ((uint64_t)(4 * lane + b) << sh);
                    s_need = need - (int)c;
                }
            }
            __syncthreads();
            prefix = s_prefix;
            need = s_need;
            mask |= (uint64_t)255 << sh;
        }
        thr = prefix;
    }
#pragma unroll
    for (int i = 0; i < PT; i++)
        if (key[i] && key[i] >= thr) sk[atomicAdd(&s_cnt, 1u)] = key[i];
    int n2 = 64;
    while (n2 < K) n2 <<= 1;
    __syncthreads();
    for (int i = K + tid; i < n2; i += 256) sk[i] = 0;  // padding sorts last
    __syncthreads();
    for (int size = 2; size <= n2; size <<= 1) {  // bitonic sort, descending
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = tid; i < n2 / 2; i += 256) {
                const int lo = 2 * i - (i & (stride - 1)), hi = lo + stride;
                const bool desc = (lo & size) == 0;
                const uint64_t a = sk[lo], b = sk[hi];
                if ((a < b) == desc) {
                    sk[lo] = b;
                    sk[hi] = a;
                }
            }
            __syncthreads();
        }
    }
    uint16_t* oj = d.ro_j + (long)t * RO_K;
    float* op = d.ro_p + (long)t * RO_K;
    for (int i = tid; i < K; i += 256) {
        const uint64_t k = sk[i];
        oj[i] = (uint16_t)(0xFFFFu - (uint32_t)(k & 0xFFFFu));
        op[i] = __uint_as_float((uint32_t)(k >> 16));
    }
    if (tid == 0) {  // the next descent need not look the root up; .w: the order's stored entries
        d.root_c[2 * t] = make_uint4((uint32_t)nid + 1, p_off, (uint32_t)V, (uint32_t)K);
        d.root_c[2 * t + 1] = make_uint4((uint32_t)nd.vinfo, (uint32_t)(nd.vinfo >> 32),
                                         s_nv <= (uint32_t)RV_CAP ? s_nv : RV_OFF, 0);
    }
}

// getActionProb tail (MCTS.py:40-54) + Coach sampling/step (Coach.py:59-72).  One wave per game.
__global__ __launch_bounds__(256) void k_move_end(EngDev d, int move) {
    __shared__ uint32_t vis_all[GAMES_PER_BLOCK][ASIZE];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int e = d.e_lo + blockIdx.x * GAMES_PER_BLOCK + w;
    if (e >= d.e_hi) return;
    if (d.done[e]) return;
    uint32_t* vis = vis_all[w];
    const int t = tree_of(d, e);  // before the real step changes cur
    const int g = d.gen[t];
    const YkS r = ld_state(d.root + e);
    const bool idle = d.idle[e] != 0;
    const int nid = idle ? -1 : lookup(d, g, t, r, index_hash(r));
    int nvis = 0;
    uint32_t root_ns = 0xFFFFFFFFu;
    if (idle) {
    } else if (nid >= 0) {
        const NodeRec& nd = d.nodes[g][(long)t * d.NCAP + nid];
        root_ns = nd.Ns;
        const VInfo vi = unpack_vinfo(nd.vinfo, nd.nvalid);
        const uint16_t* S = d.arenaS + (long)t * d.AE + nd.p_off;
        const Edge* edges = d.edges[g] + (long)t * d.ECAP;
        // 8 pieces of 64 entries at a time: their slot loads, then their edge loads, all in flight
        // together (one round trip each per 512 entries instead of per 64)
        constexpr int MB = 8;
        const int nv = (int)nd.nvalid;
        for (int j0 = 0; j0 < nv; j0 += 64 * MB) {
            uint16_t sl[MB];
#pragma unroll
            for (int b = 0; b < MB; b++) {
                const int j = j0 + 64 * b + lane;
                const uint16_t x = S[j < nv ? j : 0];  // unconditional loads (in bounds): no wait at a branch join
                sl[b] = j < nv ? x : 0;
            }
            uint32_t n[MB];
#pragma unroll
            for (int b = 0; b < MB; b++) {
                const uint32_t x = edges[sl[b] ? sl[b] - 1 : 0].N;
                n[b] = sl[b] ? x : 0u;
            }
#pragma unroll
            for (int b = 0; b < MB; b++) {
                const int j = j0 + 64 * b + lane;
                const uint64_t bal = __ballot(sl[b] != 0);
                if (sl[b]) {
                    const int pos = nvis + __popcll(bal & ((1ull << lane) - 1));
                    vis[pos] = ((uint32_t)compact_to_action(vi, j) << 16) | (n[b] & 0xFFFF);
                }
                nvis += __popcll(bal);
            }
        }
    } else if (lane == 0) {
        atomicOr(d.err, ERR_ROOT);
    }
    // GreedyYachtPlayer's heuristic needs the whole wave (YachtPlayers.py:186-214)
    int gact = -1;
    if (idle && (d.cur[e] == d.seat[e] ? d.arena_agent : d.arena_opp) == YK_PLAYER_GREEDY)
        gact = greedy_heuristic_wave(r, lane);
    wave_sync();
    // record the visit counts (sparse, ascending action)
    const long vbase = (long)e * d.VCAP;
    const int voff = d.rec_voff[(long)e * (d.M + 1) + move];
    const bool room = voff + nvis <= d.VCAP;
    if (room)
        for (int i = lane; i < nvis; i += 64) d.rec_visits[vbase + voff + i] = vis[i];
    if (lane != 0) return;
    if (!room) atomicOr(d.err, ERR_VISITS);
    d.rec_voff[(long)e * (d.M + 1) + move + 1] = room ? voff + nvis : voff;
    const int stepi = move + 1;
    const int temp = d.arena ? 0 : (stepi < d.temp_threshold ? 1 : 0);  // Coach.py:58
    Stream rs{d.seed, d.env_id[e], d.ctr[e]};
    int action = 0;
    if (idle && gact >= 0) {
        action = gact;  // the greedy heuristic's (valid) choice
    } else if (idle) {
        // RandomYachtPlayer.play, and GreedyYachtPlayer's fallback: np.random.choice over the
        // ascending legal actions of the canonical board (YachtPlayers.py:174-183, 204-214);
        // no legal action -> 0 without a draw
        const VInfo vi = valid_info(r, 1);
        if (vi.V > 0) action = compact_to_action(vi, rs.below(vi.V));
    } else if (temp == 0) {
        // bestAs = argwhere(counts == max(counts)); np.random.choice(bestAs)  (MCTS.py:44-49)
        uint32_t mx = 0;
        for (int i = 0; i < nvis; i++) mx = max(mx, vis[i] & 0xFFFF);
        if (mx == 0) {
            action = rs.below(ASIZE);  // every count is 0: all 3226 actions tie
        } else {
            int nb = 0;
            for (int i = 0; i < nvis; i++) nb += (vis[i] & 0xFFFF) == mx;
            int pick = rs.below(nb);
            for (int i = 0; i < nvis; i++)
                if ((vis[i] & 0xFFFF) == mx && pick-- == 0) {
                    action = (int)(vis[i] >> 16);
                    break;
                }
        }
        // np.random.choice(len(pi), p=one-hot) still draws in Coach (Coach.py:65); the Arena
        // agent is np.argmax(pi) (Coach.py:124-125), which does not
        if (!d.arena) (void)rs.uniform53();
    } else {
        // probs = counts / sum; np.random.choice(len(pi), p=probs): cumsum, /= cdf[-1],
        // searchsorted(u, 'right')
        double total = 0.0;
        for (int i = 0; i < nvis; i++) total += (double)(vis[i] & 0xFFFF);
        if (total == 0.0) {
            atomicOr(d.err, ERR_ZERO_COUNTS);
        } else {
            double c = 0.0;
            for (int i = 0; i < nvis; i++) c += (double)(vis[i] & 0xFFFF) / total;
            const double last = c;
            const double u = rs.uniform53();
            c = 0.0;
            action = ASIZE;
            for (int i = 0; i < nvis; i++) {
                c += (double)(vis[i] & 0xFFFF) / total;
                if (c / last > u) {
                    action = (int)(vis[i] >> 16);
                    break;
                }
            }
        }
    }
    // record + real step (Coach.py:61-67)
    const long ri = (long)e * d.M + move;
    st_state(d.rec_state + ri, r);
    d.rec_ctr[ri * 2 + 1] = rs.ctr;
    const int player = d.cur[e];
    YkS b = ld_state(d.board + e);
    int np = 0;
    const int st = step_state(b, player, action, rs, np);
    int32_t* info = d.rec_info + ri * 8;
    info[0] = temp;
    info[1] = player;
    info[2] = action;
    info[3] = (int32_t)d.gstats[(long)e * GST + 0];
    info[4] = (int32_t)root_ns;
    info[5] = nvis;
    info[6] = st;
    info[7] = 0;
    d.nmoves[e] = stepi;
    if (st != YK_ST_OK) {
        atomicOr(d.err, ERR_STEP);
        d.done[e] = 1;
        return;
    }
    st_state(d.board + e, b);
    d.cur[e] = np;
    d.ctr[e] = rs.ctr;
    const double rgame = game_ended(b, np);  // Coach.py:69
    if (rgame != 0.0) {
        d.done[e] = 1;
        d.final_r[e] = rgame;
        d.final_cur[e] = np;
        d.final_tot[2 * e] = total_with_bonus(b, 0);
        d.final_tot[2 * e + 1] = total_with_bonus(b, 1);
    } else if (stepi >= d.M) {
        atomicOr(d.err, ERR_MOVES);
        d.done[e] = 1;
        d.final_r[e] = 0.0;
        d.final_cur[e] = np;
    }
}

// example values r * (-1)**(player != curPlayer)  (Coach.py:71-72)
__global__ void k_finalize(EngDev d) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long)d.E * d.M) return;
    const int e = (int)(t / d.M), m = (int)(t % d.M);
    if (m >= d.nmoves[e]) {
        d.rec_val[t] = 0.0;
        return;
    }
    const int pl = d.rec_info[t * 8 + 1];
    d.rec_val[t] = d.final_r[e] * ((pl != d.final_cur[e]) ? -1.0 : 1.0);
}

// dense root visit counts for the MCTS plugin (MCTS.py:41-42)
__global__ void k_root_counts(EngDev d, int32_t* counts) {
    const int lane = threadIdx.x & 63;
    const int e = d.e_lo + blockIdx.x * GAMES_PER_BLOCK + (threadIdx.x >> 6);
    if (e >= d.e_hi) return;
    int32_t* c = counts + (long)e * ASIZE;
    for (int a = lane; a < ASIZE; a += 64) c[a] = 0;
    wave_sync();
    const int g = d.gen[e];
    const YkS r = ld_state(d.root + e);
    const int nid = lookup(d, g, e, r, index_hash(r));
    if (nid < 0) return;
    const NodeRec& nd = d.nodes[g][(long)e * d.NCAP + nid];
    const VInfo vi = unpack_vinfo(nd.vinfo, nd.nvalid);
    const uint16_t* S = d.arenaS + (long)e * d.AE + nd.p_off;
    const Edge* edges = d.edges[g] + (long)e * d.ECAP;
    for (int j = lane; j < (int)nd.nvalid; j += 64)
        if (S[j]) c[compact_to_action(vi, j)] = (int32_t)edges[S[j] - 1].N;
}

__global__ void k_count_done(const uint8_t* done, int E, int32_t* out) {
    __shared__ int s;
    if (threadIdx.x == 0) s = 0;
    __syncthreads();
    int c = 0;
    for (int e = threadIdx.x; e < E; e += blockDim.x) c += done[e] ? 1 : 0;
    atomicAdd(&s, c);
    __syncthreads();
    if (threadIdx.x == 0) *out = s;
}

}  // namespace

// ------------------------------------------------------------------ host object
struct yk_engine {
    yk_engine_config_t cfg;
    yk_net_t* net = nullptr;
    yk_net_t* net2 = nullptr;  // the opponent seat's net with dual trees (default: net)
    // dual trees, one game group, row tiles x head parts x 2 <= CUs: the opponent seat's forward
    // runs on its own stream beside the agent's (disjoint rows), with fparts_dual head parts
    hipStream_t dstream = nullptr;
    hipEvent_t ev_d0 = nullptr, ev_d1 = nullptr;
    int fparts_single = 1, fparts_dual = 0;  // fparts_dual 0: the two forwards stay in sequence
    EngDev d{};
    std::vector<void*> allocs;
    float* logits = nullptr;
    float* vpred = nullptr;
    float2* mlse = nullptr;
    float *lut_sq = nullptr, *lut_sqe = nullptr;
    int32_t* done_count = nullptr;
    int32_t* host_done = nullptr;
    uint32_t* mcts_env = nullptr;
    bool have_records = false;
    bool have_arena = false;
    // game groups: the batch is split into `ngroups` ranges, each on its own
    // stream, so one group's forward runs beside another group's expand
    int ngroups = 1;
    hipStream_t gs[YK_MAX_GROUPS] = {};
    hipEvent_t ev_fork = nullptr, ev_join[YK_MAX_GROUPS] = {}, ev_fwd[YK_MAX_GROUPS] = {};
    // profiling (yk_engine_profile): per-kernel-class HIP events on each group's stream; the
    // forward / expand pair is timed in every prof_stride-th simulation (an event record between
    // two dependent launches costs ~4 us of GPU time, so timing every one slows the batch ~5 %)
    bool prof = false;
    int prof_stride = 1;
    struct ProfLog {
        std::vector<hipEvent_t> ev;
        std::vector<int> cls;
        int used = 0;
    } pg[YK_MAX_GROUPS];
    double kms[8] = {0};
    int64_t klaunch[8] = {0};
    bool root_scan = true;  // the incremental root scan (k_root_sort + root_scan); YK_ROOT_SCAN=0: full scans
    bool split_descent = false;  // YK_SPLIT_DESCENT=1: the descent as its own k_select launch (same trees)
};

namespace {
// kernel classes for yk_engine_kernel_times
enum { KC_SELECT = 0, KC_FORWARD = 1, KC_SCAN = 2 /* k_root_sort + the second descent */, KC_EXPAND = 3, KC_MOVE_BEGIN = 4, KC_MOVE_END = 5, KC_N = 8 };

void prof_mark(yk_engine* eng, int g, int cls, hipStream_t s) {  // records an event pair boundary
    if (!eng->prof) return;
    auto& L = eng->pg[g];
    if (L.used + 1 >= (int)L.ev.size()) {
        const size_t old = L.ev.size();
        L.ev.resize(old + 4096);
        L.cls.resize(old + 4096);
        for (size_t i = old; i < L.ev.size(); i++) (void)hipEventCreate(&L.ev[i]);
    }
    L.cls[L.used] = cls;
    (void)hipEventRecord(L.ev[L.used++], s);
}
void prof_collect(yk_engine* eng) {  // call after a stream sync
    if (!eng->prof) return;
    for (int g = 0; g < eng->ngroups; g++) {
        auto& L = eng->pg[g];
        for (int i = 0; i + 1 < L.used; i++) {
            const int cls = L.cls[i];
            if (cls < 0) continue;
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, L.ev[i], L.ev[i + 1]) == hipSuccess) {
                eng->kms[cls] += ms;
                eng->klaunch[cls] += 1;
            }
        }
        L.used = 0;
    }
}

// the device view of group g (its game range)
EngDev group_dev(const yk_engine* eng, int g) {
    EngDev d = eng->d;
    const int G = eng->ngroups;
    auto bound = [&](int k) {
        const long b = (long)d.E * k / G;
        return k == G ? d.E : (int)std::min<long>(d.E, (b + GROUP_ALIGN - 1) / GROUP_ALIGN * GROUP_ALIGN);
    };
    d.e_lo = bound(g);
    d.e_hi = bound(g + 1);
    return d;
}
dim3 game_grid(const EngDev& d) {
    return dim3((unsigned)std::max(1, (d.e_hi - d.e_lo + GAMES_PER_BLOCK - 1) / GAMES_PER_BLOCK));
}

template <class T>
int dalloc(yk_engine* eng, T** p, size_t count) {
    void* q = nullptr;
    if (hipMalloc(&q, sizeof(T) * (count ? count : 1)) != hipSuccess) {
        (void)hipGetLastError();
        return YK_ERR_NOMEM;
    }
    eng->allocs.push_back(q);
    *p = static_cast<T*>(q);
    return YK_OK;
}
int check_errors(yk_engine* eng, hipStream_t s) {
    uint32_t err = 0;
    uint32_t nerr[2] = {0u, 0u};
    YK_HIP(hipMemcpyAsync(&err, eng->d.err, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    if (eng->net) YK_HIP(hipMemcpyAsync(&nerr[0], eng->net->dev.err, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    if (eng->net2) YK_HIP(hipMemcpyAsync(&nerr[1], eng->net2->dev.err, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    YK_HIP(hipStreamSynchronize(s));
    if ((nerr[0] | nerr[1]) && !(err & ERR_FWD_SYNC)) {  // into the engine's word, so yk_engine_stats shows it
        err |= ERR_FWD_SYNC;
        YK_HIP(hipMemcpy(eng->d.err, &err, sizeof(uint32_t), hipMemcpyHostToDevice));
    }
    if (err & (ERR_NODES | ERR_EDGES | ERR_ARENA | ERR_DEPTH | ERR_VISITS | ERR_HASH)) return YK_ERR_CAPACITY;
    if (err) return YK_ERR_STATE;
    return YK_OK;
}
// `sims` simulations for every game of groups 0 .. G-1, group g on stream st[g].  Within a group
// (and a game) the simulations are sequential; the groups' streams run free, so a forward runs
// beside the other groups' expand.  (Staggering them - group g's forward k waiting for group
// g-1's forward k through an event; at 8192 games x 2 groups that costs 1.2 %,
// profiles/r02h_stagger_ab.log.)
int run_sims(yk_engine* eng, int G, const hipStream_t* st, int sims, const uint32_t* env_ids, uint64_t* ctr) {
    const dim3 bb(256);
    if (sims <= 0) return YK_OK;
    EngDev dg[YK_MAX_GROUPS];
    for (int g = 0; g < G; g++) {
        dg[g] = G == 1 ? eng->d : group_dev(eng, g);
        prof_mark(eng, g, KC_SELECT, st[g]);  // the first descent; later ones run in k_expand_backup's tail
        hipLaunchKernelGGL(k_select, game_grid(dg[g]), bb, 0, st[g], dg[g], env_ids, ctr);
        YK_LAUNCHED();
    }
    for (int k = 0; k < sims; k++) {
        const bool timed = k % eng->prof_stride == 0;  // sim 0 always: it closes the select interval
        for (int g = 0; g < G; g++) {
            const EngDev& d = dg[g];
            if (d.prior == 0) {
                if (timed) prof_mark(eng, g, KC_FORWARD, st[g]);
                // predict row = game: no compaction; workgroups without a leaf exit at once
                // (dual trees: the agent's leaves on its net, then the opponent's on its own)
                const int lo = d.e_lo;
                const bool conc = d.dual && eng->dstream && G == 1;
                if (conc) {  // the opponent's forward waits for this stream's last expand only
                    YK_HIP(hipEventRecord(eng->ev_d0, st[g]));
                    YK_HIP(hipStreamWaitEvent(eng->dstream, eng->ev_d0, 0));
                }
                for (int side = 0; side < (d.dual ? 2 : 1); side++) {
                    const yk_net_t* net = side ? eng->net2 : eng->net;
                    hipStream_t fs = conc && side == 1 ? eng->dstream : st[g];
                    int rc = launch_forward(net->dev, d.leaf_state + lo, nullptr, nullptr, nullptr, d.e_hi - lo,
                                            eng->logits + (size_t)lo * PI_LD, eng->vpred + lo, fs,
                                            d.leaf_flag + lo, eng->mlse + lo, true, d.dual ? (uint8_t)(1u << side) : 0xFF,
                                            d.fparts, d.E);
                    if (rc) return rc;
                }
                if (conc) {
                    YK_HIP(hipEventRecord(eng->ev_d1, eng->dstream));
                    YK_HIP(hipStreamWaitEvent(st[g], eng->ev_d1, 0));
                }
            }
            if (timed) prof_mark(eng, g, KC_EXPAND, st[g]);
            // the move's first expansion ends without the next descent: the root's P order is built
            // in between (k_root_sort; root_scan uses it for the move's remaining simulations)
            const bool sort_root = k == 0 && sims > 1 && eng->root_scan;
            const bool fuse = k + 1 < sims && !sort_root;  // the next descent in the expand's tail
            hipLaunchKernelGGL(k_expand_backup, game_grid(d), bb, 0, st[g], d, fuse && !eng->split_descent ? 1 : 0,
                               env_ids, ctr);
            YK_LAUNCHED();
            if (fuse && eng->split_descent) {
                hipLaunchKernelGGL(k_select, game_grid(d), bb, 0, st[g], d, env_ids, ctr);
                YK_LAUNCHED();
            }
            if (sort_root) {
                if (timed) prof_mark(eng, g, KC_SCAN, st[g]);
                hipLaunchKernelGGL(k_root_sort, dim3((unsigned)(d.e_hi - d.e_lo)), bb, 0, st[g], d);
                YK_LAUNCHED();
                hipLaunchKernelGGL(k_select, game_grid(d), bb, 0, st[g], d, env_ids, ctr);
                YK_LAUNCHED();
            }
            if (timed && eng->prof_stride > 1) prof_mark(eng, g, -1, st[g]);  // untimed sims follow
        }
    }
    for (int g = 0; g < G; g++) prof_mark(eng, g, -1, st[g]);
    return YK_OK;
}
}  // namespace

extern "C" {


int yk_engine_create(yk_engine_t** out, const yk_engine_config_t* cfg, yk_net_t* net) {
    if (!out || !cfg) return YK_ERR_ARG;
    if (cfg->n_envs <= 0 || cfg->sims < 1 || cfg->max_moves < 1 || cfg->max_moves > 4096) return YK_ERR_ARG;
    if (cfg->prior == 0 && !net) return YK_ERR_ARG;
    if (cfg->prior != 0 && cfg->prior != 1) return YK_ERR_ARG;
    yk_engine* eng = new yk_engine();
    eng->cfg = *cfg;
    eng->net = net;
    EngDev& d = eng->d;
    d.E = cfg->n_envs;
    d.sims = cfg->sims;
    d.c32 = (float)cfg->cpuct;
    d.temp_threshold = cfg->temp_threshold;
    d.prior = cfg->prior;
    d.M = cfg->max_moves;
    // capacities: one new node per simulation; a round holds <= 4 real moves
    // and round 2 also keeps the round-2 nodes made while searching round 1 (<= 2 moves).
    d.NCAP = 6 * cfg->sims + 64;
    int hcap = 1;
    while (hcap < 2 * d.NCAP) hcap <<= 1;
    d.HCAP = hcap;
    d.ECAP = std::min(4 * d.NCAP, 65535);
    // Arena: the worst case (every live node a 3024-action score node) cannot overflow; use it
    // when it fits in 60% of free HBM, else a measured-footprint default (overflow is detected).
    if (cfg->arena_entries > 0) {
        d.AE = (cfg->arena_entries + 3) & ~3LL;
    } else {
        const int64_t worst = (int64_t)d.NCAP * 3024;
        size_t free_b = 0, total_b = 0;
        (void)hipMemGetInfo(&free_b, &total_b);
        const double need = (double)worst * 6.0 * cfg->n_envs * (cfg->dual_trees ? 2 : 1);
        d.AE = (need < 0.6 * (double)free_b) ? worst : (int64_t)cfg->sims * 9000 + 65536;
    }
    d.VCAP = (int)record_vcap(cfg->max_moves, cfg->sims);
    d.rec_pred = cfg->record_predictions ? 1 : 0;
    d.max_exp = cfg->record_predictions ? std::max(cfg->max_expansions, 1) : 0;
    d.rec_stride = std::max(cfg->record_stride, 1);
    d.e_lo = 0;
    d.e_hi = d.E;
    d.T = cfg->dual_trees ? 2 * d.E : d.E;
    d.dual = 0;  // set by yk_arena for MCTS vs MCTS
    eng->net2 = net;
    // game groups: auto = 2 with the net prior at >= 8192 games (the forward of 4096 rows fills the
    // chip in one round, so there a second group's forward beside the first's expand pays: +3.8 %
    // measured), else 1 (below that each simulation is latency-bound: F + X per group does not
    // shrink with the group); each group needs at least one forward row tile
    int G = cfg->groups > 0 ? cfg->groups : ((cfg->prior == 0 && cfg->n_envs >= 8192) ? 2 : 1);
    G = std::max(1, std::min({G, YK_MAX_GROUPS, (cfg->n_envs + GROUP_ALIGN - 1) / GROUP_ALIGN}));
    eng->ngroups = G;
    // forward head split: when a group's row tiles do not fill the CUs, 2 or 4
    // workgroups per tile each take a slice of the policy head (the trunk runs in each)
constexpr int YK_FPARTS_MAX = 4;
    {
        int cus = 256, dev = 0;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        // the G groups' forwards run at once on their own streams: the bound counts every group's
        // tiles (sizing from one group's tiles oversubscribed the chip at G = 4)
        const int tiles = G * (((cfg->n_envs + G - 1) / G + 15) / 16);
        d.fparts = 1;
        while (d.fparts * 2 <= YK_FPARTS_MAX && tiles * d.fparts * 2 <= cus) d.fparts *= 2;
        eng->fparts_single = d.fparts;
        if (cfg->dual_trees && G == 1 && cfg->prior == 0 && 2 * tiles <= cus) {
            eng->fparts_dual = 1;
            while (eng->fparts_dual * 2 <= YK_FPARTS_MAX && 2 * tiles * eng->fparts_dual * 2 <= cus) eng->fparts_dual *= 2;
        }
    }
    const size_t R = ((size_t)cfg->n_envs + d.rec_stride - 1) / d.rec_stride;
    const size_t E = (size_t)d.E, T = (size_t)d.T;
    int rc = YK_OK;
#define A(p, n) \
    if (rc == YK_OK) rc = dalloc(eng, &(p), (n))
    for (int g = 0; g < 2; g++) {
        A(d.nodes[g], T * d.NCAP);
        A(d.hidx[g], T * d.HCAP);
        A(d.edges[g], T * d.ECAP);
    }
    A(d.node_count, 2 * T);
    A(d.edge_count, 2 * T);
    A(d.arenaP, T * (size_t)d.AE);
    A(d.arenaS, T * (size_t)d.AE);
    A(d.arena_top, T);
    A(d.gen, T);
    A(d.cur_round, T);
    A(d.root_c, 2 * T);
    A(d.rv, T * RV_CAP);
    A(d.ro_j, T * RO_K);
    A(d.ro_p, T * RO_K);
    A(d.board, E);
    A(d.cur, E);
    A(d.ctr, E);
    A(d.env_id, E);
    A(d.done, E);
    A(d.nmoves, E);
    A(d.root, E);
    A(d.leaf_state, E);
    A(d.leaf_hash, E);
    A(d.leaf_flag, E);
    A(d.path, E * MAXD);
    A(d.path_len, E);
    A(d.end_node, E);
    A(d.res_v, E);
    A(d.res_t, E);
    A(eng->vpred, E);
    A(eng->mlse, E * (size_t)d.fparts);
    A(eng->lut_sq, (size_t)LUT_N);
    A(eng->lut_sqe, (size_t)LUT_N);
    A(d.rec_state, E * d.M);
    A(d.rec_info, E * d.M * 8);
    A(d.rec_ctr, E * d.M * 2);
    A(d.rec_val, E * d.M);
    A(d.rec_visits, E * (size_t)d.VCAP);
    A(d.rec_voff, E * (d.M + 1));
    A(d.final_r, E);
    A(d.final_cur, E);
    A(d.final_tot, 2 * E);
    A(d.seat, E);
    A(d.idle, E);
    A(d.gstats, E * GST);
    A(d.err, 1);
    A(eng->done_count, 1);
    A(eng->mcts_env, E);
    if (d.prior == 0) {
        A(eng->logits, E * (size_t)PI_LD);
    }
    if (d.rec_pred) {
        A(d.rec_pi, R * (size_t)d.max_exp * ASIZE);
        A(d.rec_v, R * (size_t)d.max_exp);
        A(d.rec_leaf, R * (size_t)d.max_exp);
    }
#undef A
    if (rc == YK_OK && hipHostMalloc((void**)&eng->host_done, sizeof(int32_t)) != hipSuccess) rc = YK_ERR_NOMEM;
    {  // YK_ROOT_SCAN=0: every descent scans the root's whole compact set (A/B, and the test that both
       // give the same trees)
        const char* ev = getenv("YK_ROOT_SCAN");
        eng->root_scan = !(ev && ev[0] == '0');
        const char* ek = getenv("YK_ROOT_K");  // a shorter kept order (>= 1): the tests' fallback cases
        d.ro_k = ek ? std::max(1, std::min(RO_K, atoi(ek))) : RO_K;
        // YK_SPLIT_DESCENT=1 (measurement): k_expand_backup stops after the backup and each next
        // descent is its own k_select launch, so rocprofv3 times and counts the expansion + backup
        // and the descent apart (the same work: the trees are identical)
        const char* es = getenv("YK_SPLIT_DESCENT");
        eng->split_descent = es && es[0] == '1';
    }
    if (rc == YK_OK && G > 1) {
        if (hipEventCreateWithFlags(&eng->ev_fork, hipEventDisableTiming) != hipSuccess) rc = YK_ERR_HIP;
        for (int g = 0; g < G && rc == YK_OK; g++)
            if (hipStreamCreateWithFlags(&eng->gs[g], hipStreamNonBlocking) != hipSuccess ||
                hipEventCreateWithFlags(&eng->ev_join[g], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&eng->ev_fwd[g], hipEventDisableTiming) != hipSuccess)
                rc = YK_ERR_HIP;
    }
    if (rc == YK_OK && eng->fparts_dual > 0) {
        if (hipStreamCreateWithFlags(&eng->dstream, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&eng->ev_d0, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&eng->ev_d1, hipEventDisableTiming) != hipSuccess)
            rc = YK_ERR_HIP;
    }
    if (rc != YK_OK) {
        yk_engine_destroy(eng);
        return rc;
    }
    d.logits = eng->logits;
    d.vpred = eng->vpred;
    d.mlse = eng->mlse;
    d.lut_sq = eng->lut_sq;
    d.lut_sqe = eng->lut_sqe;
    hipLaunchKernelGGL(k_lut, dim3(LUT_N / 256), dim3(256), 0, 0, eng->lut_sq, eng->lut_sqe);
    YK_LAUNCHED();
    YK_HIP(hipMemset(d.err, 0, sizeof(uint32_t)));
    YK_HIP(hipMemset(d.done, 0, E));
    YK_HIP(hipMemset(d.idle, 0, E));
    YK_HIP(hipMemset(d.leaf_state, 0, sizeof(yk_state_t) * E));
    std::vector<uint32_t> ids(E);
    for (size_t i = 0; i < E; i++) ids[i] = (uint32_t)i;
    YK_HIP(hipMemcpy(eng->mcts_env, ids.data(), sizeof(uint32_t) * E, hipMemcpyHostToDevice));
    YK_HIP(hipDeviceSynchronize());
    *out = eng;
    return YK_OK;
}

int yk_engine_destroy(yk_engine_t* eng) {
    if (!eng) return YK_OK;
    for (auto& L : eng->pg)
        for (hipEvent_t e : L.ev) (void)hipEventDestroy(e);
    for (int g = 0; g < YK_MAX_GROUPS; g++) {
        if (eng->gs[g]) (void)hipStreamDestroy(eng->gs[g]);
        if (eng->ev_join[g]) (void)hipEventDestroy(eng->ev_join[g]);
        if (eng->ev_fwd[g]) (void)hipEventDestroy(eng->ev_fwd[g]);
    }
    if (eng->ev_fork) (void)hipEventDestroy(eng->ev_fork);
    if (eng->dstream) (void)hipStreamDestroy(eng->dstream);
    if (eng->ev_d0) (void)hipEventDestroy(eng->ev_d0);
    if (eng->ev_d1) (void)hipEventDestroy(eng->ev_d1);
    for (void* p : eng->allocs) (void)hipFree(p);
    if (eng->host_done) (void)hipHostFree(eng->host_done);
    delete eng;
    return YK_OK;
}

}  // extern "C"

namespace {
// One lock-step batch of complete games: self-play (Coach.executeEpisode) or, with
// d.arena set, Arena.playGame against the uniform-random player.
int play_batch(yk_engine* eng, uint64_t seed, uint32_t env_base, hipStream_t s) {
    EngDev& d = eng->d;
    d.seed = seed;
    const int G = eng->ngroups;
    hipStream_t st[YK_MAX_GROUPS];
    EngDev dg[YK_MAX_GROUPS];
    for (int g = 0; g < G; g++) {
        st[g] = G == 1 ? s : eng->gs[g];
        dg[g] = G == 1 ? d : group_dev(eng, g);
    }
    const dim3 bb(256);
    YK_HIP(hipMemsetAsync(d.err, 0, sizeof(uint32_t), s));
    YK_HIP(hipMemsetAsync(d.hidx[0], 0, sizeof(uint32_t) * (size_t)d.T * d.HCAP, s));
    hipLaunchKernelGGL(k_reset, dim3((d.E + 255) / 256), dim3(256), 0, s, d, 1, env_base);
    YK_LAUNCHED();
    if (G > 1) {  // the group streams start after the reset on the caller's stream
        YK_HIP(hipEventRecord(eng->ev_fork, s));
        for (int g = 0; g < G; g++) YK_HIP(hipStreamWaitEvent(st[g], eng->ev_fork, 0));
    }
    eng->have_records = false;
    for (int move = 0; move < d.M; move++) {
        for (int g = 0; g < G; g++) {
            prof_mark(eng, g, KC_MOVE_BEGIN, st[g]);
            hipLaunchKernelGGL(k_move_begin, game_grid(dg[g]), bb, 0, st[g], dg[g], move, 0);
            YK_LAUNCHED();
        }
        if (!d.arena || d.arena_agent == YK_PLAYER_MCTS || d.arena_opp == YK_PLAYER_MCTS) {
            int rc = run_sims(eng, G, st, d.sims, d.env_id, d.ctr);
            if (rc) return rc;
        }
        for (int g = 0; g < G; g++) {
            prof_mark(eng, g, KC_MOVE_END, st[g]);
            hipLaunchKernelGGL(k_move_end, game_grid(dg[g]), bb, 0, st[g], dg[g], move);
            YK_LAUNCHED();
            prof_mark(eng, g, -1, st[g]);
            if (G > 1) {
                YK_HIP(hipEventRecord(eng->ev_join[g], st[g]));
                YK_HIP(hipStreamWaitEvent(s, eng->ev_join[g], 0));
            }
        }
        hipLaunchKernelGGL(k_count_done, dim3(1), dim3(1024), 0, s, d.done, d.E, eng->done_count);
        YK_LAUNCHED();
        YK_HIP(hipMemcpyAsync(eng->host_done, eng->done_count, sizeof(int32_t), hipMemcpyDeviceToHost, s));
        YK_HIP(hipStreamSynchronize(s));
        prof_collect(eng);
        if (*eng->host_done >= d.E) break;
    }
    hipLaunchKernelGGL(k_finalize, dim3((unsigned)(((long)d.E * d.M + 255) / 256)), dim3(256), 0, s, d);
    YK_LAUNCHED();
    eng->have_records = true;
    return check_errors(eng, s);
}
}  // namespace

extern "C" {

int yk_selfplay(yk_engine_t* eng, uint64_t seed, uint32_t env_base, void* stream) {
    if (!eng) return YK_ERR_ARG;
    eng->d.arena = 0;
    eng->have_arena = false;
    return play_batch(eng, seed, env_base, as_stream(stream));
}

int yk_arena(yk_engine_t* eng, uint64_t seed, uint32_t env_base, const int32_t* agent_seat, int agent, int opponent,
             void* stream) {
    if (!eng || !agent_seat) return YK_ERR_ARG;
    if (agent < YK_PLAYER_MCTS || agent > YK_PLAYER_GREEDY || opponent < YK_PLAYER_MCTS || opponent > YK_PLAYER_GREEDY)
        return YK_ERR_ARG;
    EngDev& d = eng->d;
    for (int e = 0; e < d.E; e++)
        if (agent_seat[e] != 1 && agent_seat[e] != -1) return YK_ERR_ARG;
    hipStream_t s = as_stream(stream);
    YK_HIP(hipMemcpyAsync(d.seat, agent_seat, sizeof(int32_t) * (size_t)d.E, hipMemcpyHostToDevice, s));
    d.arena = 1;
    d.arena_agent = agent;
    d.arena_opp = opponent;
    // two MCTS players each keep their own tree (and net) when the engine has dual trees
    d.dual = (d.T == 2 * d.E && agent == YK_PLAYER_MCTS && opponent == YK_PLAYER_MCTS) ? 1 : 0;
    if (d.dual && eng->dstream) d.fparts = eng->fparts_dual;  // the two seats' forwards side by side
    eng->have_arena = false;
    const int rc = play_batch(eng, seed, env_base, s);
    d.arena = 0;
    d.dual = 0;
    d.fparts = eng->fparts_single;
    eng->have_arena = rc == YK_OK || rc == YK_ERR_STATE;
    return rc;
}

int yk_engine_set_opponent_net(yk_engine_t* eng, yk_net_t* net) {
    if (!eng || !net) return YK_ERR_ARG;
    if (eng->d.T != 2 * eng->d.E || eng->d.prior != 0) return YK_ERR_ARG;  // needs dual trees and the net prior
    if (net->dev.H != eng->net->dev.H) return YK_ERR_ARG;
    eng->net2 = net;
    return YK_OK;
}

int yk_arena_results(yk_engine_t* eng, double* result, int32_t* totals, int32_t* n_moves, int32_t* actions,
                     uint64_t* final_states, uint64_t* rng_ctr) {
    if (!eng) return YK_ERR_ARG;
    if (!eng->have_arena) return YK_ERR_STATE;
    EngDev& d = eng->d;
    const size_t E = d.E, M = d.M;
    YK_HIP(hipDeviceSynchronize());
    std::vector<int32_t> nm(E), fc(E), info;
    std::vector<double> fr(E);
    YK_HIP(hipMemcpy(nm.data(), d.nmoves, sizeof(int32_t) * E, hipMemcpyDeviceToHost));
    if (result) {
        YK_HIP(hipMemcpy(fr.data(), d.final_r, sizeof(double) * E, hipMemcpyDeviceToHost));
        YK_HIP(hipMemcpy(fc.data(), d.final_cur, sizeof(int32_t) * E, hipMemcpyDeviceToHost));
        for (size_t e = 0; e < E; e++) result[e] = (double)fc[e] * fr[e];  // Arena.py:93
    }
    if (totals) YK_HIP(hipMemcpy(totals, d.final_tot, sizeof(int32_t) * 2 * E, hipMemcpyDeviceToHost));
    if (n_moves) std::copy(nm.begin(), nm.end(), n_moves);
    if (actions) {
        info.resize(E * M * 8);
        YK_HIP(hipMemcpy(info.data(), d.rec_info, sizeof(int32_t) * info.size(), hipMemcpyDeviceToHost));
        for (size_t e = 0; e < E; e++)
            for (size_t m = 0; m < M; m++) actions[e * M + m] = (int)m < nm[e] ? info[(e * M + m) * 8 + 2] : -1;
    }
    if (final_states) YK_HIP(hipMemcpy(final_states, d.board, sizeof(yk_state_t) * E, hipMemcpyDeviceToHost));
    if (rng_ctr) YK_HIP(hipMemcpy(rng_ctr, d.ctr, sizeof(uint64_t) * E, hipMemcpyDeviceToHost));
    return YK_OK;
}

int yk_engine_profile(yk_engine_t* eng, int enable) {
    if (!eng) return YK_ERR_ARG;
    if (enable < 0) return YK_ERR_ARG;
    eng->prof = enable != 0;
    eng->prof_stride = enable > 0 ? enable : 1;
    for (auto& L : eng->pg) L.used = 0;
    for (int i = 0; i < 8; i++) {
        eng->kms[i] = 0;
        eng->klaunch[i] = 0;
    }
    return YK_OK;
}

int yk_engine_kernel_times(yk_engine_t* eng, double* ms, int64_t* launches) {
    if (!eng || !ms || !launches) return YK_ERR_ARG;
    for (int i = 0; i < 8; i++) {
        ms[i] = eng->kms[i];
        launches[i] = eng->klaunch[i];
    }
    return YK_OK;
}

int yk_engine_stats(yk_engine_t* eng, int64_t* out) {
    if (!eng || !out) return YK_ERR_ARG;
    EngDev& d = eng->d;
    std::vector<uint64_t> gs((size_t)d.E * GST);
    std::vector<int32_t> nm(d.E);
    uint32_t err = 0;
    YK_HIP(hipDeviceSynchronize());
    YK_HIP(hipMemcpy(gs.data(), d.gstats, sizeof(uint64_t) * gs.size(), hipMemcpyDeviceToHost));
    YK_HIP(hipMemcpy(nm.data(), d.nmoves, sizeof(int32_t) * nm.size(), hipMemcpyDeviceToHost));
    YK_HIP(hipMemcpy(&err, d.err, sizeof(uint32_t), hipMemcpyDeviceToHost));
    for (int i = 0; i < 16; i++) out[i] = 0;
    for (int e = 0; e < d.E; e++) {
        const uint64_t* g = &gs[(size_t)e * GST];
        out[0] += (int64_t)g[0];
        out[1] += (int64_t)g[1];
        out[2] = std::max<int64_t>(out[2], nm[e]);
        out[4] = std::max<int64_t>(out[4], (int64_t)g[4]);
        out[5] = std::max<int64_t>(out[5], (int64_t)g[5]);
        out[6] = std::max<int64_t>(out[6], (int64_t)g[6]);
        out[7] += (int64_t)g[3];
        out[8] += (int64_t)g[2];
        out[9] = std::max<int64_t>(out[9], (int64_t)g[7]);
    }
    out[3] = err;
    out[10] = d.NCAP;
    out[11] = d.ECAP;
    out[12] = d.AE;
    out[13] = d.VCAP;
    out[14] = eng->ngroups;
    out[15] = d.fparts;
    return YK_OK;
}

int yk_engine_counters(yk_engine_t* eng, int64_t* out, int n) {
    if (!eng || !out || n < 0) return YK_ERR_ARG;
    EngDev& d = eng->d;
    std::vector<uint64_t> gs((size_t)d.E * GST);
    YK_HIP(hipDeviceSynchronize());
    YK_HIP(hipMemcpy(gs.data(), d.gstats, sizeof(uint64_t) * gs.size(), hipMemcpyDeviceToHost));
    int64_t c[1] = {0};
    for (int e = 0; e < d.E; e++) c[0] += (int64_t)gs[(size_t)e * GST + 8];
    for (int i = 0; i < n; i++) out[i] = i < 1 ? c[i] : 0;
    return YK_OK;
}

int yk_engine_records(yk_engine_t* eng, uint64_t* states, int32_t* info, uint64_t* ctr, double* values,
                      uint64_t* final_states, int32_t* n_moves, int64_t* visits_off, int32_t* visits,
                      int64_t* n_visits) {
    if (!eng) return YK_ERR_ARG;
    if (!eng->have_records) return YK_ERR_STATE;
    EngDev& d = eng->d;
    const size_t E = d.E, M = d.M;
    YK_HIP(hipDeviceSynchronize());
    if (states) YK_HIP(hipMemcpy(states, d.rec_state, sizeof(yk_state_t) * E * M, hipMemcpyDeviceToHost));
    if (info) YK_HIP(hipMemcpy(info, d.rec_info, sizeof(int32_t) * E * M * 8, hipMemcpyDeviceToHost));
    if (ctr) YK_HIP(hipMemcpy(ctr, d.rec_ctr, sizeof(uint64_t) * E * M * 2, hipMemcpyDeviceToHost));
    if (values) YK_HIP(hipMemcpy(values, d.rec_val, sizeof(double) * E * M, hipMemcpyDeviceToHost));
    if (final_states) YK_HIP(hipMemcpy(final_states, d.board, sizeof(yk_state_t) * E, hipMemcpyDeviceToHost));
    if (n_moves) YK_HIP(hipMemcpy(n_moves, d.nmoves, sizeof(int32_t) * E, hipMemcpyDeviceToHost));
    if (visits_off || visits || n_visits) {
        std::vector<int32_t> voff(E * (M + 1));
        std::vector<int32_t> nm(E);
        YK_HIP(hipMemcpy(voff.data(), d.rec_voff, sizeof(int32_t) * voff.size(), hipMemcpyDeviceToHost));
        YK_HIP(hipMemcpy(nm.data(), d.nmoves, sizeof(int32_t) * E, hipMemcpyDeviceToHost));
        int64_t total = 0;
        for (size_t e = 0; e < E; e++) total += voff[e * (M + 1) + nm[e]];
        if (n_visits) *n_visits = total;
        if (visits_off || visits) {
            std::vector<uint32_t> raw(E * (size_t)d.VCAP);
            YK_HIP(hipMemcpy(raw.data(), d.rec_visits, sizeof(uint32_t) * raw.size(), hipMemcpyDeviceToHost));
            int64_t k = 0;
            for (size_t e = 0; e < E; e++) {
                for (size_t m = 0; m < M; m++) {
                    const int32_t a0 = voff[e * (M + 1) + m];
                    const int32_t a1 = (int)m < nm[e] ? voff[e * (M + 1) + m + 1] : a0;
                    if (visits_off) visits_off[e * M + m] = k;
                    for (int32_t i = a0; i < a1; i++, k++)
                        if (visits) {
                            const uint32_t x = raw[e * d.VCAP + i];
                            visits[2 * k] = (int32_t)(x >> 16);
                            visits[2 * k + 1] = (int32_t)(x & 0xFFFF);
                        }
                }
            }
            if (visits_off) visits_off[E * M] = k;
        }
    }
    return YK_OK;
}

int yk_engine_predictions(yk_engine_t* eng, float* pi, float* v, yk_state_t* leaves, int32_t* count) {
    if (!eng || !eng->d.rec_pred) return YK_ERR_ARG;
    EngDev& d = eng->d;
    const size_t R = ((size_t)d.E + d.rec_stride - 1) / d.rec_stride, X = (size_t)d.max_exp;
    YK_HIP(hipDeviceSynchronize());
    if (pi) YK_HIP(hipMemcpy(pi, d.rec_pi, sizeof(float) * R * X * ASIZE, hipMemcpyDeviceToHost));
    if (v) YK_HIP(hipMemcpy(v, d.rec_v, sizeof(float) * R * X, hipMemcpyDeviceToHost));
    if (leaves) YK_HIP(hipMemcpy(leaves, d.rec_leaf, sizeof(yk_state_t) * R * X, hipMemcpyDeviceToHost));
    if (count) {
        std::vector<uint64_t> gs((size_t)d.E * GST);
        YK_HIP(hipMemcpy(gs.data(), d.gstats, sizeof(uint64_t) * gs.size(), hipMemcpyDeviceToHost));
        for (size_t r = 0; r < R; r++) count[r] = (int32_t)gs[r * d.rec_stride * GST];  // > max_expansions: truncated
    }
    return YK_OK;
}

static void record_parts(yk_engine* eng, void** p, RecordLayout& L) {
    EngDev& d = eng->d;
    L = record_layout(d.E, d.M, d.VCAP);
    void* pp[REC_PARTS] = {d.rec_state, d.rec_info, d.rec_ctr, d.rec_val, d.rec_visits, d.rec_voff, d.nmoves, d.board};
    for (int i = 0; i < REC_PARTS; i++) p[i] = pp[i];
}

int64_t yk_engine_record_bytes(yk_engine_t* eng) {
    if (!eng) return YK_ERR_ARG;
    return record_layout(eng->d.E, eng->d.M, eng->d.VCAP).total;
}

int yk_engine_pack_records(yk_engine_t* eng, void* dst, int64_t capacity, void* stream) {
    if (!eng || !dst) return YK_ERR_ARG;
    if (!eng->have_records) return YK_ERR_STATE;
    void* p[REC_PARTS];
    RecordLayout L;
    record_parts(eng, p, L);
    if (capacity < L.total) return YK_ERR_ARG;
    for (int i = 0; i < REC_PARTS; i++)
        YK_HIP(hipMemcpyAsync((char*)dst + L.off[i], p[i], (size_t)L.bytes[i], hipMemcpyDeviceToDevice,
                              as_stream(stream)));
    return YK_OK;
}

int yk_mcts_reset(yk_engine_t* eng) {
    if (!eng) return YK_ERR_ARG;
    EngDev& d = eng->d;
    YK_HIP(hipMemset(d.err, 0, sizeof(uint32_t)));
    YK_HIP(hipMemset(d.hidx[0], 0, sizeof(uint32_t) * (size_t)d.T * d.HCAP));
    YK_HIP(hipMemset(d.done, 0, (size_t)d.E));
    hipLaunchKernelGGL(k_reset, dim3((d.E + 255) / 256), dim3(256), 0, 0, d, 0, 0u);
    YK_LAUNCHED();
    YK_HIP(hipDeviceSynchronize());
    return YK_OK;
}

int yk_mcts_search(yk_engine_t* eng, const yk_state_t* roots, uint64_t seed, const uint32_t* env_ids,
                   uint64_t* rng_ctr, int sims, int32_t* counts, void* stream) {
    if (!eng || !roots || !env_ids || !rng_ctr || !counts || sims < 0) return YK_ERR_ARG;
    hipStream_t s = as_stream(stream);
    EngDev& d = eng->d;
    d.seed = seed;
    const dim3 gb = game_grid(d), bb(256);
    YK_HIP(hipMemcpyAsync(d.root, roots, sizeof(yk_state_t) * (size_t)d.E, hipMemcpyDeviceToDevice, s));
    YK_HIP(hipMemsetAsync(d.done, 0, (size_t)d.E, s));
    YK_HIP(hipMemsetAsync(d.err, 0, sizeof(uint32_t), s));
    hipLaunchKernelGGL(k_move_begin, gb, bb, 0, s, d, 0, 1);
    YK_LAUNCHED();
    int rc = run_sims(eng, 1, &s, sims, env_ids, rng_ctr);  // the plugin path: one group on the caller's stream
    if (rc) return rc;
    hipLaunchKernelGGL(k_root_counts, gb, bb, 0, s, d, counts);
    YK_LAUNCHED();
    return check_errors(eng, s);
}

}  // extern "C"
