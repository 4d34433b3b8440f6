/*
 * yk_oracle.c - CPU restatement of the reference self-play hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed CPU
 * baseline.  The product (nypc-yacht-auction_amd/) never links or calls it.
 *
 * Parity: pinned against golden vectors produced by running the reference itself
 * (tests/golden/make_golden.py, tests/test_oracle_golden.py).
 *
 * Every function cites the reference file:line it restates (paths relative to
 * /root/reference).  Data contracts (packed state, Philox stream, hash prior) are
 * stated in oracle/spec.py.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define NCAT 12
#define BID_LEVELS 101
#define NBID 202
#define NCOMB 252
#define ASIZE 3226
#define FEAT 59

/* ------------------------------------------------------------------ combos */
/* COMB_5_OF_10 = list(itertools.combinations(range(10), 5))  YachtGame.py:35 */
static uint8_t COMB[NCOMB][5];
static int comb_ready = 0;
static void init_comb(void) {
    if (comb_ready) return;
    int k = 0;
    for (int a = 0; a < 10; a++)
        for (int b = a + 1; b < 10; b++)
            for (int c = b + 1; c < 10; c++)
                for (int d = c + 1; d < 10; d++)
                    for (int e = d + 1; e < 10; e++) {
                        COMB[k][0] = a; COMB[k][1] = b; COMB[k][2] = c; COMB[k][3] = d; COMB[k][4] = e;
                        k++;
                    }
    comb_ready = 1;
}

/* ------------------------------------------------------------------ RNG contract */
static inline void mulhilo(uint32_t a, uint32_t b, uint32_t* hi, uint32_t* lo) {
    uint64_t p = (uint64_t)a * b;
    *hi = (uint32_t)(p >> 32);
    *lo = (uint32_t)p;
}
uint64_t or_draw64(uint64_t seed, uint32_t env, uint64_t ctr) {
    uint32_t c0 = (uint32_t)ctr, c1 = (uint32_t)(ctr >> 32), c2 = env, c3 = 0;
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    for (int r = 0; r < 10; r++) {
        uint32_t hi0, lo0, hi1, lo1;
        mulhilo(0xD2511F53u, c0, &hi0, &lo0);
        mulhilo(0xCD9E8D57u, c2, &hi1, &lo1);
        uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return (uint64_t)c0 | ((uint64_t)c1 << 32);
}
typedef struct { uint64_t seed; uint32_t env; uint64_t ctr; } stream_t;
static inline uint64_t st_next(stream_t* s) { return or_draw64(s->seed, s->env, s->ctr++); }
static inline int st_below(stream_t* s, int n) { return (int)(((st_next(s) >> 32) * (uint64_t)n) >> 32); }
static inline int st_die(stream_t* s) { return 1 + st_below(s, 6); }
static inline double st_uniform53(stream_t* s) { return (double)(st_next(s) >> 11) * (1.0 / 9007199254740992.0); }

/* ------------------------------------------------------------------ state */
/* YachtState / PlayerState  YachtGame.py:115-147 */
typedef struct {
    int n;            /* len(carry) */
    int d[10];        /* carry, in order (combo indices are positional, Q10) */
    int used;         /* 12-bit used_mask */
    int cat[NCAT];    /* cat_scores (points) */
    int32_t bid;      /* bid_score */
} pl_t;
typedef struct {
    int round, phase;
    int hasA, hasB;
    int A[5], B[5];
    int bset[2], bt[2], ba[2]; /* p1_bid/p2_bid: set?, target (0=A,1=B), amount */
    pl_t p[2];
} st_t;

static void unpack(const uint64_t* w, st_t* s) {
    memset(s, 0, sizeof(*s));
    uint64_t w0 = w[0];
    s->round = (int)(w0 & 0xF);
    s->phase = (int)((w0 >> 4) & 1);
    s->hasA = (int)((w0 >> 5) & 1);
    s->hasB = (int)((w0 >> 6) & 1);
    for (int b = 0; b < 2; b++) {
        int code = (int)((w0 >> (8 + 8 * b)) & 0xFF);
        if (code != 0xFF) { s->bset[b] = 1; s->bt[b] = code >> 7; s->ba[b] = 500 * (code & 0x7F); }
    }
    for (int i = 0; i < 5; i++) {
        s->A[i] = (int)((w0 >> (24 + 4 * i)) & 0xF);
        s->B[i] = (int)((w0 >> (44 + 4 * i)) & 0xF);
    }
    for (int p = 0; p < 2; p++) {
        uint64_t wa = w[1 + 3 * p], wb = w[2 + 3 * p], wc = w[3 + 3 * p];
        pl_t* q = &s->p[p];
        q->n = (int)((wa >> 40) & 0xF);
        for (int i = 0; i < 10; i++) q->d[i] = (int)((wa >> (4 * i)) & 0xF);
        q->used = (int)((wa >> 44) & 0xFFF);
        for (int i = 0; i < 8; i++) q->cat[i] = 1000 * (int)((wb >> (8 * i)) & 0xFF);
        for (int i = 0; i < 4; i++) q->cat[8 + i] = 1000 * (int)((wc >> (8 * i)) & 0xFF);
        q->bid = (int32_t)(uint32_t)(wc >> 32);
    }
}
static void pack(const st_t* s, uint64_t* w) {
    uint64_t w0 = (uint64_t)(s->round & 0xF) | ((uint64_t)(s->phase & 1) << 4);
    if (s->hasA) w0 |= 1ull << 5;
    if (s->hasB) w0 |= 1ull << 6;
    for (int b = 0; b < 2; b++) {
        uint64_t code = s->bset[b] ? (((uint64_t)s->bt[b] << 7) | (uint64_t)(s->ba[b] / 500)) : 0xFF;
        w0 |= code << (8 + 8 * b);
    }
    for (int i = 0; i < 5; i++) {
        if (s->hasA) w0 |= (uint64_t)s->A[i] << (24 + 4 * i);
        if (s->hasB) w0 |= (uint64_t)s->B[i] << (44 + 4 * i);
    }
    w[0] = w0;
    for (int p = 0; p < 2; p++) {
        const pl_t* q = &s->p[p];
        uint64_t wa = 0, wb = 0, wc = 0;
        for (int i = 0; i < q->n; i++) wa |= (uint64_t)q->d[i] << (4 * i);
        wa |= (uint64_t)q->n << 40;
        wa |= (uint64_t)(q->used & 0xFFF) << 44;
        for (int i = 0; i < 8; i++) wb |= (uint64_t)(q->cat[i] / 1000) << (8 * i);
        for (int i = 0; i < 4; i++) wc |= (uint64_t)(q->cat[8 + i] / 1000) << (8 * i);
        wc |= (uint64_t)(uint32_t)q->bid << 32;
        w[1 + 3 * p] = wa; w[2 + 3 * p] = wb; w[3 + 3 * p] = wc;
    }
    w[7] = 0;
}

/* ------------------------------------------------------------------ scoring */
/* score_category  YachtGame.py:57-108 */
int or_score_category(int cat, const int* dice) {
    int cnt[7] = {0}, sum = 0;
    for (int i = 0; i < 5; i++) { cnt[dice[i]]++; sum += dice[i]; }
    if (cat <= 5) return 1000 * (cat + 1) * cnt[cat + 1];
    if (cat == 6) return 1000 * sum;
    if (cat == 7) {
        for (int v = 1; v <= 6; v++) if (cnt[v] >= 4) return 1000 * sum;
        return 0;
    }
    if (cat == 8) {
        int pair = 0, triple = 0;
        for (int v = 1; v <= 6; v++) {
            if (cnt[v] == 2 || cnt[v] == 5) pair = 1;
            if (cnt[v] == 3 || cnt[v] == 5) triple = 1;
        }
        return (pair && triple) ? 1000 * sum : 0;
    }
    int e[7];
    for (int v = 1; v <= 6; v++) e[v] = cnt[v] > 0;
    if (cat == 9) return ((e[1] && e[2] && e[3] && e[4]) || (e[2] && e[3] && e[4] && e[5]) ||
                          (e[3] && e[4] && e[5] && e[6])) ? 15000 : 0;
    if (cat == 10) return ((e[1] && e[2] && e[3] && e[4] && e[5]) || (e[2] && e[3] && e[4] && e[5] && e[6]))
                              ? 30000 : 0;
    if (cat == 11) {
        for (int v = 1; v <= 6; v++) if (cnt[v] == 5) return 50000;
        return 0;
    }
    return -1;
}

static int popcount12(int m) { return __builtin_popcount((unsigned)m & 0xFFF); }
static int total_with_bonus(const pl_t* q) { /* YachtGame.py:125-130 */
    int basic = 0, all = 0;
    for (int i = 0; i < 6; i++) basic += q->cat[i];
    for (int i = 0; i < NCAT; i++) all += q->cat[i];
    return all + (basic >= 63000 ? 35000 : 0) + q->bid;
}

/* ------------------------------------------------------------------ transitions */
enum { ST_OK = 0, ST_VALUE_BID = 1, ST_VALUE_SCORE = 2, ST_RUNTIME = 3, ST_ASSERT = 4, ST_CAPACITY = 5 };

static int extend(pl_t* q, const int* dice, int has) {
    if (!has) return 0;
    if (q->n + 5 > 10) return -1;
    for (int i = 0; i < 5; i++) q->d[q->n++] = dice[i];
    return 0;
}

/* _resolve_bids_and_assign  YachtGame.py:502-542 */
static int resolve(st_t* s, stream_t* rs) {
    if (!(s->bset[0] && s->bset[1])) return ST_ASSERT;
    int t1 = s->bt[0], a1 = s->ba[0], t2 = s->bt[1], a2 = s->ba[1];
    int g0 = t1, g1 = t2;
    if (g0 == g1) {
        int winner;
        if (a1 > a2) winner = 0;
        else if (a2 > a1) winner = 1;
        else winner = st_below(rs, 2); /* tiebreak_uniform  YachtGame.py:158-159 */
        if (winner == 0) g1 = 1 - g0;
        else g0 = 1 - g1;
    }
    s->p[0].bid += (g0 == t1) ? -a1 : +a1;
    s->p[1].bid += (g1 == t2) ? -a2 : +a2;
    if (extend(&s->p[0], g0 == 0 ? s->A : s->B, g0 == 0 ? s->hasA : s->hasB)) return ST_CAPACITY;
    if (extend(&s->p[1], g1 == 0 ? s->A : s->B, g1 == 0 ? s->hasA : s->hasB)) return ST_CAPACITY;
    return ST_OK;
}
static void roll_five(stream_t* rs, int* d) { for (int i = 0; i < 5; i++) d[i] = st_die(rs); }

/* getNextState  YachtGame.py:260-372 */
static int step(const st_t* in, int player, int action, stream_t* rs, st_t* s, int* next_player) {
    *s = *in; /* _copy_state  YachtGame.py:480-500 */
    if (s->phase == 0 && s->round != 13) {
        if (!(action >= 0 && action < NBID)) return ST_VALUE_BID;
        int t = action / BID_LEVELS, amt = 500 * (action % BID_LEVELS);
        if (!s->bset[0] && !s->bset[1]) {
            int b = (player == 1) ? 0 : 1;
            s->bset[b] = 1; s->bt[b] = t; s->ba[b] = amt;
            *next_player = -player;
            return ST_OK;
        }
        int b = (player == 1) ? 0 : 1;
        s->bset[b] = 1; s->bt[b] = t; s->ba[b] = amt;
        int r = resolve(s, rs);
        if (r) return r;
        if (s->round != 1) {
            s->phase = 1;
            *next_player = 1;
        } else {
            s->round += 1;
            s->bset[0] = s->bset[1] = 0; s->bt[0] = s->bt[1] = 0; s->ba[0] = s->ba[1] = 0;
            roll_five(rs, s->A); s->hasA = 1;
            roll_five(rs, s->B); s->hasB = 1;
            s->phase = 0;
            *next_player = 1;
        }
        return ST_OK;
    }
    if (s->phase == 1) {
        if (!(action >= NBID && action < ASIZE)) return ST_VALUE_SCORE;
        int base = action - NBID, cat = base / NCOMB, ci = base % NCOMB;
        pl_t* me = &s->p[player == 1 ? 0 : 1];
        if ((me->used >> cat) & 1) { *next_player = -player; return ST_OK; }
        const uint8_t* cb = COMB[ci];
        if (cb[4] >= me->n) { *next_player = -player; return ST_OK; }
        int chosen[5];
        for (int i = 0; i < 5; i++) chosen[i] = me->d[cb[i]];
        int sc = or_score_category(cat, chosen);
        int nd[10], k = 0, j = 0;
        for (int i = 0; i < me->n; i++) {
            if (j < 5 && cb[j] == i) { j++; continue; }
            nd[k++] = me->d[i];
        }
        for (int i = 0; i < 10; i++) me->d[i] = i < k ? nd[i] : 0;
        me->n = k;
        me->used |= 1 << cat;
        me->cat[cat] = sc;
        if (s->round == 13) {
            if (popcount12(s->p[0].used) == NCAT && popcount12(s->p[1].used) == NCAT) *next_player = 1;
            else *next_player = -player;
            return ST_OK;
        }
        if (player == -1) {
            s->round += 1;
            s->bset[0] = s->bset[1] = 0; s->bt[0] = s->bt[1] = 0; s->ba[0] = s->ba[1] = 0;
            if (s->round != 13) {
                roll_five(rs, s->A); s->hasA = 1;
                roll_five(rs, s->B); s->hasB = 1;
                s->phase = 0;
            } else {
                s->phase = 1;
            }
            *next_player = 1;
            return ST_OK;
        }
        *next_player = -player;
        return ST_OK;
    }
    return ST_RUNTIME;
}

/* getValidMoves  YachtGame.py:374-406 */
static int valid_moves(const st_t* s, int player, uint8_t* v) {
    memset(v, 0, ASIZE);
    if (s->phase == 0 && s->round != 13) {
        memset(v, 1, NBID);
        return NBID;
    }
    if (s->phase == 1) {
        const pl_t* me = &s->p[player == 1 ? 0 : 1];
        int n = me->n, cnt = 0;
        if (n < 5) return 0;
        for (int c = 0; c < NCAT; c++) {
            if ((me->used >> c) & 1) continue;
            for (int ci = 0; ci < NCOMB; ci++)
                if (COMB[ci][4] < n) { v[NBID + c * NCOMB + ci] = 1; cnt++; }
        }
        return cnt;
    }
    return 0;
}

/* getGameEnded  YachtGame.py:408-428 */
static double game_ended(const st_t* s, int player, int* totals) {
    int t1 = total_with_bonus(&s->p[0]), t2 = total_with_bonus(&s->p[1]);
    if (totals) { totals[0] = t1; totals[1] = t2; }
    if (!(popcount12(s->p[0].used) == NCAT && popcount12(s->p[1].used) == NCAT)) return 0.0;
    if (t1 == t2) return 1e-4;
    int winner = t1 > t2 ? 1 : -1;
    return (double)(player == 1 ? winner : -winner);
}

/* getCanonicalForm  YachtGame.py:430-442 (no bid masking, despite the docstring) */
static void canonical(const st_t* in, int player, st_t* out) {
    *out = *in;
    if (player == 1) return;
    out->p[0] = in->p[1]; out->p[1] = in->p[0];
    out->bset[0] = in->bset[1]; out->bt[0] = in->bt[1]; out->ba[0] = in->ba[1];
    out->bset[1] = in->bset[0]; out->bt[1] = in->bt[0]; out->ba[1] = in->ba[0];
}

/* state_to_vec  yacht/NNet.py:50-86 */
static void featurize(const st_t* s, float* x) {
    int k = 0;
    x[k++] = (float)((double)s->round / 13.0);
    x[k++] = s->phase == 0 ? 1.0f : 0.0f;
    x[k++] = s->phase == 1 ? 1.0f : 0.0f;
    for (int p = 0; p < 2; p++)
        for (int i = 0; i < 10; i++)
            x[k++] = i < s->p[p].n ? (float)(((double)s->p[p].d[i] - 3.5) / 3.5) : -1.0f;
    int vis = (s->phase == 0 && s->round != 13);
    for (int r = 0; r < 2; r++) {
        int has = r == 0 ? s->hasA : s->hasB;
        const int* d = r == 0 ? s->A : s->B;
        for (int i = 0; i < 5; i++) x[k++] = (vis && has) ? (float)(((double)d[i] - 3.5) / 3.5) : -1.0f;
    }
    for (int p = 0; p < 2; p++)
        for (int i = 0; i < NCAT; i++) x[k++] = (float)((s->p[p].used >> i) & 1);
    x[k++] = (float)((double)s->p[0].bid * 1e-5);
    x[k++] = (float)((double)s->p[1].bid * 1e-5);
}

/* ------------------------------------------------------------------ hash + hash prior (spec.py) */
static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
uint64_t or_key_hash(const uint64_t* w) {
    uint64_t h = 0x243F6A8885A308D3ull;
    for (int i = 0; i < 8; i++) h = mix64(h ^ (w[i] + 0x9E3779B97F4A7C15ull * (uint64_t)(i + 1)));
    return h;
}
static void hash_prior(const uint64_t* w, float* pi, float* v) {
    uint64_t h = or_key_hash(w);
    for (int a = 0; a < ASIZE; a++) {
        uint64_t z = mix64(h ^ (0xD1B54A32D192ED03ull * (uint64_t)(a + 1)));
        pi[a] = ((float)((z >> 40) & 0xFFFF) + 1.0f) * (1.0f / 65536.0f);
    }
    uint64_t zv = mix64(h ^ 0x8CB92BA72F3D8DD7ull);
    *v = (float)((double)((int64_t)((zv >> 40) & 0xFFFF) - 32768) / 32768.0);
}

/* ------------------------------------------------------------------ numpy float32 pairwise sum */
/* numpy/_core/src/umath/loops_utils.h.src  @TYPE@_pairwise_sum  (np.sum of a contiguous
 * float32 array, MCTS.py:89); verified bitwise against numpy 2.2.6 */
static float pw_sum(const float* a, long n) {
    if (n < 8) {
        float r = 0.0f;
        for (long i = 0; i < n; i++) r += a[i];
        return r;
    } else if (n <= 128) {
        float r[8];
        for (int j = 0; j < 8; j++) r[j] = a[j];
        long i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; j++) r[j] += a[i + j];
        float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += a[i];
        return res;
    } else {
        long n2 = n / 2;
        n2 -= n2 % 8;
        return pw_sum(a, n2) + pw_sum(a + n2, n - n2);
    }
}
float or_pairwise_sum(const float* a, long n) { return pw_sum(a, n); }

/* ------------------------------------------------------------------ MLP (YachtNNet) */
/* yacht/pytorch/YachtNNet.py:8-70, eval mode (dropout = identity). Weights are kept
 * transposed ([in][out]) so the f32 loops vectorise without reassociation. */
typedef struct {
    int H, NB;
    int rev; /* 1: every Linear sums its inputs last to first - another valid f32 order (tests only) */
    float *w_in, *b_in, *g_in, *be_in;                       /* [59][H] */
    float **w1, **b1, **g1, **be1, **w2, **b2, **g2, **be2;  /* per block [H][H] */
    float *g_pi, *be_pi, *w_pi, *b_pi;                        /* w_pi [H][3226] */
    float *g_v, *be_v, *w_v1, *b_v1, *w_v2, *b_v2;            /* w_v1 [H][128], w_v2 [128] */
} net_t;

static float* tr_copy(const float* w, int out, int in) { /* torch [out][in] -> [in][out] */
    float* t = (float*)malloc(sizeof(float) * (size_t)out * in);
    for (int o = 0; o < out; o++)
        for (int i = 0; i < in; i++) t[(size_t)i * out + o] = w[(size_t)o * in + i];
    return t;
}
static float* dup(const float* w, int n) {
    float* t = (float*)malloc(sizeof(float) * n);
    memcpy(t, w, sizeof(float) * n);
    return t;
}
/* params: flat list in state_dict order (names: spec.closed_form_weights) */
void* or_net_create(int H, int NB, const float* const* p) {
    net_t* n = (net_t*)calloc(1, sizeof(net_t));
    n->H = H; n->NB = NB;
    int k = 0;
    n->w_in = tr_copy(p[k++], H, FEAT); n->b_in = dup(p[k++], H);
    n->g_in = dup(p[k++], H); n->be_in = dup(p[k++], H);
    n->w1 = calloc(NB, sizeof(float*)); n->b1 = calloc(NB, sizeof(float*));
    n->g1 = calloc(NB, sizeof(float*)); n->be1 = calloc(NB, sizeof(float*));
    n->w2 = calloc(NB, sizeof(float*)); n->b2 = calloc(NB, sizeof(float*));
    n->g2 = calloc(NB, sizeof(float*)); n->be2 = calloc(NB, sizeof(float*));
    for (int b = 0; b < NB; b++) {
        n->w1[b] = tr_copy(p[k++], H, H); n->b1[b] = dup(p[k++], H);
        n->g1[b] = dup(p[k++], H); n->be1[b] = dup(p[k++], H);
        n->w2[b] = tr_copy(p[k++], H, H); n->b2[b] = dup(p[k++], H);
        n->g2[b] = dup(p[k++], H); n->be2[b] = dup(p[k++], H);
    }
    n->g_pi = dup(p[k++], H); n->be_pi = dup(p[k++], H);
    n->w_pi = tr_copy(p[k++], ASIZE, H); n->b_pi = dup(p[k++], ASIZE);
    n->g_v = dup(p[k++], H); n->be_v = dup(p[k++], H);
    n->w_v1 = tr_copy(p[k++], 128, H); n->b_v1 = dup(p[k++], 128);
    n->w_v2 = dup(p[k++], 128); n->b_v2 = dup(p[k++], 1);
    return n;
}
void or_net_set_order(void* h, int rev) { ((net_t*)h)->rev = rev ? 1 : 0; }
void or_net_destroy(void* h) {
    net_t* n = (net_t*)h;
    if (!n) return;
    free(n->w_in); free(n->b_in); free(n->g_in); free(n->be_in);
    for (int b = 0; b < n->NB; b++) {
        free(n->w1[b]); free(n->b1[b]); free(n->g1[b]); free(n->be1[b]);
        free(n->w2[b]); free(n->b2[b]); free(n->g2[b]); free(n->be2[b]);
    }
    free(n->w1); free(n->b1); free(n->g1); free(n->be1); free(n->w2); free(n->b2); free(n->g2); free(n->be2);
    free(n->g_pi); free(n->be_pi); free(n->w_pi); free(n->b_pi);
    free(n->g_v); free(n->be_v); free(n->w_v1); free(n->b_v1); free(n->w_v2); free(n->b_v2);
    free(n);
}
static void linear(const float* wt, const float* b, const float* x, int in, int out, float* y, int rev) {
    for (int o = 0; o < out; o++) y[o] = 0.0f;
    for (int k = 0; k < in; k++) {
        const int i = rev ? in - 1 - k : k;
        const float xi = x[i];
        const float* row = wt + (size_t)i * out;
        for (int o = 0; o < out; o++) y[o] += row[o] * xi;
    }
    for (int o = 0; o < out; o++) y[o] += b[o];
}
static void layernorm(float* x, int n, const float* g, const float* b) { /* nn.LayerNorm eps 1e-5 */
    double m = 0, v = 0;
    for (int i = 0; i < n; i++) m += x[i];
    m /= n;
    for (int i = 0; i < n; i++) v += (x[i] - m) * (x[i] - m);
    v /= n;
    double r = 1.0 / sqrt(v + 1e-5);
    for (int i = 0; i < n; i++) x[i] = (float)((x[i] - m) * r) * g[i] + b[i];
}
static inline float silu(float x) { return x / (1.0f + expf(-x)); }

static void net_forward(const net_t* n, const float* x, float* pi, float* v) {
    int H = n->H;
    float h[1024], t[1024], u[1024];
    linear(n->w_in, n->b_in, x, FEAT, H, h, n->rev);
    layernorm(h, H, n->g_in, n->be_in);
    for (int i = 0; i < H; i++) h[i] = silu(h[i]);
    for (int b = 0; b < n->NB; b++) {
        linear(n->w1[b], n->b1[b], h, H, H, t, n->rev);
        for (int i = 0; i < H; i++) t[i] = silu(t[i]);
        layernorm(t, H, n->g1[b], n->be1[b]);
        linear(n->w2[b], n->b2[b], t, H, H, u, n->rev);
        for (int i = 0; i < H; i++) u[i] = silu(u[i]);
        layernorm(u, H, n->g2[b], n->be2[b]);
        for (int i = 0; i < H; i++) h[i] += u[i];
    }
    memcpy(t, h, sizeof(float) * H);
    layernorm(t, H, n->g_pi, n->be_pi);
    for (int i = 0; i < H; i++) t[i] = silu(t[i]);
    linear(n->w_pi, n->b_pi, t, H, ASIZE, pi, n->rev);
    memcpy(t, h, sizeof(float) * H);
    layernorm(t, H, n->g_v, n->be_v);
    for (int i = 0; i < H; i++) t[i] = silu(t[i]);
    linear(n->w_v1, n->b_v1, t, H, 128, u, n->rev);
    double acc = n->b_v2[0];
    for (int i = 0; i < 128; i++) acc += (double)n->w_v2[i] * silu(u[i]);
    *v = tanhf((float)acc);
    /* exp(log_softmax(pi))  NNet.py:193 */
    float mx = pi[0];
    for (int a = 1; a < ASIZE; a++) mx = pi[a] > mx ? pi[a] : mx;
    double se = 0;
    for (int a = 0; a < ASIZE; a++) se += exp((double)pi[a] - mx);
    double lse = log(se);
    for (int a = 0; a < ASIZE; a++) pi[a] = (float)exp((double)pi[a] - mx - lse);
}

/* ------------------------------------------------------------------ MCTS */
/* Python value kinds on the search path (Q11): python int 0 (dead node, MCTS.py:147),
 * python float (terminal -Es, MCTS.py:82), numpy float32 (-v of predict, MCTS.py:115). */
enum { T_INT = 0, T_F64 = 1, T_F32 = 2 };
typedef struct { double v; int t; } pyv;
static inline pyv pv(double v, int t) { pyv r = {v, t}; return r; }
static inline pyv pv_neg(pyv a) { return pv(-a.v, a.t); }
static inline pyv pv_mul_int(int n, pyv q) {
    if (q.t == T_F32) return pv((double)((float)n * (float)q.v), T_F32);
    return pv((double)n * q.v, q.t);
}
static inline pyv pv_add(pyv a, pyv b) {
    if (a.t == T_F32 || b.t == T_F32) return pv((double)((float)a.v + (float)b.v), T_F32);
    if (a.t == T_F64 || b.t == T_F64) return pv(a.v + b.v, T_F64);
    return pv(a.v + b.v, T_INT);
}
static inline pyv pv_div_int(pyv a, int d) {
    if (a.t == T_F32) return pv((double)((float)a.v / (float)d), T_F32);
    return pv(a.v / (double)d, T_F64); /* int / int is python true division */
}

typedef struct { int N; pyv Q; } edge_t;
typedef struct {
    uint64_t key[8];
    double Es;
    int hasP, Ns, nvalid;
    float* P;
    uint8_t* valid;
    int32_t* eidx; /* per action -> edge index or -1 */
    int ne, ecap;
    edge_t* e;
} node_t;
typedef struct {
    node_t* nodes;
    int n, cap;
    int32_t* slots; /* open addressing, -1 empty */
    int hcap;
} tree_t;

static void tree_init(tree_t* t) {
    t->cap = 1024; t->n = 0;
    t->nodes = (node_t*)calloc(t->cap, sizeof(node_t));
    t->hcap = 4096;
    t->slots = (int32_t*)malloc(sizeof(int32_t) * t->hcap);
    memset(t->slots, 0xFF, sizeof(int32_t) * t->hcap);
}
static void tree_free(tree_t* t) {
    for (int i = 0; i < t->n; i++) {
        free(t->nodes[i].P); free(t->nodes[i].valid); free(t->nodes[i].eidx); free(t->nodes[i].e);
    }
    free(t->nodes); free(t->slots);
}
static int tree_find(tree_t* t, const uint64_t* key, uint64_t h) {
    uint32_t m = t->hcap - 1;
    for (uint32_t s = (uint32_t)h & m;; s = (s + 1) & m) {
        int id = t->slots[s];
        if (id < 0) return -1 - (int)s;
        if (memcmp(t->nodes[id].key, key, 64) == 0) return id;
    }
}
static void tree_grow(tree_t* t) {
    int nh = t->hcap * 2;
    int32_t* ns = (int32_t*)malloc(sizeof(int32_t) * nh);
    memset(ns, 0xFF, sizeof(int32_t) * nh);
    for (int i = 0; i < t->n; i++) {
        uint32_t m = nh - 1;
        uint32_t s = (uint32_t)or_key_hash(t->nodes[i].key) & m;
        while (ns[s] >= 0) s = (s + 1) & m;
        ns[s] = i;
    }
    free(t->slots);
    t->slots = ns; t->hcap = nh;
}
static int tree_insert(tree_t* t, const uint64_t* key, int* created) {
    *created = 0;
    if (t->n == t->cap) {
        t->cap *= 2;
        t->nodes = (node_t*)realloc(t->nodes, sizeof(node_t) * t->cap);
        memset(t->nodes + t->n, 0, sizeof(node_t) * (t->cap - t->n));
    }
    if (2 * (t->n + 1) > t->hcap) tree_grow(t);
    uint64_t h = or_key_hash(key);
    int f = tree_find(t, key, h);
    if (f >= 0) return f;
    int id = t->n++;
    *created = 1;
    memcpy(t->nodes[id].key, key, 64);
    t->slots[-1 - f] = id;
    return id;
}

typedef struct {
    int mode; /* 0 hash prior, 1 mlp, 2 replay */
    const net_t* net;
    const float* rpi; const float* rv; long rn; long ri; /* replay log */
    long calls;
    int error;
} pred_t;
static void predict(pred_t* pr, const st_t* s, const uint64_t* key, float* pi, float* v) {
    pr->calls++;
    if (pr->mode == 0) { hash_prior(key, pi, v); return; }
    if (pr->mode == 1) {
        float x[FEAT];
        featurize(s, x);
        net_forward(pr->net, x, pi, v);
        return;
    }
    if (pr->ri >= pr->rn) { pr->error = 1; memset(pi, 0, sizeof(float) * ASIZE); *v = 0; return; }
    memcpy(pi, pr->rpi + (size_t)pr->ri * ASIZE, sizeof(float) * ASIZE);
    *v = pr->rv[pr->ri];
    pr->ri++;
}

typedef struct {
    tree_t tree;
    pred_t* pred;
    stream_t* rs;
    float c32;
    long scanned; /* valid actions scanned by UCB loops */
    int error;
} mcts_t;

/* MCTS.search  MCTS.py:56-164 */
static pyv search(mcts_t* m, const st_t* s) {
    uint64_t key[8];
    pack(s, key);
    int created;
    int id = tree_insert(&m->tree, key, &created);
    node_t* nd = &m->tree.nodes[id];
    if (created) nd->Es = game_ended(s, 1, NULL); /* Es cache, MCTS.py:78-79 */
    if (nd->Es != 0.0) return pv(-nd->Es, T_F64);
    if (!nd->hasP) {
        float* pi = (float*)malloc(sizeof(float) * ASIZE);
        float v;
        predict(m->pred, s, key, pi, &v);
        nd = &m->tree.nodes[id];
        nd->valid = (uint8_t*)malloc(ASIZE);
        nd->nvalid = valid_moves(s, 1, nd->valid);
        float* P = pi;
        for (int a = 0; a < ASIZE; a++) P[a] = P[a] * (float)nd->valid[a];
        float sum = pw_sum(P, ASIZE);
        if (sum > 0.0f) {
            for (int a = 0; a < ASIZE; a++) P[a] = P[a] / sum;
        } else {
            for (int a = 0; a < ASIZE; a++) P[a] = P[a] + (float)nd->valid[a];
            float sv = pw_sum(P, ASIZE);
            if (sv > 0.0f) {
                for (int a = 0; a < ASIZE; a++) P[a] = P[a] / sv;
            } else {
                for (int a = 0; a < ASIZE; a++) P[a] = 0.0f;
                P[0] = 1.0f;
            }
        }
        nd->P = P;
        nd->eidx = (int32_t*)malloc(sizeof(int32_t) * ASIZE);
        memset(nd->eidx, 0xFF, sizeof(int32_t) * ASIZE);
        nd->hasP = 1;
        nd->Ns = 0;
        return pv(-(double)v, T_F32);
    }
    /* UCB argmax, MCTS.py:117-135 (float32 arithmetic, strict '>' => lowest index wins) */
    float cur_best = -INFINITY;
    int best = -1;
    int Ns = nd->Ns;
    float sq = (float)sqrt((double)Ns), sqe = (float)sqrt((double)Ns + 1e-8);
    for (int a = 0; a < ASIZE; a++) {
        if (!nd->valid[a]) continue;
        m->scanned++;
        float u;
        int ei = nd->eidx[a];
        if (ei >= 0) {
            const edge_t* e = &nd->e[ei];
            float term = ((m->c32 * nd->P[a]) * sq) / (float)(1 + e->N);
            u = (float)e->Q.v + term;
        } else {
            u = (m->c32 * nd->P[a]) * sqe;
        }
        if (u > cur_best) { cur_best = u; best = a; }
    }
    int a = best;
    if (a == -1 || !nd->valid[a]) {
        a = -1;
        for (int b = 0; b < ASIZE; b++) if (nd->valid[b]) { a = b; break; }
        if (a < 0) return pv(0.0, T_INT);
    }
    st_t nx, cn;
    int np_;
    int stt = step(s, 1, a, m->rs, &nx, &np_);
    if (stt) { m->error = 100 + stt; return pv(0.0, T_INT); }
    canonical(&nx, np_, &cn);
    pyv v = search(m, &cn);
    nd = &m->tree.nodes[id];
    int ei = nd->eidx[a];
    if (ei >= 0) {
        edge_t* e = &nd->e[ei];
        e->Q = pv_div_int(pv_add(pv_mul_int(e->N, e->Q), v), e->N + 1);
        e->N += 1;
    } else {
        if (nd->ne == nd->ecap) {
            nd->ecap = nd->ecap ? 2 * nd->ecap : 4;
            nd->e = (edge_t*)realloc(nd->e, sizeof(edge_t) * nd->ecap);
        }
        nd->eidx[a] = nd->ne;
        nd->e[nd->ne].N = 1;
        nd->e[nd->ne].Q = v;
        nd->ne++;
    }
    nd->Ns += 1;
    return pv_neg(v);
}

/* ------------------------------------------------------------------ episode (Coach.executeEpisode) */
typedef struct {
    int sims, temp_threshold, max_moves;
    double cpuct;
    int mode;
} ep_cfg_t;

/* Per-move outputs; arrays are [max_moves] for one env (NULL allowed). */
typedef struct {
    uint64_t* canon;   /* [M][8] */
    int32_t* mv;       /* [M][8]: temp, player, action, n_ps, root_ns, nvisited, status, 0 */
    uint64_t* ctr;     /* [M][2]: ctr before search, ctr before real step */
    int32_t* counts;   /* [M][3226] dense visit counts (may be NULL) */
    double* values;    /* [M] */
    int64_t* stats;    /* [8]: moves, expansions, nodes, scanned, ctr_end, error, 0, 0 */
    uint64_t* final_state; /* [8] */
} ep_out_t;

static int run_episode(const ep_cfg_t* cfg, pred_t* pr, uint64_t seed, uint32_t env, ep_out_t* out) {
    init_comb();
    stream_t rs = {seed, env, 0};
    mcts_t m;
    memset(&m, 0, sizeof(m));
    tree_init(&m.tree);
    m.pred = pr; m.rs = &rs; m.c32 = (float)cfg->cpuct;
    /* getInitBoard  YachtGame.py:232-237 */
    st_t board;
    memset(&board, 0, sizeof(board));
    board.round = 1; board.phase = 0;
    roll_five(&rs, board.A); board.hasA = 1;
    roll_five(&rs, board.B); board.hasB = 1;
    int cur = 1, stepi = 0, err = 0;
    int* players = (int*)malloc(sizeof(int) * (cfg->max_moves > 0 ? cfg->max_moves : 1));
    int32_t* counts = (int32_t*)malloc(sizeof(int32_t) * ASIZE);
    double* cdf = (double*)malloc(sizeof(double) * ASIZE);
    double r = 0.0;
    while (1) {
        if (stepi >= cfg->max_moves) { err = 1; break; }
        int j = stepi;
        stepi++;
        st_t canon;
        canonical(&board, cur, &canon);
        int temp = stepi < cfg->temp_threshold ? 1 : 0;
        if (out->ctr) out->ctr[2 * j] = rs.ctr;
        for (int i = 0; i < cfg->sims; i++) search(&m, &canon);
        if (m.error || pr->error) { err = m.error ? m.error : 2; break; }
        /* getActionProb  MCTS.py:40-54 */
        uint64_t key[8];
        pack(&canon, key);
        int id = tree_find(&m.tree, key, or_key_hash(key));
        const node_t* nd = id >= 0 ? &m.tree.nodes[id] : NULL;
        int nvis = 0, mx = 0;
        for (int a = 0; a < ASIZE; a++) {
            int c = (nd && nd->eidx && nd->eidx[a] >= 0) ? nd->e[nd->eidx[a]].N : 0;
            counts[a] = c;
            if (c) nvis++;
            if (c > mx) mx = c;
        }
        int action;
        if (temp == 0) {
            int nb = 0;
            for (int a = 0; a < ASIZE; a++) if (counts[a] == mx) nb++;
            int pick = st_below(&rs, nb), bestA = -1;
            for (int a = 0; a < ASIZE; a++) if (counts[a] == mx && pick-- == 0) { bestA = a; break; }
            /* np.random.choice(len(pi), p=one-hot): cdf step at bestA, one uniform draw */
            double u = st_uniform53(&rs);
            (void)u;
            action = bestA;
        } else {
            double total = 0.0;
            for (int a = 0; a < ASIZE; a++) total += (double)counts[a];
            if (total == 0.0) { err = 3; break; }
            double c = 0.0;
            for (int a = 0; a < ASIZE; a++) { c += (double)counts[a] / total; cdf[a] = c; }
            double last = cdf[ASIZE - 1];
            double u = st_uniform53(&rs);
            action = ASIZE;
            for (int a = 0; a < ASIZE; a++) if (cdf[a] / last > u) { action = a; break; }
        }
        if (out->canon) memcpy(out->canon + 8 * j, key, 64);
        if (out->counts) memcpy(out->counts + (size_t)ASIZE * j, counts, sizeof(int32_t) * ASIZE);
        players[j] = cur;
        if (out->ctr) out->ctr[2 * j + 1] = rs.ctr;
        st_t nb;
        int np_;
        int stt = step(&board, cur, action, &rs, &nb, &np_);
        if (out->mv) {
            int32_t* q = out->mv + 8 * j;
            q[0] = temp; q[1] = cur; q[2] = action; q[3] = (int32_t)pr->calls;
            q[4] = nd ? nd->Ns : -1; q[5] = nvis; q[6] = stt; q[7] = 0;
        }
        if (stt) { err = 200 + stt; break; }
        board = nb; cur = np_;
        r = game_ended(&board, cur, NULL);
        if (r != 0.0) break;
    }
    if (out->values)
        for (int j = 0; j < stepi; j++) out->values[j] = r * ((players[j] != cur) ? -1.0 : 1.0);
    if (out->stats) {
        out->stats[0] = stepi; out->stats[1] = pr->calls; out->stats[2] = m.tree.n; out->stats[3] = m.scanned;
        out->stats[4] = (int64_t)rs.ctr; out->stats[5] = err;
    }
    if (out->final_state) pack(&board, out->final_state);
    if (out->stats) { /* live-set footprint under round eviction (engine sizing): max over root rounds
                         of live nodes / valid entries / edges */
        long nv[16] = {0}, nn[16] = {0}, ne[16] = {0};
        for (int i = 0; i < m.tree.n; i++) {
            int rr = (int)(m.tree.nodes[i].key[0] & 0xF);
            nn[rr]++; nv[rr] += m.tree.nodes[i].nvalid; ne[rr] += m.tree.nodes[i].ne;
        }
        long bv = nv[1] + nv[2], bn = nn[1] + nn[2], be = ne[1] + ne[2];
        for (int rr = 2; rr < 14; rr++) {
            if (nv[rr] > bv) bv = nv[rr];
            if (nn[rr] > bn) bn = nn[rr];
            if (ne[rr] > be) be = ne[rr];
        }
        out->stats[6] = bv; out->stats[7] = bn | (be << 32);
    }
    free(counts); free(cdf); free(players);
    tree_free(&m.tree);
    return err;
}

/* ------------------------------------------------------------------ GreedyYachtPlayer */
/* YachtPlayers.py:38-171, 186-214 on a canonical board.  Points are the game's units (x1000). */
#define BASIC_BONUS 35000
#define BASIC_BONUS_THRESHOLD 63000
static int basic_sum(const pl_t* q) {
    int b = 0;
    for (int c = 0; c < 6; c++) b += q->cat[c];
    return b;
}
/* best immediate gain (score + basic bonus when it crosses the threshold) over unused
 * categories x combos of `dice`; the scorer walks combos in order and stops at the first one
 * reaching past the carry (YachtPlayers.py:151-153); the bid potential filters max(comb) < n
 * (:67) - identical for carries of 0, 5 and 10 dice.  *best_action = first maximum. */
static int greedy_best(const pl_t* me, const int* dice, int n, int stop_at_first_invalid, int* best_action) {
    const int basic_before = basic_sum(me);
    int best = INT32_MIN, ba = -1;
    for (int c = 0; c < NCAT; c++) {
        if ((me->used >> c) & 1) continue;
        for (int ci = 0; ci < NCOMB; ci++) {
            if (COMB[ci][4] >= n) {
                if (stop_at_first_invalid) break;
                continue;
            }
            int chosen[5];
            for (int k = 0; k < 5; k++) chosen[k] = dice[COMB[ci][k]];
            const int sc = or_score_category(c, chosen);
            int gain = sc;
            if (c < 6 && basic_before < BASIC_BONUS_THRESHOLD && BASIC_BONUS_THRESHOLD <= basic_before + sc)
                gain += BASIC_BONUS;
            if (gain > best) { best = gain; ba = NBID + c * NCOMB + ci; }
        }
    }
    if (best_action) *best_action = ba;
    return best;
}
/* _score_potential_after_bid  YachtPlayers.py:38-87 */
static int greedy_potential(const st_t* s, const pl_t* me, const int* bundle, int has_bundle) {
    int dice[15], n = 0;
    for (int i = 0; i < me->n; i++) dice[n++] = me->d[i];
    if (has_bundle) /* an absent roll is an empty list */
        for (int i = 0; i < 5; i++) dice[n++] = bundle[i];
    if (s->round == 1) {
        int sum = 0, counts[7] = {0}, mx = 0;
        for (int i = 0; i < n; i++) { sum += dice[i]; counts[dice[i]]++; }
        int v = 1000 * sum;
        for (int f = 1; f <= 6; f++) if (counts[f] > mx) mx = counts[f];
        if (mx >= 4) v += 6000;
        else if (mx == 3) v += 3000;
        const int e1 = counts[1] > 0, e2 = counts[2] > 0, e3 = counts[3] > 0, e4 = counts[4] > 0,
                  e5 = counts[5] > 0, e6 = counts[6] > 0;
        if ((e1 && e2 && e3 && e4) || (e2 && e3 && e4 && e5) || (e3 && e4 && e5 && e6)) v += 5000;
        return v;
    }
    if (n < 5) return 0;
    const int best = greedy_best(me, dice, n, 0, NULL);
    return best == INT32_MIN ? 0 : best;
}
static int total_bb(const pl_t* q) {
    int all = 0;
    for (int c = 0; c < NCAT; c++) all += q->cat[c];
    return q->bid + all + (basic_sum(q) >= BASIC_BONUS_THRESHOLD ? BASIC_BONUS : 0);
}
/* _choose_bid  YachtPlayers.py:90-127: the action may encode past index 100 (bids up to 100,000) */
static int greedy_choose_bid(const st_t* s) {
    const pl_t* me = &s->p[0];
    const int valA = greedy_potential(s, me, s->A, s->hasA), valB = greedy_potential(s, me, s->B, s->hasB);
    int target, gap;
    if (valA >= valB) { target = 0; gap = valA - valB > 0 ? valA - valB : 0; }
    else { target = 1; gap = valB - valA > 0 ? valB - valA : 0; }
    const int diff = total_bb(me) - total_bb(&s->p[1]);
    const double bid_k = 0.5 * ((double)gap / 1000.0) - 0.15 * ((double)diff / 1000.0);
    double r = nearbyint(1000.0 * bid_k);  /* python round(): half to even */
    long bid = (long)r;
    if (bid > 100000) bid = 100000;
    if (bid < 0) bid = 0;
    bid = (bid / 500) * 500;
    return target * BID_LEVELS + (int)(bid / 500);
}
/* _choose_scoring  YachtPlayers.py:131-171 */
static int greedy_choose_scoring(const st_t* s) {
    const pl_t* me = &s->p[0];
    if (me->n < 5) return 0;
    int ba = -1;
    greedy_best(me, me->d, me->n, 1, &ba);
    return ba >= 0 ? ba : 0;
}
/* GreedyYachtPlayer.play  YachtPlayers.py:199-214: the heuristic's action if valid, else
 * np.random.choice(legal) (one below(n) draw), else 0 */
static int greedy_action(const st_t* s, uint8_t* valid, stream_t* rs) {
    const int nv = valid_moves(s, 1, valid);
    const int a = (s->phase == 0 && s->round != 13) ? greedy_choose_bid(s) : greedy_choose_scoring(s);
    if (a >= 0 && a < ASIZE && valid[a]) return a;
    if (nv == 0) return 0;
    int pick = st_below(rs, nv);
    for (int b = 0; b < ASIZE; b++) if (valid[b] && pick-- == 0) return b;
    return 0;
}
/* the heuristic alone (for fixtures / the device kernel): -1 when the player would fall back */
void or_greedy_heuristic(const uint64_t* states, int32_t* actions, int n) {
    init_comb();
    uint8_t* valid = (uint8_t*)malloc(ASIZE);
    for (int i = 0; i < n; i++) {
        st_t s;
        unpack(states + 8 * i, &s);
        valid_moves(&s, 1, valid);
        const int a = (s.phase == 0 && s.round != 13) ? greedy_choose_bid(&s) : greedy_choose_scoring(&s);
        actions[i] = (a >= 0 && a < ASIZE && valid[a]) ? a : -1;
    }
    free(valid);
}

/* GreedyYachtPlayer.play with each state's stream (seed, envs[i], ctr[i]); ctr advanced */
void or_greedy_play(const uint64_t* states, uint64_t seed, const uint32_t* envs, uint64_t* ctr, int32_t* actions,
                    int n) {
    init_comb();
    uint8_t* valid = (uint8_t*)malloc(ASIZE);
    for (int i = 0; i < n; i++) {
        st_t s;
        unpack(states + 8 * i, &s);
        stream_t rs = {seed, envs[i], ctr[i]};
        actions[i] = greedy_action(&s, valid, &rs);
        ctr[i] = rs.ctr;
    }
    free(valid);
}

/* ------------------------------------------------------------------ Arena.playGame (agent vs random) */
/* Arena.py:30-93 with player1/player2 = {MCTS agent: np.argmax(mcts.getActionProb(x, temp=0))
 * (Coach.py:124-125), RandomYachtPlayer.play (YachtPlayers.py:174-183)}.  The agent keeps one
 * MCTS tree for the whole game.  out: result = curPlayer * getGameEnded (Arena.py:93),
 * totals, moves, actions[max_moves], final state, stream counter. */
enum { PK_MCTS = 0, PK_RANDOM = 1, PK_GREEDY = 2 };
/* One Arena.playGame (Arena.py:30-93).  Two MCTS seats share one tree unless `dual`, where the
 * agent's seat searches with trees[0] and the opponent's with trees[1], each with its own
 * predictor (Coach.py:120-125: pmcts and nmcts are two MCTS objects).  `trees` may carry state
 * in from earlier games (the reference's MCTS objects live across a playGames call); NULL: fresh
 * trees for this game. */
static int run_arena(const ep_cfg_t* cfg, pred_t* pr, pred_t* pr2, uint64_t seed, uint32_t env, int agent_seat,
                     int agent_kind, int opp_kind, int dual, mcts_t* trees, double* result, int32_t* totals,
                     int32_t* actions, int64_t* stats, uint64_t* final_state) {
    init_comb();
    stream_t rs = {seed, env, 0};
    mcts_t own[2];
    mcts_t* m = trees ? trees : own;
    if (!trees) {
        memset(own, 0, sizeof(own));
        tree_init(&own[0].tree);
        tree_init(&own[1].tree);
    }
    m[0].pred = pr; m[1].pred = dual ? pr2 : pr;
    for (int k = 0; k < 2; k++) { m[k].rs = &rs; m[k].c32 = (float)cfg->cpuct; }
    const long calls0 = pr->calls + (pr2 && pr2 != pr ? pr2->calls : 0);
    st_t board;
    memset(&board, 0, sizeof(board));
    board.round = 1; board.phase = 0;
    roll_five(&rs, board.A); board.hasA = 1;
    roll_five(&rs, board.B); board.hasB = 1;
    int cur = 1, it = 0, err = 0;
    uint8_t* valid = (uint8_t*)malloc(ASIZE);
    while (game_ended(&board, cur, NULL) == 0.0) {
        if (it >= cfg->max_moves) { err = 1; break; }
        st_t canon;
        canonical(&board, cur, &canon);
        int action = 0;
        const int kind = cur == agent_seat ? agent_kind : opp_kind;
        if (kind == PK_MCTS) {
            mcts_t* mt = &m[dual && cur != agent_seat ? 1 : 0];
            for (int i = 0; i < cfg->sims; i++) search(mt, &canon);
            if (mt->error || mt->pred->error) { err = mt->error ? mt->error : 2; break; }
            uint64_t key[8];
            pack(&canon, key);
            int id = tree_find(&mt->tree, key, or_key_hash(key));
            const node_t* nd = id >= 0 ? &mt->tree.nodes[id] : NULL;
            int mx = 0, nb = 0;
            for (int a = 0; a < ASIZE; a++) {
                int c = (nd && nd->eidx && nd->eidx[a] >= 0) ? nd->e[nd->eidx[a]].N : 0;
                if (c > mx) { mx = c; nb = 0; }
                if (c == mx) nb++;
            }
            int pick = st_below(&rs, nb);  /* np.random.choice(bestAs)  MCTS.py:46 */
            for (int a = 0; a < ASIZE; a++) {
                int c = (nd && nd->eidx && nd->eidx[a] >= 0) ? nd->e[nd->eidx[a]].N : 0;
                if (c == mx && pick-- == 0) { action = a; break; }
            }
        } else if (kind == PK_GREEDY) {
            action = greedy_action(&canon, valid, &rs);
        } else {
            int nv = valid_moves(&canon, 1, valid);
            if (nv > 0) {
                int pick = st_below(&rs, nv);  /* np.random.choice(legal) */
                for (int a = 0; a < ASIZE; a++) if (valid[a] && pick-- == 0) { action = a; break; }
            }
        }
        if (actions) actions[it] = action;
        it++;
        st_t nb_;
        int np_;
        int stt = step(&board, cur, action, &rs, &nb_, &np_);
        if (stt) { err = 200 + stt; break; }
        board = nb_; cur = np_;
    }
    *result = (double)cur * game_ended(&board, cur, totals);
    if (stats) {
        stats[0] = it; stats[1] = pr->calls + (pr2 && pr2 != pr ? pr2->calls : 0) - calls0;
        stats[2] = m[0].tree.n + (dual ? m[1].tree.n : 0); stats[3] = m[0].scanned + m[1].scanned;
        stats[4] = (int64_t)rs.ctr; stats[5] = err;
    }
    if (final_state) pack(&board, final_state);
    free(valid);
    if (!trees) {
        tree_free(&own[0].tree);
        tree_free(&own[1].tree);
    }
    return err;
}

/* ------------------------------------------------------------------ exported batch API (ctypes) */
void or_score_table(const uint64_t* w, const int32_t* players, int32_t* out, int n) {
    init_comb();
    for (int i = 0; i < n; i++) {
        st_t s;
        unpack(w + 8 * i, &s);
        const pl_t* me = &s.p[players[i] == 1 ? 0 : 1];
        for (int c = 0; c < NCAT; c++)
            for (int ci = 0; ci < NCOMB; ci++) {
                int32_t v = -1;
                if (COMB[ci][4] < me->n) {
                    int d[5];
                    for (int k = 0; k < 5; k++) d[k] = me->d[COMB[ci][k]];
                    v = or_score_category(c, d);
                }
                out[((size_t)i * NCAT + c) * NCOMB + ci] = v;
            }
    }
}
void or_score_dice(const int8_t* dice, int32_t* out, int n) {
    for (int i = 0; i < n; i++) {
        int d[5];
        for (int k = 0; k < 5; k++) d[k] = dice[5 * i + k];
        for (int c = 0; c < NCAT; c++) out[i * NCAT + c] = or_score_category(c, d);
    }
}
void or_step(const uint64_t* w, const int32_t* players, const int32_t* actions, uint64_t seed,
             const uint32_t* envs, uint64_t* ctr, uint64_t* out, int32_t* next_players, int8_t* status, int n) {
    init_comb();
    for (int i = 0; i < n; i++) {
        st_t s, o;
        unpack(w + 8 * i, &s);
        stream_t rs = {seed, envs[i], ctr[i]};
        int np_ = 0;
        int st = step(&s, players[i], actions[i], &rs, &o, &np_);
        status[i] = (int8_t)st;
        if (st == 0) { pack(&o, out + 8 * i); next_players[i] = np_; ctr[i] = rs.ctr; }
        else { memset(out + 8 * i, 0, 64); next_players[i] = 0; }
    }
}
void or_valid(const uint64_t* w, const int32_t* players, uint8_t* out, int32_t* counts, int n) {
    init_comb();
    for (int i = 0; i < n; i++) {
        st_t s;
        unpack(w + 8 * i, &s);
        counts[i] = valid_moves(&s, players[i], out + (size_t)ASIZE * i);
    }
}
void or_ended(const uint64_t* w, const int32_t* players, double* r, int32_t* totals, int n) {
    for (int i = 0; i < n; i++) {
        st_t s;
        unpack(w + 8 * i, &s);
        r[i] = game_ended(&s, players[i], totals + 2 * i);
    }
}
void or_canonical(const uint64_t* w, const int32_t* players, uint64_t* out, int n) {
    for (int i = 0; i < n; i++) {
        st_t s, o;
        unpack(w + 8 * i, &s);
        canonical(&s, players[i], &o);
        pack(&o, out + 8 * i);
    }
}
void or_featurize(const uint64_t* w, float* x, int n) {
    for (int i = 0; i < n; i++) {
        st_t s;
        unpack(w + 8 * i, &s);
        featurize(&s, x + (size_t)FEAT * i);
    }
}
void or_init_board(uint64_t seed, const uint32_t* envs, uint64_t* ctr, uint64_t* out, int n) {
    for (int i = 0; i < n; i++) {
        stream_t rs = {seed, envs[i], ctr[i]};
        st_t b;
        memset(&b, 0, sizeof(b));
        b.round = 1;
        roll_five(&rs, b.A); b.hasA = 1;
        roll_five(&rs, b.B); b.hasB = 1;
        pack(&b, out + 8 * i);
        ctr[i] = rs.ctr;
    }
}
void or_key_hash_batch(const uint64_t* w, uint64_t* out, int n) {
    for (int i = 0; i < n; i++) out[i] = or_key_hash(w + 8 * i);
}
void or_hash_prior(const uint64_t* w, float* pi, float* v, int n) {
    for (int i = 0; i < n; i++) hash_prior(w + 8 * i, pi + (size_t)ASIZE * i, v + i);
}
void or_net_predict(void* net, const uint64_t* w, float* pi, float* v, int n) {
#pragma omp parallel for schedule(dynamic, 16)
    for (int i = 0; i < n; i++) {
        st_t s;
        float x[FEAT];
        unpack(w + 8 * i, &s);
        featurize(&s, x);
        net_forward((const net_t*)net, x, pi + (size_t)ASIZE * i, v + i);
    }
}
void or_net_forward_x(void* net, const float* x, float* pi, float* v, int n) {
    for (int i = 0; i < n; i++) net_forward((const net_t*)net, x + (size_t)FEAT * i, pi + (size_t)ASIZE * i, v + i);
}
void or_draws(uint64_t seed, uint32_t env, uint64_t ctr0, uint64_t* out, int n) {
    for (int i = 0; i < n; i++) out[i] = or_draw64(seed, env, ctr0 + (uint64_t)i);
}

/* Self-play of n independent games (env ids envs[i]).  Output arrays are per env with
 * stride max_moves; any may be NULL.  mode: 0 hash prior, 1 mlp (net), 2 replay
 * (rpi/rv/rn per env: pointers into caller arrays of rn[i] predictions).  Runs the
 * games in parallel with OpenMP when threads > 1. */
int or_selfplay(int n, const uint32_t* envs, uint64_t seed, int sims, double cpuct, int temp_threshold,
                int max_moves, int mode, void* net, const float* const* rpi, const float* const* rv,
                const int64_t* rn, uint64_t* canon, int32_t* mv, uint64_t* ctr, int32_t* counts,
                double* values, int64_t* stats, uint64_t* final_state, int threads) {
    init_comb();
    ep_cfg_t cfg = {sims, temp_threshold, max_moves, cpuct, mode};
    int nerr = 0;
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads > 0 ? threads : 1) reduction(+ : nerr)
    for (int i = 0; i < n; i++) {
        pred_t pr;
        memset(&pr, 0, sizeof(pr));
        pr.mode = mode;
        pr.net = (const net_t*)net;
        if (mode == 2) { pr.rpi = rpi[i]; pr.rv = rv[i]; pr.rn = rn[i]; }
        ep_out_t o;
        o.canon = canon ? canon + (size_t)8 * max_moves * i : NULL;
        o.mv = mv ? mv + (size_t)8 * max_moves * i : NULL;
        o.ctr = ctr ? ctr + (size_t)2 * max_moves * i : NULL;
        o.counts = counts ? counts + (size_t)ASIZE * max_moves * i : NULL;
        o.values = values ? values + (size_t)max_moves * i : NULL;
        o.stats = stats ? stats + (size_t)8 * i : NULL;
        o.final_state = final_state ? final_state + (size_t)8 * i : NULL;
        if (run_episode(&cfg, &pr, seed, envs[i], &o)) nerr++;
    }
    return nerr;
}

int or_arena(int n, const uint32_t* envs, const int32_t* agent_seat, int agent_kind, int opp_kind, uint64_t seed,
             int sims, double cpuct, int max_moves, int mode, void* net, const float* const* rpi, const float* const* rv,
             const int64_t* rn, double* result, int32_t* totals, int32_t* actions, int64_t* stats,
             uint64_t* final_state, int threads) {
    init_comb();
    ep_cfg_t cfg = {sims, 0, max_moves, cpuct, mode};
    int nerr = 0;
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads > 0 ? threads : 1) reduction(+ : nerr)
    for (int i = 0; i < n; i++) {
        pred_t pr;
        memset(&pr, 0, sizeof(pr));
        pr.mode = mode;
        pr.net = (const net_t*)net;
        if (mode == 2) { pr.rpi = rpi[i]; pr.rv = rv[i]; pr.rn = rn[i]; }
        if (run_arena(&cfg, &pr, NULL, seed, envs[i], agent_seat[i], agent_kind, opp_kind, 0, NULL, result + i,
                      totals + 2 * i, actions ? actions + (size_t)max_moves * i : NULL, stats ? stats + 8 * i : NULL,
                      final_state ? final_state + 8 * i : NULL))
            nerr++;
    }
    return nerr;
}

/* The gating arena of Coach.learn (Coach.py:117-139): MCTS (temp 0, net) in seat agent_seat[i]
 * against MCTS (temp 0, net2), each with its own tree.  mode 2 replays ONE prediction log per game
 * (both seats' expansions in call order).  shared = 1 plays the n games in order with the two
 * trees kept across games, as the reference's pmcts / nmcts live across playGames (single thread);
 * 0: fresh trees per game (the engine's semantics, parallel). */
int or_arena_dual(int n, const uint32_t* envs, const int32_t* agent_seat, uint64_t seed, int sims, double cpuct,
                  int max_moves, int mode, void* net, void* net2, const float* const* rpi, const float* const* rv,
                  const int64_t* rn, int shared, double* result, int32_t* totals, int32_t* actions, int64_t* stats,
                  uint64_t* final_state, int threads) {
    init_comb();
    ep_cfg_t cfg = {sims, 0, max_moves, cpuct, mode};
    int nerr = 0;
    if (shared) {
        mcts_t m[2];
        memset(m, 0, sizeof(m));
        tree_init(&m[0].tree);
        tree_init(&m[1].tree);
        pred_t pr, pr2;
        memset(&pr, 0, sizeof(pr));
        memset(&pr2, 0, sizeof(pr2));
        pr.mode = pr2.mode = mode;
        pr.net = (const net_t*)net;
        pr2.net = (const net_t*)(net2 ? net2 : net);
        for (int i = 0; i < n; i++) {
            if (mode == 2) { pr.rpi = rpi[i]; pr.rv = rv[i]; pr.rn = rn[i]; pr.ri = 0; }
            if (run_arena(&cfg, &pr, mode == 2 ? &pr : &pr2, seed, envs[i], agent_seat[i], PK_MCTS, PK_MCTS, 1, m,
                          result + i, totals + 2 * i, actions ? actions + (size_t)max_moves * i : NULL,
                          stats ? stats + 8 * i : NULL, final_state ? final_state + 8 * i : NULL))
                nerr++;
        }
        tree_free(&m[0].tree);
        tree_free(&m[1].tree);
        return nerr;
    }
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads > 0 ? threads : 1) reduction(+ : nerr)
    for (int i = 0; i < n; i++) {
        pred_t pr, pr2;
        memset(&pr, 0, sizeof(pr));
        memset(&pr2, 0, sizeof(pr2));
        pr.mode = pr2.mode = mode;
        pr.net = (const net_t*)net;
        pr2.net = (const net_t*)(net2 ? net2 : net);
        if (mode == 2) { pr.rpi = rpi[i]; pr.rv = rv[i]; pr.rn = rn[i]; }
        if (run_arena(&cfg, &pr, mode == 2 ? &pr : &pr2, seed, envs[i], agent_seat[i], PK_MCTS, PK_MCTS, 1, NULL,
                      result + i, totals + 2 * i, actions ? actions + (size_t)max_moves * i : NULL,
                      stats ? stats + 8 * i : NULL, final_state ? final_state + 8 * i : NULL))
            nerr++;
    }
    return nerr;
}
