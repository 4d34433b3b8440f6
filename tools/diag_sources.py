"""Diagnostic builds (not the product): writes a copy of the kernel sources with measurement hooks
inserted at anchor lines, so the production sources carry none of them.

  python tools/diag_sources.py OUT_DIR     -> OUT_DIR/csrc (the sources with the hooks)

The hooks, each active only under its define (tools/variant_lib.sh NAME -DYK_...):
  YK_SEL_TIMING  per-game s_memtime accumulators of the descent's and the expansion's phases
                 (g_sel[e][16], read by yk_diag_select; tools/diag_select.py)
  YK_XSPAN       per-game start / end stamps of 16 sampled k_expand_backup launches
                 (yk_diag_xspan; tools/diag_xspan.py)
  YK_TIMING      per-phase stamps of k_forward's wave 0 and per-wave stamps of one trunk layer's
                 ring waits, A-fragment reads and MFMA groups (g_tstamp, tools/trunk_ablate.cpp)
  YK_AMP_TIMING  per-wave stamps of residual block 2 in the AMP train forward / backward
                 (k_amp_fwd / k_amp_bwd phases; yk_diag_amp_ts, tools/diag_amp.py)
Every anchor must match exactly once; a source change that moves one fails loudly here."""
import os
import re
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "nypc-yacht-auction_amd", "csrc")

ENGINE_GLOBALS = r'''
// ---- diagnostic hooks (tools/diag_sources.py) ----
#ifdef YK_SEL_TIMING
__device__ unsigned long long g_sel[16384 * 16];
#define SEL_T0(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define SEL_ACC(k, t0) \
    if (lane == 0) g_sel[(long)e * 16 + (k)] += __builtin_amdgcn_s_memtime() - (t0)
#define SEL_ADD(k, x) \
    if (lane == 0) g_sel[(long)e * 16 + (k)] += (unsigned long long)(x)
#else
#define SEL_T0(v)
#define SEL_ACC(k, t0)
#define SEL_ADD(k, x)
#endif
#ifdef YK_XSPAN
constexpr int XS_SAMPLES = 16, XS_GAMES = 4096;
__device__ unsigned long long g_xs[XS_SAMPLES][XS_GAMES][8];
__device__ int g_xs_slot = -1;
#endif
'''

XSPAN_BEGIN = r'''#ifdef YK_XSPAN
    const int xs = g_xs_slot;
    const unsigned long long xs0 = __builtin_amdgcn_s_memtime(), xr0 = __builtin_amdgcn_s_memrealtime();
    const uint32_t xs_v = d.leaf_flag[e] ? (uint32_t)valid_info(ld_state(d.leaf_state + e), 1).V : 0xFFFFFFFFu;
#endif
#ifdef YK_SEL_TIMING
    const unsigned long long t_ex = __builtin_amdgcn_s_memtime();
#endif
'''
XSPAN_MID = r'''#ifdef YK_XSPAN
    const unsigned long long xs1 = __builtin_amdgcn_s_memtime();
#endif
#ifdef YK_SEL_TIMING
    if (lane == 0) g_sel[(long)e * 16 + 6] += __builtin_amdgcn_s_memtime() - t_ex;
#endif
'''
XSPAN_END = r'''#ifdef YK_XSPAN
    if (xs >= 0 && xs < XS_SAMPLES && e < XS_GAMES && lane == 0) {
        const unsigned long long xs2 = __builtin_amdgcn_s_memtime(), xr2 = __builtin_amdgcn_s_memrealtime();
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
        const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
        unsigned long long* o = g_xs[xs][e];
        o[0] = xs0;
        o[1] = xs1;
        o[2] = xs2;
        o[3] = xs_v;
        o[4] = d.path_len[e];
        o[5] = ((unsigned long long)xcc << 32) | hw;
        o[6] = xr0;
        o[7] = xr2;
    }
#endif
'''
XSPAN_HOST = r'''#ifdef YK_XSPAN
            {
                static long xs_launch = 0;
                const long q = xs_launch++;
                const int slot = (q % 300 == 150 && q / 300 < XS_SAMPLES) ? (int)(q / 300) : -1;
                YK_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_xs_slot), &slot, sizeof(int), 0, hipMemcpyHostToDevice, st[g]));
                YK_HIP(hipStreamSynchronize(st[g]));
            }
#endif
'''
ENGINE_EXPORTS = r'''#ifdef YK_XSPAN
int yk_diag_xspan(uint64_t* out) {  // HOST out[16][4096][8]
    YK_HIP(hipDeviceSynchronize());
    YK_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_xs), sizeof(uint64_t) * XS_SAMPLES * XS_GAMES * 8));
    return YK_OK;
}
#endif
#ifdef YK_SEL_TIMING
int yk_diag_select(uint64_t* out, int n) {  // HOST out[n][16]; resets the accumulators
    YK_HIP(hipDeviceSynchronize());
    YK_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sel), sizeof(uint64_t) * 16 * (size_t)n));
    std::vector<uint64_t> z((size_t)16 * n, 0);
    YK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_sel), z.data(), sizeof(uint64_t) * z.size()));
    return YK_OK;
}
#endif
'''

# (anchor regex, 'before' | 'after', text).  Slots of g_sel: 0 lookup, 1 UCB scan (below the root
# or the root's full scan), 2 step + canonical, 3 whole descent, 4 levels, 5 entries scanned, 6 expand
# + backup, 8-10 expand phases, 12 backup, 13 the root's incremental scan (root_scan), 14 its entries
ENGINE = [
    (r"^constexpr uint32_t RV_OFF = .*\n", "after", ENGINE_GLOBALS),
    (r"^    PyV res\{0\.0, T_INT\};\n    // the root's pick", "before_line2", "    SEL_T0(t_all);\n"),
    (r"^        if \(rc\.x != 0 && rc1\.z != RV_OFF\) \{  // k_root_sort ran this move.*\n", "after", "            SEL_T0(t_rs);\n            const uint64_t sc0 = scanned;\n"),
    (r"^            pre = pre_bj != -1;\n", "after", "            SEL_ACC(13, t_rs);\n            SEL_ADD(14, scanned - sc0);\n"),
    (r"^        if \(known >= 0\) \{  // the cached child.*\n", "before", "        SEL_T0(t_lv);\n"),
    (r"^        if \(V == 0\) \{  // no valid action: MCTS.py:141-147.*\n", "before", "        SEL_ACC(0, t_lv);\n        SEL_T0(t_sc);\n"),
    (r"^        const int bj = bj_out;\n", "after", "        SEL_ACC(1, t_sc);\n        SEL_ADD(4, 1);\n        SEL_ADD(5, V);\n        SEL_T0(t_st);\n"),
    (r"^        s = canonical\(s, np\);  // MCTS.py:150\n", "after", "        SEL_ACC(2, t_st);\n"),
    (r"^        d\.gstats\[\(long\)e \* GST \+ 8\] \+= gathered;\n    \}\n\}\n", "before_last_brace", "    SEL_ACC(3, t_all);\n"),
    (r"^    if \(d\.done\[e\]\) return;\n    expand_backup_game\(d, e, lane\);\n", "replace",
     "    if (d.done[e]) return;\n" + XSPAN_BEGIN + "    expand_backup_game(d, e, lane);\n" + XSPAN_MID),
    (r"^        select_game\(d, e, lane, env_ids, ctr_arr\);\n    \}\n\}\n\n__device__ __forceinline__ void expand_backup_game",
     "replace_fn", None),
    (r"^        // ---- prior, Ps \* valids \(MCTS.py:88\)", "before", "        SEL_T0(t_x0);\n"),
    (r"^        // numpy pairwise_sum on the leaf:", "before", "        SEL_ACC(8, t_x0);\n        SEL_T0(t_x1);\n"),
    (r"^        // ---- allocate \+ write P over the compact valid set", "before", "        SEL_ACC(9, t_x1);\n        SEL_T0(t_x2);\n"),
    (r"^        res = PyV\{-\(double\)v, T_F32\};  // return -v", "before", "        SEL_ACC(10, t_x2);\n"),
    (r"^    // ---- backup \(MCTS.py:154-164\)", "before", "    SEL_T0(t_bk);\n"),
    (r"^            if \(timed\) prof_mark\(eng, g, KC_EXPAND, st\[g\]\);\n", "after", XSPAN_HOST),
    (r"^int yk_engine_create\(yk_engine_t\*\* out", "before", ENGINE_EXPORTS),
]


FWD_GLOBALS = r'''
// ---- diagnostic hooks (tools/diag_sources.py) ----
#ifdef YK_TIMING
constexpr int TS_STRIDE = 48;  // stamp slots per workgroup
__device__ unsigned long long g_tstamp[4096 * TS_STRIDE];
__device__ unsigned long long g_wstamp[4096 * 16 * 8];  // [workgroup][wave][event] of block 2
#define TSTAMP(i) \
    if (threadIdx.x == 0) g_tstamp[blockIdx.x * TS_STRIDE + (i)] = __builtin_amdgcn_s_memtime()
#define WSTAMP(i) \
    if ((threadIdx.x & 63) == 0) g_tstamp[blockIdx.x * TS_STRIDE + (i) + (threadIdx.x >> 6)] = __builtin_amdgcn_s_memtime()
#define LSTAMP(k) \
    if ((threadIdx.x & 63) == 0) g_wstamp[(blockIdx.x * 16 + (threadIdx.x >> 6)) * 8 + (k)] = __builtin_amdgcn_s_memtime()
extern "C" int yk_diag_fwd_ts(void* dst, int nwg) {  // the last launch's stamps of workgroups 0 .. nwg-1
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_tstamp), sizeof(unsigned long long) * TS_STRIDE * nwg) == hipSuccess ? 0 : -2;
}
// every launch's stamps, summed relative to each workgroup's start (slot 47: workgroups summed)
__device__ unsigned long long g_tacc[TS_STRIDE];
#define TACC()                                                                                      \
    if (threadIdx.x == 0) {                                                                         \
        const unsigned long long* ts = g_tstamp + blockIdx.x * TS_STRIDE;                           \
        for (int i = 1; i < TS_STRIDE - 1; i++) atomicAdd(&g_tacc[i], ts[i] - ts[0]);              \
        atomicAdd(&g_tacc[TS_STRIDE - 1], 1ull);                                                   \
    }
extern "C" int yk_diag_fwd_tacc(void* dst, int reset) {
    if (reset) {
        static const unsigned long long z[TS_STRIDE] = {};
        return hipMemcpyToSymbol(HIP_SYMBOL(g_tacc), z, sizeof(z)) == hipSuccess ? 0 : -2;
    }
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_tacc), sizeof(unsigned long long) * TS_STRIDE) == hipSuccess ? 0 : -2;
}
#else
#define TSTAMP(i)
#define WSTAMP(i)
#define LSTAMP(k)
#define TACC()
#endif
'''

# k_forward's wave-0 phase stamps (slots as tools/trunk_ablate.cpp reads them) and, for residual
# block 2, each wave's fc1 GEMM start (LSTAMP 0) / end (1), accumulators stored (2), the barrier
# passed (3), the row pass done (4), the next barrier passed = fc2 start (5), fc2 end (6)
FWD = [
    (r"^constexpr int ROWS = 16;.*\n", "after", FWD_GLOBALS),
    (r"^    const int c0 = lane \* VPL;\n", "after", "    TSTAMP(0);\n"),
    # the prologue (slots 32-36, 38): static vectors in LDS, the weight loads issued, features
    # written, the input barrier, the input GEMM done, its barrier passed; block 0's tile-list build (39 -> 37)
    (r"^        reinterpret_cast<float4\*>\(VS\)\[tid \+ NTH \* k\] = vsv\[k\];.*\n", "after", "    TSTAMP(32);\n"),
    (r"^    if \(tid < TMW\) UM\[tid\] = 0u;\n    if \(tid == 0\) VHC = 0u;\n    lds_barrier\(\);\n", "around", ("    TSTAMP(33);\n", "    TSTAMP(34);\n")),
    (r"^    __builtin_amdgcn_sched_barrier\(0\);  // the first layer streams in under the featurize / input phase\n", "after",
     "    TSTAMP(38);\n"),
    (r"^    lds_barrier\(\);  // T complete; every wave is done reading the feature planes\n", "around",
     ("    TSTAMP(35);\n", "    TSTAMP(36);\n")),
    (r"^        if \(b == 0 && wave < 4\) build_tiles\(wave\);.*\n", "around", ("        if (b == 0) TSTAMP(39);\n", "        if (b == 0) TSTAMP(37);\n")),
    (r"^        if \(w\) atomicOr\(&UM\[lane\], w\);\n    \}\n", "after", "    TSTAMP(1);\n"),
    (r"^    lds_barrier\(\);\n\n    // ResidualBlock x NB", "before_line2", "    TSTAMP(2);\n"),
    (r"^        if \(gw\) mma_ring<PL, H, NT, RW, N1, DEF>.*\n", "around",
     ("        if (b == 2) LSTAMP(0);\n", "        if (b == 2) { LSTAMP(1); TSTAMP(16); }\n")),
    (r"^        lds_barrier\(\);  // T complete; every wave is done reading x's planes\n", "around",
     ("        if (b == 2) LSTAMP(2);\n", "        if (b == 2) { LSTAMP(3); TSTAMP(17); }\n")),
    (r"^        lds_barrier\(\);\n        if \(gw\) \{\n            // \(the last block: v_head", "around_line1",
     ("        if (b == 2) LSTAMP(4);\n", "        if (b == 2) { LSTAMP(5); TSTAMP(18); }\n")),
    (r"^            else mma_ring<PL, H, NT, RW, N2, DEF, V>.*\n        \}\n", "after", "        if (b == 2) { LSTAMP(6); TSTAMP(19); }\n"),
    (r"^        lds_barrier\(\);  // T complete; every wave is done reading h's planes\n", "after", "        if (b == 2) TSTAMP(21);\n"),
    (r"^        lds_barrier\(\);\n    \};\n    for \(int b = 0; b \+ 1 < net.NB", "after_line1", "        if (b < 6) TSTAMP(3 + b);\n"),
    (r"^    lds_barrier\(\);\n    // The policy head over all real tiles", "after_line1", "    TSTAMP(9);\n"),
    (r"^        for \(int t = 0; t < PC; t\+\+\) tcur\[t\] = tnxt\[t\];\n", "after",
     "        if (c == 1 || c == 3) TSTAMP(10 + (c >> 1));\n        if (c == 5) TSTAMP(12);\n"),
    (r"^    float sm\[4\], ss\[4\];  // running max", "before", "    TSTAMP(40);\n"),
    (r"^    chunk_tiles\(0, tcur\);\n", "around", ("    TSTAMP(43);\n", "    TSTAMP(41);\n")),
    (r"^            for \(int t = 0; t < PC; t\+\+\) pring\[ks\]\[t\] = ld_w2<PL>\(net.w_pi, KS, tcur\[t\], ks, lane\);\n        __builtin_amdgcn_sched_barrier\(0\);\n",
     "after", "        TSTAMP(42);\n"),
    (r"^#undef YK_PI_CHUNK\n", "after", "    TSTAMP(14);\n    WSTAMP(24);\n"),
    (r"^        for \(int j = 0; j < 4; j\+\+\) SS\[wave \* ROWS.*\n    \}\n", "after", "    TSTAMP(23);\n"),
    (r"^    lds_barrier\(\);  // every wave is done with v_head.2", "around_line1", ("    TSTAMP(44);\n", "    TSTAMP(45);\n")),
    (r"^            if \(lane == 0 && part == 0 && row < n.*\n        \}\n    \}\n", "after", "    TSTAMP(46);\n"),
    (r"^            mlse\[\(long\)part \* mstride.*\n        \}\n    \}\n", "after", "    TSTAMP(15);\n    TACC();\n"),
]


AMP_GLOBALS = r'''
// ---- diagnostic hooks (tools/diag_sources.py) ----
#ifdef YK_AMP_TIMING
__device__ unsigned long long g_amp_ts[2][64][8][16];  // [fwd, bwd][tile][wave][half * 8 + k]
#define AMP_STAMP(kk, k)                                                                      \
    if (b == 2 && (threadIdx.x & 63) == 0 && blockIdx.x < 64)                                 \
    g_amp_ts[kk][blockIdx.x][threadIdx.x >> 6][half * 8 + (k)] = __builtin_amdgcn_s_memtime()
extern "C" int yk_diag_amp_ts(void* dst) {
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_amp_ts), sizeof(g_amp_ts)) == hipSuccess ? 0 : -2;
}
#else
#define AMP_STAMP(kk, k)
#endif
'''
# k_amp_fwd, block 2, per half: 0 before the GEMM, 1 GEMM + accumulator store done, 2 the T-layout
# store of waves 0-3 done, 3 the barrier passed, 4 the row pass done, 5 the next barrier passed
AMP = [
    (r"^constexpr int SQ_BLOCKS = 1024;\n", "after", AMP_GLOBALS),
    (r"^            const float4\* nxt = half == 0 \? d.w2f.*\n            const float4\* dsrc.*\n            if \(gw\) \{\n"
     r"                gemm_ring<KS, NT, RW, FDEF>\(Pa, SA, ring, acc, cur, nxt, nt0\);\n"
     r"                store_acc<NT>\(Ts, LD, nt0, acc\);\n            \}\n", "around",
     ("            AMP_STAMP(0, 0);\n", "            AMP_STAMP(0, 1);\n")),
    (r"^                              zero_rest, 256\);\n", "after", "            AMP_STAMP(0, 2);\n"),
    (r"^            lds_barrier\(\);\n            float\* U = ", "after_line1", "            AMP_STAMP(0, 3);\n"),
    (r"^            lds_barrier\(\);\n        \}\n    \}\n\n    // the heads' LayerNorms", "around_line1",
     ("            AMP_STAMP(0, 4);\n", "            AMP_STAMP(0, 5);\n")),
    # k_amp_bwd, block 2, per half: 0 row pass start, 1 its end, 2 the barrier passed, 3 column
    # partials flushed, 4 T-layout store done, 5 next row's operands issued, 6 GEMM + store done,
    # 7 the barrier passed
    (r"^            // row pass: \(half 1\) dL2 = dh; \(half 0\) dL1", "before", "            AMP_STAMP(1, 0);\n"),
    (r"^            lds_barrier\(\);\n            flush_gbb<H>", "around_line1",
     ("            AMP_STAMP(1, 1);\n", "            AMP_STAMP(1, 2);\n")),
    (r"^            flush_gbb<H>\(d, CP, tile, CV_BLK.*\n", "after", "            AMP_STAMP(1, 3);\n"),
    (r"^            write_tl<TRV>\(Pa, SA, 0, H, \(half == 0 \? d.du1T.*\n", "after", "            AMP_STAMP(1, 4);\n"),
    (r"^            __builtin_amdgcn_sched_barrier\(0\);\n            const float4\* nxt = half == 1", "after_line1",
     "            AMP_STAMP(1, 5);\n"),
    (r"^            const float4\* nxt = half == 1 \? d.w1t.*\n            if \(gw\) \{\n"
     r"                gemm_ring<KS, NT, RW, BDEF>\(Pa, SA, ring, acc, cur, nxt, nt0\);\n"
     r"                store_acc<NT>\(Ts, LD, nt0, acc\);\n            \}\n", "after", "            AMP_STAMP(1, 6);\n"),
    (r"^            lds_barrier\(\);\n            if \(half == 0\) \{  // residual", "after_line1",
     "            AMP_STAMP(1, 7);\n"),
]


def apply(text, rules, name):
    for pat, where, ins in rules:
        ms = list(re.finditer(pat, text, flags=re.M))
        if len(ms) != 1:
            raise SystemExit(f"{name}: anchor {pat!r} matched {len(ms)} times")
        m = ms[0]
        if where == "after":
            text = text[:m.end()] + ins + text[m.end():]
        elif where == "before":
            text = text[:m.start()] + ins + text[m.start():]
        elif where == "before_line2":  # before the second line of the match
            k = text.index("\n", m.start()) + 1
            text = text[:k] + ins + text[k:]
        elif where == "before_last_brace":  # before the match's closing "}\n" (end of the function)
            k = m.end() - 2
            text = text[:k] + ins + text[k:]
        elif where == "around":
            text = text[:m.start()] + ins[0] + m.group(0) + ins[1] + text[m.end():]
        elif where in ("around_line1", "after_line1"):  # around / after the first line of the match
            k = text.index("\n", m.start()) + 1
            if where == "around_line1":
                text = text[:m.start()] + ins[0] + text[m.start():k] + ins[1] + text[k:]
            else:
                text = text[:k] + ins + text[k:]
        elif where == "replace":
            text = text[:m.start()] + ins + text[m.end():]
        elif where == "replace_fn":  # k_expand_backup's tail: the span stamps after the descent
            seg = m.group(0)
            text = text[:m.start()] + seg.replace("    }\n}\n\n__device__", "    }\n" + XSPAN_END + "}\n\n__device__", 1) + \
                text[m.end():]
    return text


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "/tmp/yk_hooks"
    dst = os.path.join(out, "csrc")
    if os.path.exists(dst):
        shutil.rmtree(dst)
    shutil.copytree(SRC, dst)
    p = os.path.join(dst, "yk_engine.hip")
    with open(p) as f:
        text = f.read()
    text = apply(text, ENGINE, "yk_engine.hip")
    # the backup's end stamp: the last statement of expand_backup_game
    m = re.search(r"(    \}\n\}\n\n// The root's P order for root_scan)", text)
    if not m:
        raise SystemExit("yk_engine.hip: end of expand_backup_game not found")
    text = text[:m.start()] + "    }\n    SEL_ACC(12, t_bk);\n}\n\n// The root's P order for root_scan" + text[m.end():]
    with open(p, "w") as f:
        f.write(text)
    p = os.path.join(dst, "yk_fwd.h")
    with open(p) as f:
        text = f.read()
    text = apply(text, FWD, "yk_fwd.h")
    with open(p, "w") as f:
        f.write(text)
    p = os.path.join(dst, "yk_train_amp.hip")
    with open(p) as f:
        text = f.read()
    text = apply(text, AMP, "yk_train_amp.hip")
    with open(p, "w") as f:
        f.write(text)
    print(dst)


if __name__ == "__main__":
    main()
