// Checks yk::xlane<O> (DPP / permlane-swap exchanges, yk_common.h) against __shfl_xor for every
// offset, for 32- and 64-bit values, and the butterfly sums / argmax built on it, on random waves.
// GPU box: hipcc -O3 --offload-arch=gfx950 -std=c++17 -Iinclude -Inypc-yacht-auction_amd/csrc
//          tools/xlane_check.hip -o /tmp/xlane_check && /tmp/xlane_check
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "yk_common.h"

using namespace yk;

constexpr int NW = 256;  // waves checked
constexpr int NCHK = 16;

__global__ void k_check(const uint32_t* in, const double* ind, uint32_t* bad) {
    const int w = blockIdx.x, lane = threadIdx.x;
    const uint32_t v = in[w * 64 + lane];
    const double d = ind[w * 64 + lane];
    uint32_t b = 0;
    b |= (xlane_u<1>(v) != (uint32_t)__shfl_xor((int)v, 1, 64)) << 0;
    b |= (xlane_u<2>(v) != (uint32_t)__shfl_xor((int)v, 2, 64)) << 1;
    b |= (xlane_u<4>(v) != (uint32_t)__shfl_xor((int)v, 4, 64)) << 2;
    b |= (xlane_u<8>(v) != (uint32_t)__shfl_xor((int)v, 8, 64)) << 3;
    b |= (xlane_u<16>(v) != (uint32_t)__shfl_xor((int)v, 16, 64)) << 4;
    b |= (xlane_u<32>(v) != (uint32_t)__shfl_xor((int)v, 32, 64)) << 5;
    b |= (xlane<16>(d) != __shfl_xor(d, 16, 64)) << 6;
    b |= (xlane<1>(d) != __shfl_xor(d, 1, 64)) << 7;
    // the butterfly sum against the __shfl_xor loop, bitwise
    const float f = __builtin_bit_cast(float, (v & 0x807FFFFFu) | 0x3F000000u);  // values in +-[0.5, 1)
    float r = f;
    for (int o = 32; o >= 1; o >>= 1) r += __shfl_xor(r, o, 64);
    b |= (__builtin_bit_cast(uint32_t, xlane_sum(f)) != __builtin_bit_cast(uint32_t, r)) << 8;
    double rd = d;
    for (int o = 32; o >= 1; o >>= 1) rd += __shfl_xor(rd, o, 64);
    b |= (__builtin_bit_cast(uint64_t, xlane_sum(d)) != __builtin_bit_cast(uint64_t, rd)) << 9;
    // argmax with the lowest index on ties (small value range: many ties)
    float best = (float)(v % 7u);
    int bj = (int)((v >> 8) % 1000u);
    float best2 = best;
    int bj2 = bj;
    wave_argmax_step(best, bj);
    for (int o = 32; o >= 1; o >>= 1) {
        const float ob = __shfl_xor(best2, o, 64);
        const int oj = __shfl_xor(bj2, o, 64);
        if (ob > best2 || (ob == best2 && oj < bj2)) {
            best2 = ob;
            bj2 = oj;
        }
    }
    b |= (best != best2 || bj != bj2) << 10;
    // the even lane's value, and lane_val
    b |= (dpp_mov<0xA0>(v) != (uint32_t)__shfl((int)v, lane & ~1, 64)) << 11;
    const int f0 = (int)(in[w * 64] & 63u);
    b |= (__builtin_bit_cast(uint32_t, lane_val(f, f0)) != __builtin_bit_cast(uint32_t, __shfl(f, f0, 64))) << 12;
    bad[w * 64 + lane] = b;
}

int main() {
    std::vector<uint32_t> h(NW * 64);
    std::vector<double> hd(NW * 64);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (int i = 0; i < NW * 64; i++) {
        x ^= x << 13, x ^= x >> 7, x ^= x << 17;
        h[i] = (uint32_t)x;
        hd[i] = (double)(int64_t)(x >> 11) * 0x1p-40;
    }
    uint32_t *din, *dbad;
    double* dd;
    hipMalloc(&din, NW * 64 * 4);
    hipMalloc(&dd, NW * 64 * 8);
    hipMalloc(&dbad, NW * 64 * 4);
    hipMemcpy(din, h.data(), NW * 64 * 4, hipMemcpyHostToDevice);
    hipMemcpy(dd, hd.data(), NW * 64 * 8, hipMemcpyHostToDevice);
    k_check<<<NW, 64>>>(din, dd, dbad);
    std::vector<uint32_t> bad(NW * 64);
    if (hipMemcpy(bad.data(), dbad, NW * 64 * 4, hipMemcpyDeviceToHost) != hipSuccess) {
        printf("xlane_check: HIP error\n");
        return 2;
    }
    int cnt[NCHK] = {};
    for (uint32_t b : bad)
        for (int k = 0; k < NCHK; k++) cnt[k] += (b >> k) & 1;
    const char* names[NCHK] = {"x1", "x2", "x4", "x8", "x16", "x32", "d16", "d1", "sum_f", "sum_d", "argmax", "even", "lane_val"};
    int tot = 0;
    for (int k = 0; k < 13; k++) {
        printf("%-8s mismatching lanes %d\n", names[k], cnt[k]);
        tot += cnt[k];
    }
    printf(tot ? "xlane_check: FAIL\n" : "xlane_check: ok (%d waves)\n", NW);
    return tot ? 1 : 0;
}
