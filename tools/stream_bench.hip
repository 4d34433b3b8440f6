// Diagnostic (not part of the product): how fast can ONE CU stream a weight set that every CU
// reads (the k_forward situation: 6.7 MB of f32 weights, L2/MALL-resident, 256 workgroups)?
//   mode 0: 8 waves, global_load_dwordx4 into registers, D loads in flight per wave
//   mode 1: 8 waves, global_load_lds_dwordx4 (LDS-DMA) into a per-wave LDS ring
//   mode 2: 4 of 8 waves, LDS-DMA
// usage: stream_bench [MB]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int NTHR = 512;
__device__ unsigned long long g_clk[4];
#define CLK_BEGIN unsigned long long c0_ = __builtin_amdgcn_s_memtime(), r0_ = __builtin_amdgcn_s_memrealtime();
#define CLK_END                                                                                    \
    if (blockIdx.x == 0 && threadIdx.x == 0) {                                                     \
        g_clk[0] = __builtin_amdgcn_s_memtime() - c0_;                                             \
        g_clk[1] = __builtin_amdgcn_s_memrealtime() - r0_;                                         \
    }

template <int D>
__global__ __launch_bounds__(NTHR) void k_vgpr(const float4* __restrict__ w, long n4, float* out) {
    CLK_BEGIN
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    const long per = n4 / 64;  // 1 KB chunks
    // wave w takes chunks w, w + 8, ...; rotate the start per workgroup
    for (long c0 = wave; c0 < per; c0 += 8 * D) {
        float4 v[D];
#pragma unroll
        for (int d = 0; d < D; d++) {
            const long c = c0 + 8 * d;
            v[d] = c < per ? w[c * 64 + lane] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int d = 0; d < D; d++) acc.x += v[d].x + v[d].y + v[d].z + v[d].w;
    }
    if (acc.x == 12345.f) out[blockIdx.x] = acc.x;
    CLK_END
}

template <int LW>
__global__ __launch_bounds__(NTHR) void k_glds(const float4* __restrict__ w, long n4, float* out) {
    CLK_BEGIN
    __shared__ __attribute__((aligned(16))) float ring[8][16][256];  // 8 waves x 16 slots x 1 KB = 128 KB
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (wave >= LW) return;
    const long per = n4 / 64;
    int slot = 0;
    for (long c = wave; c < per; c += LW) {
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(w + c * 64 + lane),
                                         (__attribute__((address_space(3))) void*)(&ring[wave][slot][0]),
                                         16, 0, 0);
        slot = (slot + 1) & 15;
        asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (ring[wave][lane & 15][lane] == 12345.f) out[blockIdx.x] = 1.f;
    CLK_END
}

// per-wave LDS-DMA ring feeding MFMA: R slots of 1 KB per wave; per fragment: wait for the
// oldest slot, ds_read_b128 it, 4 x v_mfma_f32_16x16x4_f32, refill the slot
typedef float floatx4 __attribute__((ext_vector_type(4)));
template <int R>
__global__ __launch_bounds__(NTHR) void k_glds_mfma(const float4* __restrict__ w, long n4, float* out) {
    CLK_BEGIN
    __shared__ __attribute__((aligned(16))) float ring[8][R][256];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const long per = n4 / 64 / 8;  // fragments per wave
    const float4* src = w + (long)wave * per * 64 + lane;
    typedef __attribute__((address_space(3))) void* lds_t;
#pragma unroll
    for (int r = 0; r < R; r++)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + (long)r * 64), (lds_t)(&ring[wave][r][0]), 16, 0, 0);
    floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
    const float a = (float)lane * 0.001f;
    int slot = 0;
    for (long f = 0; f < per; f++) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(R - 1) : "memory");
        const float4 b = *reinterpret_cast<const float4*>(&ring[wave][slot][lane * 4]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b.x, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b.y, acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b.z, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b.w, acc1, 0, 0, 0);
        const long g = f + R < per ? f + R : f;  // keep the count uniform at the tail
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + g * 64), (lds_t)(&ring[wave][slot][0]), 16, 0, 0);
        slot = slot + 1 == R ? 0 : slot + 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (acc0[0] + acc1[1] == 12345.f) out[blockIdx.x] = 1.f;
    CLK_END
}
// the same with the LDS reads pipelined: fragment f+1's ds_read is in flight while f's MFMAs run
template <int R>
__global__ __launch_bounds__(NTHR) void k_glds_mfma2(const float4* __restrict__ w, long n4, float* out) {
    CLK_BEGIN
    __shared__ __attribute__((aligned(16))) float ring[8][R][256];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const long per = n4 / 64 / 8;
    const float4* src = w + (long)wave * per * 64 + lane;
    typedef __attribute__((address_space(3))) void* lds_t;
#pragma unroll
    for (int r = 0; r < R; r++)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + (long)r * 64), (lds_t)(&ring[wave][r][0]), 16, 0, 0);
    floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
    const float a = (float)lane * 0.001f;
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(R - 1) : "memory");
    float4 b = *reinterpret_cast<const float4*>(&ring[wave][0][lane * 4]);
    int slot = 0;
    for (long f = 0; f < per; f++) {
        const int nslot = slot + 1 == R ? 0 : slot + 1;
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(R - 2) : "memory");  // fragment f+1 landed
        const float4 bn = *reinterpret_cast<const float4*>(&ring[wave][nslot][lane * 4]);
        asm volatile("s_waitcnt lgkmcnt(1)" ::: "memory");  // fragment f's read returned
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b.x, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b.y, acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b.z, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b.w, acc1, 0, 0, 0);
        const long g = f + R < per ? f + R : f;
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + g * 64), (lds_t)(&ring[wave][slot][0]), 16, 0, 0);
        b = bn;
        slot = nslot;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (acc0[0] + acc1[1] == 12345.f) out[blockIdx.x] = 1.f;
    CLK_END
}
// as k_glds_mfma2 with the LDS reads in inline asm: hipcc would otherwise put a vmcnt(0)
// (draining every DMA in flight) in front of each C++ LDS read; waits are explicit, and the
// lgkmcnt wait names the register it guards so the MFMA cannot move above it
__device__ __forceinline__ floatx4 ds_read16(const float* p) {
    floatx4 v;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"((uint32_t)(uintptr_t)p) : "memory");
    return v;
}
template <int R>
__global__ __launch_bounds__(NTHR) void k_glds_mfma3(const float4* __restrict__ w, long n4, float* out) {
    CLK_BEGIN
    __shared__ __attribute__((aligned(16))) float ring[8][R][256];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const long per = n4 / 64 / 8;
    const float4* src = w + (long)wave * per * 64 + lane;
    typedef __attribute__((address_space(3))) void* lds_t;
#pragma unroll
    for (int r = 0; r < R; r++)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + (long)r * 64), (lds_t)(&ring[wave][r][0]), 16, 0, 0);
    floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
    const float a = (float)lane * 0.001f;
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(R - 1) : "memory");
    floatx4 b0 = ds_read16(&ring[wave][0][lane * 4]), b1;
    int slot = 0;
    auto step = [&](long f, floatx4& cur, floatx4& nxt) {
        const int nslot = slot + 1 == R ? 0 : slot + 1;
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(R - 2) : "memory");
        nxt = ds_read16(&ring[wave][nslot][lane * 4]);
        asm volatile("s_waitcnt lgkmcnt(1)" : "+v"(cur) :: "memory");
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, cur[0], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, cur[1], acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, cur[2], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, cur[3], acc1, 0, 0, 0);
        const long g = f + R < per ? f + R : f;
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + g * 64), (lds_t)(&ring[wave][slot][0]), 16, 0, 0);
        slot = nslot;
    };
    for (long f = 0; f + 1 < per; f += 2) {
        step(f, b0, b1);
        step(f + 1, b1, b0);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    if (acc0[0] + acc1[1] == 12345.f) out[blockIdx.x] = 1.f;
    CLK_END
}
// the same MFMA count with the fragments from registers only (the MFMA floor)
__global__ __launch_bounds__(NTHR) void k_mfma_only(const float4* __restrict__ w, long n4, float* out) {
    CLK_BEGIN
    const int lane = threadIdx.x & 63;
    const long per = n4 / 64 / 8;
    floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
    const float a = (float)lane * 0.001f;
    float4 b = make_float4(a, a, a, a);
    for (long f = 0; f < per; f++) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b.x, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b.y, acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b.z, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b.w, acc1, 0, 0, 0);
    }
    if (acc0[0] + acc1[1] == 12345.f) out[blockIdx.x] = 1.f;
    CLK_END
}

// role split: waves 0-3 (one per SIMD) run all the MFMAs on register data (4 accumulators),
// waves 4-7 stream the weights by LDS-DMA and consume nothing (MFMA_ON / STREAM_ON select)
template <bool MFMA_ON, bool STREAM_ON, int PRIO = 0>
__global__ __launch_bounds__(NTHR) void k_split(const float4* __restrict__ w, long n4, float* out) {
    CLK_BEGIN
    __shared__ __attribute__((aligned(16))) float ring[4][16][256];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const long per = n4 / 64;  // fragments per CU
    if (wave < 4) {
        if (MFMA_ON) {
            floatx4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
            const float a = (float)lane * 0.001f;
            for (long f = 0; f < per / 4; f++) {
                c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, a, c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, a, c1, 0, 0, 0);
                c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, a, c2, 0, 0, 0);
                c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, a, c3, 0, 0, 0);
            }
            if (c0[0] + c1[1] + c2[2] + c3[3] == 12345.f) out[blockIdx.x] = 1.f;
        }
    } else if (STREAM_ON) {
        if (PRIO) __builtin_amdgcn_s_setprio(PRIO);
        const int lw = wave - 4;
        typedef __attribute__((address_space(3))) void* lds_t;
        int slot = 0;
        for (long c = lw; c < per; c += 4) {
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(w + c * 64 + lane), (lds_t)(&ring[lw][slot][0]),
                                             16, 0, 0);
            slot = (slot + 1) & 15;
            asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (ring[lw][lane & 15][lane] == 12345.f) out[blockIdx.x] = 1.f;
    }
    CLK_END
}

// role split variants: MODE 0 = MFMA waves + VGPR-load stream waves; MODE 1 = VALU-FMA waves
// + LDS-DMA stream waves; MODE 2 = VALU-FMA waves alone; MODE 3 = VALU-FMA waves + VGPR-load
// stream waves; MODE 4 = VGPR-load stream waves alone
template <int MODE>
__global__ __launch_bounds__(NTHR) void k_split2(const float4* __restrict__ w, long n4, float* out) {
    CLK_BEGIN
    __shared__ __attribute__((aligned(16))) float ring[4][16][256];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const long per = n4 / 64;
    if (wave < 4) {
        if (MODE == 4) {
        } else if (MODE == 0) {
            floatx4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
            const float a = (float)lane * 0.001f;
            for (long f = 0; f < per / 4; f++) {
                c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, a, c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, a, c1, 0, 0, 0);
                c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, a, c2, 0, 0, 0);
                c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, a, c3, 0, 0, 0);
            }
            if (c0[0] + c1[1] + c2[2] + c3[3] == 12345.f) out[blockIdx.x] = 1.f;
        } else {
            // the same FLOP as the MFMA waves: per fragment 4 MFMA = 8192 FLOP = 64 lanes x 64 FMA
            float x[16];
#pragma unroll
            for (int i = 0; i < 16; i++) x[i] = lane * 0.001f + i;
            const float a = lane * 0.5f, b = 0.999f;
            for (long f = 0; f < per / 4; f++) {
#pragma unroll
                for (int r = 0; r < 16; r++)
#pragma unroll
                    for (int i = 0; i < 16; i++) x[i] = fmaf(x[i], b, a);
            }
            float t = 0.f;
#pragma unroll
            for (int i = 0; i < 16; i++) t += x[i];
            if (t == 12345.f) out[blockIdx.x] = 1.f;
        }
    } else if (MODE == 0 || MODE == 3 || MODE == 4) {
        const int lw = wave - 4;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        constexpr int D = 12;
        float4 v[D];
#pragma unroll
        for (int d = 0; d < D; d++) v[d] = w[(long)(lw + 4 * d) * 64 + lane];
        for (long c = lw + 4 * D; c < per; c += 4 * D) {
#pragma unroll
            for (int d = 0; d < D; d++) {
                acc.x += v[d].x;
                const long cc = c + 4 * d;
                v[d] = w[(cc < per ? cc : 0) * 64 + lane];
            }
        }
#pragma unroll
        for (int d = 0; d < D; d++) acc.x += v[d].y;
        if (acc.x == 12345.f) out[blockIdx.x] = 1.f;
    } else if (MODE == 1) {
        const int lw = wave - 4;
        typedef __attribute__((address_space(3))) void* lds_t;
        int slot = 0;
        for (long c = lw; c < per; c += 4) {
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(w + c * 64 + lane), (lds_t)(&ring[lw][slot][0]),
                                             16, 0, 0);
            slot = (slot + 1) & 15;
            asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (ring[lw][lane & 15][lane] == 12345.f) out[blockIdx.x] = 1.f;
    }
    CLK_END
}

// f32-equivalent GEMM by a 2-term fp16 split (hi + lo * 2^-11): per 2 KB of weights (one
// 16-column x 32-deep slice: hi and lo planes) 3 x v_mfma_f32_16x16x32_f16, the weights
// streamed into a register ring of R slices per wave (the k_forward pattern)
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
template <int R>
__global__ __launch_bounds__(NTHR) void k_f16_ring(const float4* __restrict__ w, long n4, float* out) {
    CLK_BEGIN
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const long per = n4 / 64 / 8 / 2;  // 2-KB slices per wave
    const float4* src = w + (long)wave * per * 128 + lane;
    float4 ring[R][2];
#pragma unroll
    for (int r = 0; r < R; r++) {
        ring[r][0] = src[(long)r * 128];
        ring[r][1] = src[(long)r * 128 + 64];
    }
    floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
    half8 ah, al;
    for (int i = 0; i < 8; i++) {
        ah[i] = (_Float16)(lane * 0.01f + i);
        al[i] = (_Float16)(lane * 0.001f);
    }
    for (long f0 = 0; f0 < per; f0 += R) {
#pragma unroll
        for (int r = 0; r < R; r++) {
            const half8 wh = __builtin_bit_cast(half8, ring[r][0]);
            const half8 wl = __builtin_bit_cast(half8, ring[r][1]);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, wh, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, wl, acc1, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, wh, acc1, 0, 0, 0);
            const long g = f0 + r + R < per ? f0 + r + R : 0;
            ring[r][0] = src[g * 128];
            ring[r][1] = src[g * 128 + 64];
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    if (acc0[0] + acc1[1] == 12345.f) out[blockIdx.x] = 1.f;
    CLK_END
}
// k_f16_ring at 3 or 4 products per slice, with the workgroups of an XCD (blockIdx % 8) starting
// their walk through the weight set at DIV different offsets (DIV = 1: lock-step, every CU of the
// XCD reading the same lines together; DIV = 32: each CU of the XCD at its own place) - what a
// schedule without a global barrier does to the shared-read rate
template <int R, int NP, int DIV>
__global__ __launch_bounds__(NTHR) void k_f16_ring_rot(const float4* __restrict__ w, long n4, float* out) {
    CLK_BEGIN
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const long per = n4 / 64 / 8 / 2;  // 2-KB slices per wave
    const long off = (long)((blockIdx.x >> 3) % DIV) * (per / DIV);
    const float4* src = w + (long)wave * per * 128 + lane;
    float4 ring[R][2];
#pragma unroll
    for (int r = 0; r < R; r++) {
        const long g = (off + r) % per;
        ring[r][0] = src[g * 128];
        ring[r][1] = src[g * 128 + 64];
    }
    floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
    half8 ah, al;
    for (int i = 0; i < 8; i++) {
        ah[i] = (_Float16)(lane * 0.01f + i);
        al[i] = (_Float16)(lane * 0.001f);
    }
    for (long f0 = 0; f0 < per; f0 += R) {
#pragma unroll
        for (int r = 0; r < R; r++) {
            const half8 wh = __builtin_bit_cast(half8, ring[r][0]);
            const half8 wl = __builtin_bit_cast(half8, ring[r][1]);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, wh, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, wl, acc1, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, wh, acc1, 0, 0, 0);
            if constexpr (NP == 4) acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, wl, acc1, 0, 0, 0);
            const long g = (off + f0 + r + R) % per;
            ring[r][0] = src[g * 128];
            ring[r][1] = src[g * 128 + 64];
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    if (acc0[0] + acc1[1] == 12345.f) out[blockIdx.x] = 1.f;
    CLK_END
}
// the same MFMAs, no stream
__global__ __launch_bounds__(NTHR) void k_f16_only(const float4* __restrict__ w, long n4, float* out) {
    CLK_BEGIN
    const int lane = threadIdx.x & 63;
    const long per = n4 / 64 / 8 / 2;
    floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
    half8 ah, al;
    for (int i = 0; i < 8; i++) {
        ah[i] = (_Float16)(lane * 0.01f + i);
        al[i] = (_Float16)(lane * 0.001f);
    }
    for (long f = 0; f < per; f++) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, ah, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, al, acc1, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, ah, acc1, 0, 0, 0);
    }
    if (acc0[0] + acc1[1] == 12345.f) out[blockIdx.x] = 1.f;
    CLK_END
}

int main(int argc, char** argv) {
    const double MB = argc > 1 ? atof(argv[1]) : 6.7;
    const long n4 = (long)(MB * 1e6 / 16) / 64 * 64;
    float4* w;
    float* out;
    hipMalloc(&w, n4 * 16);
    hipMalloc(&out, 4096 * 4);
    hipMemset(w, 0, n4 * 16);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int it = 50;
    int G = 256;
    auto run = [&](const char* name, auto kern) {
        for (int i = 0; i < 5; i++) hipLaunchKernelGGL(kern, dim3(G), dim3(NTHR), 0, 0, w, n4, out);
        hipEventRecord(a);
        for (int i = 0; i < it; i++) hipLaunchKernelGGL(kern, dim3(G), dim3(NTHR), 0, 0, w, n4, out);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double us = 1000.0 * ms / it;
        unsigned long long clk[4];
        hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_clk), sizeof(clk));
        printf("G=%3d %-28s %8.2f us per launch  %6.1f GB/s per CU  %6.2f TB/s from L2  clock %.2f GHz\n", G, name, us,
               n4 * 16 / (us * 1e3), n4 * 16.0 * G / (us * 1e6), clk[1] ? 0.1 * clk[0] / clk[1] : 0.0);
    };
    if (argc > 2 && argv[2][0] == 'r') {  // desynchronised workgroups (schedule without a global barrier)
        for (int g : {256, 128}) {
            G = g;
            run("f16x3 ring R=8 lock-step", k_f16_ring_rot<8, 3, 1>);
            run("f16x3 ring R=8 4 offsets", k_f16_ring_rot<8, 3, 4>);
            run("f16x3 ring R=8 32 offsets", k_f16_ring_rot<8, 3, 32>);
            run("f16x4 ring R=8 lock-step", k_f16_ring_rot<8, 4, 1>);
            run("f16x4 ring R=8 32 offsets", k_f16_ring_rot<8, 4, 32>);
        }
        return 0;
    }
    if (argc > 2 && argv[2][0] == 'v') {  // vector-ALU waves beside a register-load stream
        run("split2: valu alone", k_split2<2>);
        run("split2: vgpr stream alone", k_split2<4>);
        run("split2: valu + vgpr stream", k_split2<3>);
        run("split2: valu + glds stream", k_split2<1>);
        run("split2: mfma + vgpr stream", k_split2<0>);
        run("split: mfma waves only", k_split<true, false>);
        return 0;
    }
    if (argc > 2) {  // grid sweep: is the per-CU rate of a shared weight set a per-CU or an L2-side limit?
        for (int g : {256, 192, 128, 96, 64, 32}) {
            G = g;
            run("vgpr  D=8", k_vgpr<8>);
            run("glds  8 waves", k_glds<8>);
            run("f16x2 mfma only", k_f16_only);
            run("f16x2 ring R=8", k_f16_ring<8>);
        }
        return 0;
    }
    run("vgpr  D=4", k_vgpr<4>);
    run("vgpr  D=8", k_vgpr<8>);
    run("vgpr  D=16", k_vgpr<16>);
    run("glds  8 waves", k_glds<8>);
    run("glds  4 waves", k_glds<4>);
    run("glds  2 waves", k_glds<2>);
    run("glds+mfma R=8", k_glds_mfma<8>);
    run("glds+mfma R=12", k_glds_mfma<12>);
    run("glds+mfma R=16", k_glds_mfma<16>);
    run("glds+mfma2 R=8", k_glds_mfma2<8>);
    run("glds+mfma2 R=12", k_glds_mfma2<12>);
    run("glds+mfma2 R=16", k_glds_mfma2<16>);
    run("glds+mfma3 R=8", k_glds_mfma3<8>);
    run("glds+mfma3 R=12", k_glds_mfma3<12>);
    run("glds+mfma3 R=16", k_glds_mfma3<16>);
    run("mfma only", k_mfma_only);
    run("split: mfma waves only", k_split<true, false>);
    run("split: stream waves only", k_split<false, true>);
    run("split: both", k_split<true, true>);
    run("f16x2 mfma only", k_f16_only);
    run("f16x2 ring R=4", k_f16_ring<4>);
    run("f16x2 ring R=8", k_f16_ring<8>);
    run("f16x2 ring R=12", k_f16_ring<12>);
    run("split: both, stream prio 3", k_split<true, true, 3>);
    run("split2: mfma + vgpr stream", k_split2<0>);
    run("split2: valu + glds stream", k_split2<1>);
    run("split2: valu alone", k_split2<2>);
    return 0;
}
