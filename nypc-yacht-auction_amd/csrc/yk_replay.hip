// yk_replay.hip - the replay buffer's device side: trajectory record images
// (yk_engine_pack_records; one per rank after the all-gather) -> the training examples
// NNetWrapper.train consumes.
//
// Coach.executeEpisode (Coach.py:34-72) returns one (canonicalBoard, pi, v) per move;
// NNetWrapper.train (yacht/NNet.py:118-174) only uses argmax(pi) of it (:145-146).  So an
// example here is (packed board 64 B, target i32, value f32), written contiguously in
// (image, game, move) order - the order a single Coach playing every rank's games in env-id
// order would produce - so the pooled buffer does not depend on the GPU count.
//
// Byte-bound copy work: one wavefront per game, one lane per move (coalesced 64-B board rows);
// the only arithmetic is the argmax over a temp-1 move's sparse visit list.
#include "yk_api.h"
#include "yk_common.h"

using namespace yk;

namespace {

constexpr int SCAN_THREADS = 1024;

struct ImgView {
    const char* base;
    int64_t stride;  // bytes per image
    RecordLayout L;
    int E, M, VCAP;
    __device__ const char* part(int img, int p) const { return base + (int64_t)img * stride + L.off[p]; }
};

// Exclusive prefix of per-game move counts over the first n_games games (image-major order).
// One workgroup: each thread sums a contiguous chunk, then a workgroup scan of the chunk sums.
__global__ void __launch_bounds__(SCAN_THREADS) k_example_offsets(ImgView v, int64_t n_games, int64_t* off) {
    __shared__ int64_t part[SCAN_THREADS];
    const int t = threadIdx.x;
    const int64_t chunk = (n_games + SCAN_THREADS - 1) / SCAN_THREADS;
    const int64_t g0 = min<int64_t>((int64_t)t * chunk, n_games), g1 = min<int64_t>(g0 + chunk, n_games);
    int64_t s = 0;
    for (int64_t g = g0; g < g1; g++) {
        const int img = (int)(g / v.E), e = (int)(g % v.E);
        const int nm = reinterpret_cast<const int32_t*>(v.part(img, REC_NMOVES))[e];
        s += nm < 0 ? 0 : (nm > v.M ? v.M : nm);
    }
    part[t] = s;
    __syncthreads();
    for (int d = 1; d < SCAN_THREADS; d <<= 1) {  // Hillis-Steele inclusive scan
        const int64_t x = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += x;
        __syncthreads();
    }
    int64_t run = part[t] - s;  // exclusive start of this chunk
    for (int64_t g = g0; g < g1; g++) {
        off[g] = run;
        const int img = (int)(g / v.E), e = (int)(g % v.E);
        const int nm = reinterpret_cast<const int32_t*>(v.part(img, REC_NMOVES))[e];
        run += nm < 0 ? 0 : (nm > v.M ? v.M : nm);
    }
    if (t == SCAN_THREADS - 1) off[n_games] = part[t];
}

// One wavefront per game, lane m = move m.  Example k = off[g] + m - skip, kept if 0 <= k < cap.
__global__ void __launch_bounds__(64) k_examples(ImgView v, const int64_t* off, int64_t skip, int64_t cap,
                                                 yk_state_t* states, int32_t* targets, float* values) {
    const int64_t g = blockIdx.x;
    const int img = (int)(g / v.E), e = (int)(g % v.E);
    const int64_t base = off[g] - skip, n = off[g + 1] - off[g];
    const uint4* st = reinterpret_cast<const uint4*>(v.part(img, REC_STATES)) + ((int64_t)e * v.M) * 4;
    const int32_t* info = reinterpret_cast<const int32_t*>(v.part(img, REC_INFO)) + (int64_t)e * v.M * 8;
    const double* val = reinterpret_cast<const double*>(v.part(img, REC_VALUES)) + (int64_t)e * v.M;
    const uint32_t* vis = reinterpret_cast<const uint32_t*>(v.part(img, REC_VISITS)) + (int64_t)e * v.VCAP;
    const int32_t* voff = reinterpret_cast<const int32_t*>(v.part(img, REC_VOFF)) + (int64_t)e * (v.M + 1);
    for (int m = threadIdx.x; m < n; m += 64) {
        const int64_t k = base + m;
        if (k < 0 || k >= cap) continue;
        uint4* dst = reinterpret_cast<uint4*>(states + k);
#pragma unroll
        for (int q = 0; q < 4; q++) dst[q] = st[(int64_t)m * 4 + q];
        const int temp = info[m * 8 + 0], action = info[m * 8 + 2];
        int target = action;  // temp 0: pi is one-hot at the played action (MCTS.py:44-49)
        if (temp != 0) {
            // temp 1: pi = N / sum N (MCTS.py:51-54); argmax = the most visited action, the lowest
            // on ties (torch.argmax, NNet.py:145-146); the visit list is in ascending action order
            uint32_t best = 0;
            for (int i = voff[m], i1 = voff[m + 1]; i < i1; i++) {
                const uint32_t x = vis[i];
                if ((x & 0xFFFFu) > best) {
                    best = x & 0xFFFFu;
                    target = (int)(x >> 16);
                }
            }
        }
        targets[k] = target;
        values[k] = (float)val[m];  // torch.tensor(float64 list) -> float32 (NNet.py AZDataset)
    }
}

// The full policies of the kept examples (Coach.py:57-61: MCTS.getActionProb's pi per move) as a
// sparse CSR, for the examples file and for code that iterates the reference's tuples.  Pass 1:
// indptr[k] = nonzero entries of example k (1 at temp 0: one-hot at the played action,
// MCTS.py:44-49; the visited actions at temp 1, MCTS.py:51-54).  Same grid as k_examples.
__global__ void __launch_bounds__(64) k_pi_counts(ImgView v, const int64_t* off, int64_t skip, int64_t cap,
                                                  int64_t* indptr) {
    const int64_t g = blockIdx.x;
    const int img = (int)(g / v.E), e = (int)(g % v.E);
    const int64_t base = off[g] - skip, n = off[g + 1] - off[g];
    const int32_t* info = reinterpret_cast<const int32_t*>(v.part(img, REC_INFO)) + (int64_t)e * v.M * 8;
    const uint32_t* vis = reinterpret_cast<const uint32_t*>(v.part(img, REC_VISITS)) + (int64_t)e * v.VCAP;
    const int32_t* voff = reinterpret_cast<const int32_t*>(v.part(img, REC_VOFF)) + (int64_t)e * (v.M + 1);
    for (int m = threadIdx.x; m < n; m += 64) {
        const int64_t k = base + m;
        if (k < 0 || k >= cap) continue;
        int64_t c = 1;
        if (info[m * 8 + 0] != 0) {
            c = 0;
            for (int i = voff[m], i1 = voff[m + 1]; i < i1; i++) c += (vis[i] & 0xFFFFu) != 0;
        }
        indptr[k] = c;
    }
}

// In-place exclusive scan of a[0..n) into a[0..n], a[n] = the total.  One workgroup, a contiguous
// chunk per thread (as k_example_offsets).
__global__ void __launch_bounds__(SCAN_THREADS) k_scan_inplace(int64_t* a, int64_t n) {
    __shared__ int64_t part[SCAN_THREADS];
    const int t = threadIdx.x;
    const int64_t chunk = (n + SCAN_THREADS - 1) / SCAN_THREADS;
    const int64_t i0 = min<int64_t>((int64_t)t * chunk, n), i1 = min<int64_t>(i0 + chunk, n);
    int64_t s = 0;
    for (int64_t i = i0; i < i1; i++) s += a[i];
    part[t] = s;
    __syncthreads();
    for (int d = 1; d < SCAN_THREADS; d <<= 1) {
        const int64_t x = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += x;
        __syncthreads();
    }
    int64_t run = part[t] - s;
    for (int64_t i = i0; i < i1; i++) {
        const int64_t x = a[i];
        a[i] = run;
        run += x;
    }
    if (t == SCAN_THREADS - 1) a[n] = part[t];
}

// Pass 2: the entries (cols ascending, vals = N / sum N in float64, MCTS.py:52-54) and the float64
// values of the kept examples.
__global__ void __launch_bounds__(64) k_pi_fill(ImgView v, const int64_t* off, int64_t skip, int64_t cap,
                                                const int64_t* indptr, int32_t* cols, double* vals,
                                                double* values) {
    const int64_t g = blockIdx.x;
    const int img = (int)(g / v.E), e = (int)(g % v.E);
    const int64_t base = off[g] - skip, n = off[g + 1] - off[g];
    const int32_t* info = reinterpret_cast<const int32_t*>(v.part(img, REC_INFO)) + (int64_t)e * v.M * 8;
    const double* val = reinterpret_cast<const double*>(v.part(img, REC_VALUES)) + (int64_t)e * v.M;
    const uint32_t* vis = reinterpret_cast<const uint32_t*>(v.part(img, REC_VISITS)) + (int64_t)e * v.VCAP;
    const int32_t* voff = reinterpret_cast<const int32_t*>(v.part(img, REC_VOFF)) + (int64_t)e * (v.M + 1);
    for (int m = threadIdx.x; m < n; m += 64) {
        const int64_t k = base + m;
        if (k < 0 || k >= cap) continue;
        if (values) values[k] = val[m];
        int64_t o = indptr[k];
        if (info[m * 8 + 0] == 0) {
            cols[o] = info[m * 8 + 2];
            vals[o] = 1.0;
            continue;
        }
        double sum = 0.0;
        for (int i = voff[m], i1 = voff[m + 1]; i < i1; i++) sum += (double)(vis[i] & 0xFFFFu);
        for (int i = voff[m], i1 = voff[m + 1]; i < i1; i++) {
            const uint32_t x = vis[i];
            if ((x & 0xFFFFu) == 0) continue;
            cols[o] = (int32_t)(x >> 16);
            vals[o] = (double)(x & 0xFFFFu) / sum;
            o++;
        }
    }
}

struct Prep {
    ImgView v;
    int64_t n_games, total;
    int64_t* off;  // device [n_games + 1], freed by the caller (hipFreeAsync)
};

// The view of the images and the per-game example offsets (HOST total = all examples).
int prepare(const void* images, int n_images, int n_envs, int max_moves, int sims, int64_t n_games, hipStream_t s,
            Prep* p) {
    const int64_t all = (int64_t)n_images * n_envs;
    p->n_games = (n_games < 0 || n_games > all) ? all : n_games;
    p->v.base = static_cast<const char*>(images);
    p->v.E = n_envs;
    p->v.M = max_moves;
    p->v.VCAP = (int)record_vcap(max_moves, sims);
    p->v.L = record_layout(n_envs, max_moves, p->v.VCAP);
    p->v.stride = p->v.L.total;
    p->off = nullptr;
    YK_HIP(hipMallocAsync(reinterpret_cast<void**>(&p->off), sizeof(int64_t) * (size_t)(p->n_games + 1), s));
    hipLaunchKernelGGL(k_example_offsets, dim3(1), dim3(SCAN_THREADS), 0, s, p->v, p->n_games, p->off);
    YK_LAUNCHED();
    p->total = 0;
    YK_HIP(hipMemcpyAsync(&p->total, p->off + p->n_games, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    return YK_OK;
}

}  // namespace

extern "C" {

int yk_examples_from_records(const void* images, int n_images, int n_envs, int max_moves, int sims,
                             int64_t n_games, int64_t skip, int64_t capacity, yk_state_t* states, int32_t* targets,
                             float* values, int64_t* n_examples, void* stream) {
    if (!images || n_images <= 0 || n_envs <= 0 || max_moves <= 0 || sims < 0 || skip < 0 || !n_examples)
        return YK_ERR_ARG;
    if (states && (!targets || !values || capacity < 0)) return YK_ERR_ARG;
    hipStream_t s = as_stream(stream);
    Prep p;
    const int rc = prepare(images, n_images, n_envs, max_moves, sims, n_games, s, &p);
    if (rc != YK_OK) return rc;
    if (states && p.n_games > 0 && capacity > 0) {
        hipLaunchKernelGGL(k_examples, dim3((unsigned)p.n_games), dim3(64), 0, s, p.v, p.off, skip, capacity, states,
                           targets, values);
        YK_LAUNCHED();
    }
    YK_HIP(hipFreeAsync(p.off, s));
    YK_HIP(hipStreamSynchronize(s));
    int64_t n = p.total - skip;
    n = n < 0 ? 0 : n;
    if (states) n = n < capacity ? n : capacity;
    *n_examples = n;
    return YK_OK;
}

int yk_examples_policies(const void* images, int n_images, int n_envs, int max_moves, int sims, int64_t n_games,
                         int64_t skip, int64_t n_examples, int64_t* pi_indptr, int32_t* pi_cols, double* pi_vals,
                         int64_t nnz_capacity, double* values, int64_t* nnz, void* stream) {
    if (!images || n_images <= 0 || n_envs <= 0 || max_moves <= 0 || sims < 0 || skip < 0 || n_examples < 0 ||
        !pi_indptr || !nnz || (pi_cols && !pi_vals))
        return YK_ERR_ARG;
    hipStream_t s = as_stream(stream);
    Prep p;
    const int rc = prepare(images, n_images, n_envs, max_moves, sims, n_games, s, &p);
    if (rc != YK_OK) return rc;
    YK_HIP(hipStreamSynchronize(s));
    if (n_examples > p.total - skip) {  // asks for examples the images do not hold
        YK_HIP(hipFree(p.off));
        return YK_ERR_ARG;
    }
    if (p.n_games > 0 && n_examples > 0) {
        hipLaunchKernelGGL(k_pi_counts, dim3((unsigned)p.n_games), dim3(64), 0, s, p.v, p.off, skip, n_examples,
                           pi_indptr);
        YK_LAUNCHED();
    }
    hipLaunchKernelGGL(k_scan_inplace, dim3(1), dim3(SCAN_THREADS), 0, s, pi_indptr, n_examples);
    YK_LAUNCHED();
    int64_t total = 0;
    YK_HIP(hipMemcpyAsync(&total, pi_indptr + n_examples, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    YK_HIP(hipStreamSynchronize(s));
    int err = YK_OK;
    if (pi_cols && total > nnz_capacity) {
        err = YK_ERR_CAPACITY;
    } else if (pi_cols && p.n_games > 0 && n_examples > 0) {
        hipLaunchKernelGGL(k_pi_fill, dim3((unsigned)p.n_games), dim3(64), 0, s, p.v, p.off, skip, n_examples,
                           pi_indptr, pi_cols, pi_vals, values);
        YK_LAUNCHED();
    }
    YK_HIP(hipFreeAsync(p.off, s));
    YK_HIP(hipStreamSynchronize(s));
    *nnz = total;
    return err;
}

}  // extern "C"
