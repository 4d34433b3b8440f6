// Diagnostic harness (not part of the product): times k_forward of yk_net.hip on
// synthetic rows (tools/timing.sh builds it with -DYK_TIMING for per-phase stamps).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "yk_net.hip"  // tools/stage_hooks.sh: the sources with tools/diag_hooks.patch applied

int main(int argc, char** argv) {
    const int H = 256, NB = 6, n = argc > 1 ? atoi(argv[1]) : 3480, iters = 200;
    std::vector<std::vector<float>> p;
    auto add = [&](size_t k, float sc) { std::vector<float> v(k); for (size_t i = 0; i < k; i++) v[i] = sc * (float)((i * 2654435761u) % 1000) / 1000.f - sc / 2; p.push_back(v); };
    add((size_t)H * 59, 0.2f); add(H, 0.1f); add(H, 1.f); add(H, 0.1f);
    for (int b = 0; b < NB; b++) { add((size_t)H * H, 0.1f); add(H, 0.1f); add(H, 1.f); add(H, 0.1f); add((size_t)H * H, 0.1f); add(H, 0.1f); add(H, 1.f); add(H, 0.1f); }
    add(H, 1.f); add(H, 0.1f); add((size_t)3226 * H, 0.1f); add(3226, 0.1f);
    add(H, 1.f); add(H, 0.1f); add((size_t)128 * H, 0.1f); add(128, 0.1f); add(128, 0.1f); add(1, 0.1f);
    std::vector<const float*> pp; for (auto& v : p) pp.push_back(v.data());
    yk_net_t* net; if (yk_net_create(&net, H, NB, pp.data(), (int)pp.size())) { printf("create failed\n"); return 1; }
    float *x, *v, *lg; hipMalloc(&x, sizeof(float) * n * 59); hipMalloc(&v, sizeof(float) * n); hipMalloc(&lg, sizeof(float) * (size_t)n * yk::PI_LD);
    std::vector<float> hx((size_t)n * 59); for (size_t i = 0; i < hx.size(); i++) hx[i] = (float)((i * 7919) % 13) / 13.f - 0.5f;
    hipMemcpy(x, hx.data(), sizeof(float) * hx.size(), hipMemcpyHostToDevice);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int w = 0; w < 20; w++) yk::launch_forward(net->dev, nullptr, x, nullptr, nullptr, n, lg, v, 0);
    hipEventRecord(e0); for (int i = 0; i < iters; i++) yk::launch_forward(net->dev, nullptr, x, nullptr, nullptr, n, lg, v, 0); hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double us = 1000.0 * ms / iters;
    printf("rows=%d forward %.2f us  %.1f TFLOP/s\n", n, us, 3320576.0 * n / (us * 1e-6) / 1e12);
#ifdef YK_TIMING
    {  // mean s_memtime ticks per phase of wave 0, over the workgroups of the last launch
        const int nb = (n + 15) / 16;
        std::vector<unsigned long long> t((size_t)nb * TS_STRIDE);
        hipMemcpyFromSymbol(t.data(), HIP_SYMBOL(g_tstamp), sizeof(unsigned long long) * t.size());
        const char* names[16] = {"start", "featurize", "input", "blk0", "blk1", "blk2", "blk3", "blk4", "blk5",
                                 "headLN", "pi01", "pi23", "pi45", "-", "pitail", "end"};
        unsigned long long tmin = ~0ull, tmax = 0;
        for (int b = 0; b < nb; b++) { tmin = std::min(tmin, t[b * TS_STRIDE]); tmax = std::max(tmax, t[b * TS_STRIDE + 15]); }
        printf("launch span %llu ticks; per-WG mean phase ticks:\n", tmax - tmin);
        int prev = 0;
        for (int i = 1; i < 16; i++) {
            if (i == 13) continue;
            double s = 0; for (int b = 0; b < nb; b++) s += (double)(t[b * TS_STRIDE + i] - t[b * TS_STRIDE + prev]);
            printf("  %-9s %9.0f\n", names[i], s / nb);
            prev = i;
        }
        double s = 0, mx = 0; for (int b = 0; b < nb; b++) { double d = (double)(t[b * TS_STRIDE + 15] - t[b * TS_STRIDE]); s += d; mx = std::max(mx, d); }
        printf("  total     %9.0f (max %9.0f)\n", s / nb, mx);
        // block 2 detail (16 fc1 GEMM, 17 LN1 vec+store+barrier, 18 LN1 pass, 19 fc2 GEMM,
        // 20 barrier, 21 store+barrier) and the end phase (22 tail barrier, 23 v store+barrier)
        const int det[][2] = {{4, 16}, {16, 13}, {13, 22}, {22, 17}, {18, 19}, {19, 20}, {20, 5}, {23, 15}};
        const char* dn[] = {"b2.fc1", "b2.ep1st", "b2.ep1bar", "b2.ep1app", "b2.fc2", "b2.ep2", "b2.rest", "vfinal"};
        for (int w = 0; w < 8; w++) {  // per-wave end of the policy head, relative to the heads LN stamp
            double a = 0; for (int b = 0; b < nb; b++) a += (double)(t[b * TS_STRIDE + 24 + w] - t[b * TS_STRIDE + 9]);
            printf("  pi.w%d    %9.0f\n", w, a / nb);
        }
        for (int k = 0; k < 8; k++) {
            double a = 0; for (int b = 0; b < nb; b++) a += (double)(t[b * TS_STRIDE + det[k][1]] - t[b * TS_STRIDE + det[k][0]]);
            printf("  %-9s %9.0f\n", dn[k], a / nb);
        }
        // block 2, per wave (tools/diag_sources.py LSTAMP): fc1 GEMM, accumulator store, first barrier,
        // row pass, second barrier, fc2 GEMM; and the spread of the waves' GEMM ends (skew)
        std::vector<unsigned long long> ws((size_t)nb * 16 * 8);
        hipMemcpyFromSymbol(ws.data(), HIP_SYMBOL(g_wstamp), sizeof(unsigned long long) * ws.size());
        const char* pn[6] = {"fc1 GEMM", "acc store", "barrier 1", "row pass", "barrier 2", "fc2 GEMM"};
        printf("block 2 per wave (mean over workgroups, ticks):\n  wave ");
        for (int k = 0; k < 6; k++) printf(" %10s", pn[k]);
        printf("\n");
        for (int w = 0; w < 8; w++) {
            printf("  %4d ", w);
            for (int k = 0; k < 6; k++) {
                double a = 0;
                for (int b = 0; b < nb; b++) a += (double)(ws[(b * 16 + w) * 8 + k + 1] - ws[(b * 16 + w) * 8 + k]);
                printf(" %10.0f", a / nb);
            }
            printf("\n");
        }
        double sk = 0, sk5 = 0;
        for (int b = 0; b < nb; b++) {
            unsigned long long lo = ~0ull, hi = 0, lo5 = ~0ull, hi5 = 0;
            for (int w = 0; w < 8; w++) {
                lo = std::min(lo, ws[(b * 16 + w) * 8 + 1]); hi = std::max(hi, ws[(b * 16 + w) * 8 + 1]);
                lo5 = std::min(lo5, ws[(b * 16 + w) * 8 + 6]); hi5 = std::max(hi5, ws[(b * 16 + w) * 8 + 6]);
            }
            sk += (double)(hi - lo); sk5 += (double)(hi5 - lo5);
        }
        printf("  spread of the waves' fc1 GEMM ends %.0f, fc2 GEMM ends %.0f ticks\n", sk / nb, sk5 / nb);
    }
#endif
    return 0;
}
