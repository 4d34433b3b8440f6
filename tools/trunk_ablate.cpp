// Diagnostic harness (not part of the product): times k_forward of yk_net.hip on
// synthetic rows.  Build one binary per -DYK_ABL variant (see tools/ablate.sh).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../nypc-yacht-auction_amd/csrc/yk_net.hip"

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
    printf("YK_ABL=%d rows=%d forward %.2f us  %.1f TFLOP/s\n", YK_ABL, n, us, 3320576.0 * n / (us * 1e-6) / 1e12);
    return 0;
}
