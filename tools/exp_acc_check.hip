// exp_acc (yk_common.h) against the library expf and __expf on [-30, 0] and its special values
// (GPU box).  build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -o tools/_exp_acc_check tools/exp_acc_check.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
__device__ __forceinline__ float exp_acc(float x) {
    constexpr float L2E = 1.44269504088896340736f, L2E_LO = 1.9259629890910904e-08f, LN2 = 0.693147180559945309f;
    const float t = x * L2E;
    const float r = t > -150.f ? fmaf(x, L2E_LO, fmaf(x, L2E, -t)) : 0.f;
    const float e = __builtin_amdgcn_exp2f(t);
    return fmaf(e, r * LN2, e);
}
__global__ void k(const float* x, float* y, float* z, float* w, int n) { int i = blockIdx.x * 256 + threadIdx.x; if (i < n) { y[i] = exp_acc(x[i]); z[i] = expf(x[i]); w[i] = __expf(x[i]); } }
int main() {
  const int n = 1 << 22; float *x, *y, *z, *w;
  (void)hipMallocManaged(&x, n * 4); (void)hipMallocManaged(&y, n * 4); (void)hipMallocManaged(&z, n * 4); (void)hipMallocManaged(&w, n * 4);
  for (int i = 0; i < n; i++) x[i] = -30.0f * (float)i / n;
  x[0] = -INFINITY; x[1] = NAN; x[2] = -200.f; x[3] = 0.f;
  k<<<n / 256, 256>>>(x, y, z, w, n); (void)hipDeviceSynchronize();
  double ma = 0, ml = 0, mf = 0;
  for (int i = 4; i < n; i++) { double ex = exp((double)x[i]); ma = fmax(ma, fabs(y[i] - ex) / ex); ml = fmax(ml, fabs(z[i] - ex) / ex); mf = fmax(mf, fabs(w[i] - ex) / ex); }
  printf("max rel err over [-30,0]: exp_acc %.3g  expf %.3g  __expf %.3g  (f32 ulp 1.19e-7 / 5.96e-8 half)\n", ma, ml, mf);
  printf("specials: exp_acc(-inf)=%g (nan)=%g (-200)=%g (0)=%g\n", y[0], y[1], y[2], y[3]);
  return 0;
}
