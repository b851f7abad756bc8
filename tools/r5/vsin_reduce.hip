// Does the hardware sine need the x - rint(x) reduction?  For y in revolutions, compare v_sin(y) with
// v_sin(y - rint(y)) bit for bit over a sweep of |y| bands, and both against double sin(2 pi y).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

__global__ void k(const float* y, float* a, float* b, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    float v = y[i];
    a[i] = __builtin_amdgcn_sinf(v);
    b[i] = __builtin_amdgcn_sinf(v - __builtin_rintf(v));
  }
}

int main() {
  const float bands[] = {0.5f, 1.f, 4.f, 16.f, 64.f, 256.f, 1024.f, 65536.f, 1.0e7f};
  const int n = 1 << 22;
  std::vector<float> y(n), a(n), b(n);
  float *dy, *da, *db;
  hipMalloc(&dy, n * 4); hipMalloc(&da, n * 4); hipMalloc(&db, n * 4);
  for (float B : bands) {
    unsigned s = 12345;
    for (int i = 0; i < n; ++i) {
      s = s * 1664525u + 1013904223u;
      y[i] = ((s >> 8) * (1.0f / 16777216.0f) * 2.f - 1.f) * B;
    }
    hipMemcpy(dy, y.data(), n * 4, hipMemcpyHostToDevice);
    k<<<(n + 255) / 256, 256>>>(dy, da, db, n);
    hipMemcpy(a.data(), da, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(b.data(), db, n * 4, hipMemcpyDeviceToHost);
    long diff = 0; double ea = 0, eb = 0, dab = 0;
    for (int i = 0; i < n; ++i) {
      double r = std::sin(2.0 * M_PI * (double)y[i]);
      ea = std::fmax(ea, std::fabs(a[i] - r)); eb = std::fmax(eb, std::fabs(b[i] - r));
      if (a[i] != b[i]) { ++diff; dab = std::fmax(dab, std::fabs((double)a[i] - b[i])); }
    }
    printf("|y|<=%6.1f rev: raw v_sin max err %.3e, reduced max err %.3e, %ld of %d differ (max |diff| %.3e)\n", B, ea, eb,
           diff, n, dab);
  }
  return 0;
}
