// Accuracy of sine evaluations on gfx950 vs a double-precision sin of the same fp32 argument:
// the previous polynomial sine, the bare hardware v_sin_f32 (argument in revolutions), a 2-part
// Cody-Waite / magic-rounding polynomial variant, and the two product sines of stif_common.h:
// stif_sin_poly (the fp32-operand decoder: pi/2 Cody-Waite + Taylor) and stif_sin_rev (the f16x3
// decoder: its argument is already in revolutions, omega / 2 pi folded into the packed weights, so it
// is fed x / 2 pi here, rounded to fp32 as the packed weights round it).  Max abs error per |x| band.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
#include "../../stif-continuous-video-representation_amd/csrc/stif_common.h"

__device__ float sin_cw2(float x) {
  const float qm = fmaf(x, 0.318309886183790671538f, 12582912.0f);   // 1.5 * 2^23: round to integer
  const float q = qm - 12582912.0f;
  float r = fmaf(q, -3.140625f, x);
  r = fmaf(q, -9.67653589793e-4f, r);
  const float r2 = r * r;
  float p = fmaf(r2, -2.3845164e-08f, 2.7522526e-06f);
  p = fmaf(r2, p, -1.9840802e-04f);
  p = fmaf(r2, p, 8.3333300e-03f);
  p = fmaf(r2, p, -1.6666667e-01f);
  const float s = fmaf(r * r2, p, r);
  return __int_as_float(__float_as_int(s) ^ (__float_as_int(qm) << 31));
}

__device__ float sin_poly(float x) {   // the previous stif_sin (3-part Cody-Waite by pi + odd polynomial)
  const float q = rintf(x * 0.318309886183790671538f);
  float r = fmaf(q, -3.140625f, x);
  r = fmaf(q, -9.67502593994140625e-4f, r);
  r = fmaf(q, -1.509957990e-7f, r);
  const float r2 = r * r;
  float p = fmaf(r2, -2.3845164e-08f, 2.7522526e-06f);
  p = fmaf(r2, p, -1.9840802e-04f);
  p = fmaf(r2, p, 8.3333300e-03f);
  p = fmaf(r2, p, -1.6666667e-01f);
  const float s = fmaf(r * r2, p, r);
  return __int_as_float(__float_as_int(s) ^ (((int)q & 1) << 31));
}

__global__ void k(const float* x, float* o, int n) {
  int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    const float v = x[i];
    o[i] = sin_poly(v);
    o[3 * n + i] = stif_sin_poly(v);
    o[4 * n + i] = stif_sin_rev(v * 0.159154943091895335769f);
    o[n + i] = __builtin_amdgcn_sinf(v * 0.159154943091895335769f);
    o[2 * n + i] = sin_cw2(v);
  }
}

int main() {
  const int n = 1 << 24;
  std::vector<float> x(n), o(5 * (size_t)n);
  for (int i = 0; i < n; ++i) x[i] = -3000.f + 6000.f * (float)((i * 2654435761u) % n) / n;
  float *dx, *dout;
  hipMalloc(&dx, n * 4);
  hipMalloc(&dout, 5 * (size_t)n * 4);
  hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
  k<<<(n + 255) / 256, 256>>>(dx, dout, n);
  hipMemcpy(o.data(), dout, 5 * (size_t)n * 4, hipMemcpyDeviceToHost);
  const float bands[] = {1, 4, 16, 64, 256, 1000, 3000};
  const char* names[] = {"poly", "v_sin_f32", "cw2_magic", "sin_poly", "sin_rev"};
  for (int m = 0; m < 5; ++m) {
    double e[7] = {0};
    for (int i = 0; i < n; ++i) {
      const double ref = std::sin((double)x[i]);
      const double d = std::fabs(o[(size_t)m * n + i] - ref);
      for (int b = 0; b < 7; ++b)
        if (std::fabs(x[i]) <= bands[b]) { if (d > e[b]) e[b] = d; break; }
    }
    printf("%-10s", names[m]);
    for (int b = 0; b < 7; ++b) printf("  |x|<=%g: %.2e", bands[b], e[b]);
    printf("\n");
  }
  return 0;
}
