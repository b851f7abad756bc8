// x2 bilinear upsampling of NHWC fp32 maps, times a scale:
//   scale * F.interpolate(x, scale_factor=2, mode='bilinear', align_corners=False)
// as PCD_Align applies it to the coarser level's offsets (x2) and aligned features (x1)
// (Sakuya_arch_test.py:86-87,90,95-96,99,112,116,121,125).  Materialising the upsampled map
// (HBM-bound, ~3 bytes moved per byte produced) lets the cat(., up(.)) convolutions run on the
// Winograd kernel with two full-resolution inputs.
#include "abi_util.h"
#include "stif.h"
#include "stif_common.h"

#include <algorithm>

namespace {

// one thread = 4 channels of one output pixel
// grid (x blocks over one output row's W * c/4 float4s, output row y, item): 32-bit index math only
// (the flat 64-bit div/mod per element dominated the old mapping)
__global__ __launch_bounds__(256) void k_up2(const float* __restrict__ in, float* __restrict__ out, int n, int h1,
                                             int w1, int c, float scale, long long in_item, long long out_item) {
  const int c4n = c >> 2;
  const int W = 2 * w1;
  const int y = blockIdx.y, item = blockIdx.z;
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= W * c4n) return;
  const int x = t / c4n, q = t - x * c4n;
  // align_corners=False source coordinates (clamped at 0 like ATen's area_pixel_compute_source_index)
  const float sy = fmaxf(0.5f * ((float)y + 0.5f) - 0.5f, 0.f);
  const float sx = fmaxf(0.5f * ((float)x + 0.5f) - 0.5f, 0.f);
  const int y0 = min((int)sy, h1 - 1), x0 = min((int)sx, w1 - 1);
  const int y1 = y0 + (y0 < h1 - 1 ? 1 : 0), x1 = x0 + (x0 < w1 - 1 ? 1 : 0);
  const float ly1 = sy - (float)y0, lx1 = sx - (float)x0;
  const float ly0 = 1.f - ly1, lx0 = 1.f - lx1;
  const float* src = in + (size_t)item * in_item + q * 4;
  const f32x4 v00 = ld4(src + ((size_t)y0 * w1 + x0) * c), v01 = ld4(src + ((size_t)y0 * w1 + x1) * c);
  const f32x4 v10 = ld4(src + ((size_t)y1 * w1 + x0) * c), v11 = ld4(src + ((size_t)y1 * w1 + x1) * c);
  const f32x4 v = (ly0 * (lx0 * v00 + lx1 * v01) + ly1 * (lx0 * v10 + lx1 * v11)) * scale;
  st4(out + (size_t)item * out_item + ((size_t)y * W + x) * c + q * 4, v);
}

// one thread = 4 channels of the 2x2 output quad of input pixel (i, j): rows 2i, 2i+1, columns 2j,
// 2j+1.  Every corner of those four outputs lies in the 3x3 input neighbourhood of (i, j), so the
// thread loads 9 float4s for 4 outputs (16 with k_up2) and evaluates each output with k_up2's
// coordinates, weights and expression (same rounding).  grid (x blocks over w1 * c/4, input row i, item)
STIF_DEV f32x4 sel3(int s, f32x4 a, f32x4 b, f32x4 c) { return s == 0 ? a : (s == 1 ? b : c); }

__global__ __launch_bounds__(256) void k_up2q(const float* __restrict__ in, float* __restrict__ out, int n, int h1,
                                              int w1, int c, float scale, long long in_item, long long out_item) {
  const int c4n = c >> 2;
  const int W = 2 * w1;
  const int i = blockIdx.y, item = blockIdx.z;
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= w1 * c4n) return;
  const int j = t / c4n, q = t - j * c4n;
  const float* src = in + (size_t)item * in_item + q * 4;
  float* dst = out + (size_t)item * out_item + q * 4;
  // neighbourhood slot s holds input row / column (i|j) - 1 + s, clamped into the image (a clamped
  // slot is never selected: every corner row / column lies inside the image)
  const int r0 = max(i - 1, 0), r2 = min(i + 1, h1 - 1);
  const int k0 = max(j - 1, 0), k2 = min(j + 1, w1 - 1);
  f32x4 R[3][3];
  const int rows[3] = {r0, i, r2}, cols[3] = {k0, j, k2};
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b) R[a][b] = ld4(src + ((size_t)rows[a] * w1 + cols[b]) * c);
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const int y = 2 * i + a;
    const float sy = fmaxf(0.5f * ((float)y + 0.5f) - 0.5f, 0.f);
    const int y0 = min((int)sy, h1 - 1);
    const int y1 = y0 + (y0 < h1 - 1 ? 1 : 0);
    const float ly1 = sy - (float)y0, ly0 = 1.f - ly1;
    const int sy0 = y0 - i + 1, sy1 = y1 - i + 1;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int x = 2 * j + b;
      const float sx = fmaxf(0.5f * ((float)x + 0.5f) - 0.5f, 0.f);
      const int x0 = min((int)sx, w1 - 1);
      const int x1 = x0 + (x0 < w1 - 1 ? 1 : 0);
      const float lx1 = sx - (float)x0, lx0 = 1.f - lx1;
      const int sx0 = x0 - j + 1, sx1 = x1 - j + 1;
      const f32x4 u0 = sel3(sy0, R[0][0], R[1][0], R[2][0]), u1 = sel3(sy0, R[0][1], R[1][1], R[2][1]),
                  u2 = sel3(sy0, R[0][2], R[1][2], R[2][2]);
      const f32x4 d0 = sel3(sy1, R[0][0], R[1][0], R[2][0]), d1 = sel3(sy1, R[0][1], R[1][1], R[2][1]),
                  d2 = sel3(sy1, R[0][2], R[1][2], R[2][2]);
      const f32x4 v00 = sel3(sx0, u0, u1, u2), v01 = sel3(sx1, u0, u1, u2);
      const f32x4 v10 = sel3(sx0, d0, d1, d2), v11 = sel3(sx1, d0, d1, d2);
      const f32x4 v = (ly0 * (lx0 * v00 + lx1 * v01) + ly1 * (lx0 * v10 + lx1 * v11)) * scale;
      st4(dst + ((size_t)y * W + x) * c, v);
    }
  }
}

}  // namespace

extern "C" int stif_upsample2x_nhwc(const float* in, float* out, int n, int h1, int w1, int c, float scale,
                                    long long in_item, long long out_item, void* stream) {
  if (!in || !out || n < 1 || h1 < 1 || w1 < 1 || c < 4 || c % 4 || in_item < (long long)h1 * w1 * c ||
      out_item < 4LL * h1 * w1 * c)
    return stif_fail(STIF_E_INVALID, "stif_upsample2x_nhwc: bad arguments");
  if (2LL * h1 > 65535 || n > 65535 || 2LL * w1 * (c / 4) > 0x7fffffffLL)
    return stif_fail(STIF_E_INVALID, "stif_upsample2x_nhwc: image too large for the row grid");
  // the 2x2-quad kernel reads 9 instead of 16 float4s per 4 outputs but runs 4x fewer threads: faster
  // on large maps (48 x 128^2 -> 256^2: 282 -> 250 us), slower on small ones whose input stays in
  // cache (48 x 64^2: 43 -> 47 us), so it takes launches of >= 8M quad threads
  const long long quads = (long long)n * h1 * w1 * (c / 4);
  const bool quad = quads >= (8LL << 20);
  if (quad) {
    const dim3 grid((unsigned)((w1 * (c / 4) + 255) / 256), (unsigned)h1, (unsigned)n);
    hipLaunchKernelGGL(k_up2q, grid, dim3(256), 0, (hipStream_t)stream, in, out, n, h1, w1, c, scale, in_item,
                       out_item);
  } else {
    const dim3 grid((unsigned)((2 * w1 * (c / 4) + 255) / 256), (unsigned)(2 * h1), (unsigned)n);
    hipLaunchKernelGGL(k_up2, grid, dim3(256), 0, (hipStream_t)stream, in, out, n, h1, w1, c, scale, in_item,
                       out_item);
  }
  return stif_check_launch("stif_upsample2x_nhwc");
}

namespace {

// one thread = one output pixel of the 8-channel image (rgb0 rgb1 0 0)
__global__ __launch_bounds__(256) void k_up_img(const float* __restrict__ x, float* __restrict__ out, int n, int h,
                                                int w, int s) {
  const int H = s * h, W = s * w;
  const long long total = (long long)n * H * W;
  const float inv = 1.0f / (float)s;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const int X = (int)(e % W);
    long long r = e / W;
    const int Y = (int)(r % H);
    const int item = (int)(r / H);
    // ATen upsample_bilinear2d, align_corners=False, scale_factor given: src = (d + 0.5) / s - 0.5, >= 0
    const float sy = fmaxf(((float)Y + 0.5f) * inv - 0.5f, 0.f);
    const float sx = fmaxf(((float)X + 0.5f) * inv - 0.5f, 0.f);
    const int y0 = min((int)sy, h - 1), x0 = min((int)sx, w - 1);
    const int y1 = y0 + (y0 < h - 1 ? 1 : 0), x1 = x0 + (x0 < w - 1 ? 1 : 0);
    const float ly1 = sy - (float)y0, lx1 = sx - (float)x0;
    const float ly0 = 1.f - ly1, lx0 = 1.f - lx1;
    const float* src = x + (size_t)item * 6 * h * w;
    float v[8];
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      const float* p = src + (size_t)c * h * w;
      v[c] = ly0 * (lx0 * p[y0 * w + x0] + lx1 * p[y0 * w + x1]) + ly1 * (lx0 * p[y1 * w + x0] + lx1 * p[y1 * w + x1]);
    }
    v[6] = v[7] = 0.f;
    float* o = out + (size_t)e * 8;
    st4(o, f32x4{v[0], v[1], v[2], v[3]});
    st4(o + 4, f32x4{v[4], v[5], v[6], v[7]});
  }
}

}  // namespace

extern "C" int stif_upsample_image(const float* x_nchw, float* out, int n, int h, int w, int s, void* stream) {
  if (!x_nchw || !out || n < 1 || h < 1 || w < 1 || s < 1) return stif_fail(STIF_E_INVALID, "stif_upsample_image: bad arguments");
  const long long total = (long long)n * s * h * s * w;
  const long long blocks = std::min<long long>((total + 255) / 256, 1 << 20);
  hipLaunchKernelGGL(k_up_img, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, x_nchw, out, n, h, w, s);
  return stif_check_launch("stif_upsample_image");
}

// ---------------------------------------------------------------- video harness I/O
// custom_video_test.py:88-92,101-103: frames come in as cv2 uint8 BGR HWC, are resized by
// data.util.imresize_np(img, 1/2, antialiasing=True) (data/util.py:302-371: separable MATLAB cubic,
// symmetric padding, H pass then W pass), scaled by 1/255 and flipped to RGB NCHW; outputs go back
// as (clamp(0,1) * 255).astype(uint8) HWC RGB.
namespace {

// symmetric-padded index (data/util.py:325-335, 350-360) -> source index
STIF_DEV int sym_src(int j, int n, int s0) {
  const int k = j - s0;
  return k < 0 ? -k - 1 : (k >= n ? 2 * n - 1 - k : k);
}

// one thread = one output pixel (3 channels) of one frame
__global__ __launch_bounds__(256) void k_resize_in(const unsigned char* __restrict__ src, float* __restrict__ out,
                                                   int nf, int H, int W, int oH, int oW,
                                                   const float* __restrict__ wH, const int* __restrict__ iH, int PH,
                                                   int sH, const float* __restrict__ wW, const int* __restrict__ iW,
                                                   int PW, int sW) {
  const long long total = (long long)nf * oH * oW;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const int x = (int)(e % oW);
    long long r = e / oW;
    const int y = (int)(r % oH);
    const int f = (int)(r / oH);
    const unsigned char* img = src + (size_t)f * H * W * 3;
    float acc[3] = {0.f, 0.f, 0.f};
    for (int p = 0; p < PW; ++p) {
      const int sx = sym_src(iW[x] + p, W, sW);
      float col[3] = {0.f, 0.f, 0.f};   // H pass at column sx (out_1 of the reference)
      for (int q = 0; q < PH; ++q) {
        const int sy = sym_src(iH[y] + q, H, sH);
        const unsigned char* px = img + ((size_t)sy * W + sx) * 3;
        const float w = wH[y * PH + q];
        col[0] = fmaf(w, (float)px[0], col[0]);
        col[1] = fmaf(w, (float)px[1], col[1]);
        col[2] = fmaf(w, (float)px[2], col[2]);
      }
      const float w = wW[x * PW + p];
      acc[0] = fmaf(w, col[0], acc[0]);
      acc[1] = fmaf(w, col[1], acc[1]);
      acc[2] = fmaf(w, col[2], acc[2]);
    }
    const size_t plane = (size_t)oH * oW;
    float* o = out + (size_t)f * 3 * plane + (size_t)y * oW + x;
    // .astype(float32) / 255, BGR -> RGB
    o[0] = acc[2] / 255.f;
    o[plane] = acc[1] / 255.f;
    o[2 * plane] = acc[0] / 255.f;
  }
}

// (img.clamp(0, 1).permute(1, 2, 0) * 255).numpy().astype(np.uint8): NCHW float -> HWC uint8
__global__ __launch_bounds__(256) void k_to_u8(const float* __restrict__ in, unsigned char* __restrict__ out, int n,
                                               int H, int W) {
  const long long total = (long long)n * H * W;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const long long item = e / ((long long)H * W);
    const long long yx = e - item * H * W;
    const float* p = in + (size_t)item * 3 * H * W + yx;
    unsigned char* o = out + (size_t)e * 3;
#pragma unroll
    for (int c = 0; c < 3; ++c) o[c] = (unsigned char)(fminf(fmaxf(p[(size_t)c * H * W], 0.f), 1.f) * 255.f);
  }
}

}  // namespace

extern "C" int stif_resize_frames(const unsigned char* bgr, float* out_rgb_nchw, int nf, int H, int W, int oH, int oW,
                                  const float* wH, const int* iH, int PH, int sH, const float* wW, const int* iW,
                                  int PW, int sW, void* stream) {
  if (!bgr || !out_rgb_nchw || !wH || !iH || !wW || !iW || nf < 1 || H < 1 || W < 1 || oH < 1 || oW < 1 || PH < 1 ||
      PW < 1 || sH < 1 || sW < 1 || sH > H || sW > W)
    return stif_fail(STIF_E_INVALID, "stif_resize_frames: bad arguments");
  const long long total = (long long)nf * oH * oW;
  const long long blocks = std::min<long long>((total + 255) / 256, 1 << 20);
  hipLaunchKernelGGL(k_resize_in, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, bgr, out_rgb_nchw, nf, H,
                     W, oH, oW, wH, iH, PH, sH, wW, iW, PW, sW);
  return stif_check_launch("stif_resize_frames");
}

extern "C" int stif_frames_to_u8(const float* nchw, unsigned char* hwc, int n, int H, int W, void* stream) {
  if (!nchw || !hwc || n < 1 || H < 1 || W < 1) return stif_fail(STIF_E_INVALID, "stif_frames_to_u8: bad arguments");
  const long long total = (long long)n * H * W;
  const long long blocks = std::min<long long>((total + 255) / 256, 1 << 20);
  hipLaunchKernelGGL(k_to_u8, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, nchw, hwc, n, H, W);
  return stif_check_launch("stif_frames_to_u8");
}
