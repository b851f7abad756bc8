// Ablation microbenchmark for the implicit-GEMM conv (not part of the product library).
// Variants of the round-1 k_conv<3,1,2,2,0,RES> structure on the C1 trunk shape
// (18 items x 256 x 256 x 64 -> 64): which phase costs what.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include "stif_common.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1);} } while (0)

// ABL bits: 1 = stage weights only for chunk 0, 2 = stage input only for chunk 0, 4 = no epilogue store,
//           8 = no MFMA (keep LDS reads live)
template <int MT, int NT, int ABL>
__global__ __launch_bounds__(256) void k(const float* in0, const float* w, const float* bias, float* out,
                                        const float* res, int nitems, int H, int W) {
  constexpr int KS = 3, S = 1, TH = 4 * MT, HR = (TH - 1) * S + KS, HC = 31 * S + KS, PS = 12, T2 = 9,
                WS = T2 * 8 + 4, NJ = NT * 32, C0 = 64;
  __shared__ __attribute__((aligned(16))) float smem[HR * HC * PS + NJ * WS];
  float* s_in = smem;
  float* s_w = smem + HR * HC * PS;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, l32 = lane & 31, hf = lane >> 5;
  const int tiles_x = (W + 31) >> 5;
  const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x, n = blockIdx.z;
  const float* inp = in0 + (size_t)n * H * W * C0;
  const int oy0 = ty * TH, ox0 = tx * 32, iy0 = oy0 - 1, ix0 = ox0 - 1;
  f32x16 acc[MT][NT];
  for (int mt = 0; mt < MT; ++mt) for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x16{0};
  for (int c = 0; c < 8; ++c) {
    if (!(ABL & 2) || c == 0)
      for (int e = tid; e < HR * HC * 2; e += 256) {
        const int half = e & 1, pix = e >> 1, r = pix / HC, cc = pix - r * HC, y = iy0 + r, x = ix0 + cc;
        f32x4 v = f32x4{0};
        if (y >= 0 && y < H && x >= 0 && x < W) v = ld4(inp + ((size_t)y * W + x) * C0 + c * 8 + half * 4);
        st4(s_in + pix * PS + half * 4, v);
      }
    if (!(ABL & 1) || c == 0) {
      const float* wc = w + (size_t)c * 64 * T2 * 8;
      for (int e = tid; e < NJ * T2 * 2; e += 256) {
        const int j = e / (T2 * 2), q = e - j * (T2 * 2);
        st4(s_w + j * WS + q * 4, ld4(wc + (size_t)j * T2 * 8 + q * 4));
      }
    }
    __syncthreads();
#pragma unroll
    for (int tap = 0; tap < T2; ++tap) {
      const int ky = tap / KS, kx = tap % KS;
      f32x4 av[MT], bv[NT];
      for (int mt = 0; mt < MT; ++mt) av[mt] = ld4(s_in + (((wv * MT + mt) + ky) * HC + l32 + kx) * PS + hf * 4);
      for (int nt = 0; nt < NT; ++nt) bv[nt] = ld4(s_w + (nt * 32 + l32) * WS + tap * 8 + hf * 4);
      if (ABL & 8) {
        for (int mt = 0; mt < MT; ++mt) for (int nt = 0; nt < NT; ++nt) acc[mt][nt][0] += av[mt][0] * bv[nt][1];
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma32(av[mt][q], bv[nt][q], acc[mt][nt]);
      }
    }
    __syncthreads();
  }
  float* o = out + (size_t)n * H * W * 64;
  const float* rs = res + (size_t)n * H * W * 64;
  for (int nt = 0; nt < NT; ++nt) {
    const int co = nt * 32 + l32;
    const float bv = bias[co];
    for (int mt = 0; mt < MT; ++mt) {
      const int y = oy0 + wv * MT + mt;
      for (int r = 0; r < 16; ++r) {
        const int x = ox0 + mfma_row(r, lane);
        const size_t p = ((size_t)y * W + x) * 64 + co;
        if (ABL & 4) {
          asm volatile("" ::"v"(acc[mt][nt][r]));
        } else {
          o[p] = rs[p] + acc[mt][nt][r] + bv;
        }
      }
    }
  }
}


// v2: LDS-DMA staging of both operands (buffer_load ... lds for the zero-padded input halo,
// global_load_lds for the lane-ordered weight fragments), double-buffered, one barrier per chunk.
// Input halo image: [row][h][col][4] (lane-linear, no padding). Weights per chunk: [tap][nt][lane][4].
template <int MT, int NT, int NW>
__global__ __launch_bounds__(NW * 64) void k2(const float* in0, const float* wpk, const float* bias, float* out,
                                             const float* res, int nitems, int H, int W) {
  constexpr int TH = NW * MT, HR = TH + 2, HC = 34, T2 = 9, C0 = 64;
  constexpr int IN_EL = HR * 2 * HC;                 // 16-B elements per input buffer
  constexpr int IN_INST = (IN_EL + 63) / 64;
  constexpr int W_EL = T2 * NT * 64;
  constexpr int W_INST = W_EL / 64;
  constexpr int IN_F = IN_INST * 64 * 4, W_F = W_EL * 4;
  __shared__ __attribute__((aligned(16))) float smem[2 * (IN_F + W_F)];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, l32 = lane & 31, hf = lane >> 5;
  const int tiles_x = (W + 31) >> 5;
  const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x, n = blockIdx.z;
  const float* inp = in0 + (size_t)n * H * W * C0;
  const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void*)inp, (short)0, H * W * C0 * 4, 0x00020000);
  const int oy0 = ty * TH, ox0 = tx * 32, iy0 = oy0 - 1, ix0 = ox0 - 1;
  auto stage = [&](int c, int buf) {
    float* si = smem + buf * (IN_F + W_F);
    float* sw = si + IN_F;
    for (int i = wv; i < IN_INST; i += NW) {
      const int e = i * 64 + lane;
      const int col = e % HC, rh = e / HC, h = rh & 1, row = rh >> 1;
      const int y = iy0 + row, x = ix0 + col;
      const bool ok = e < IN_EL && y >= 0 && y < H && x >= 0 && x < W;
      const unsigned voff = ok ? (unsigned)((((size_t)y * W + x) * C0 + c * 8 + h * 4) * 4) : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rin, si + i * 256, 16, voff, 0, 0, 0);
    }
    const float* wc = wpk + (size_t)c * W_EL * 4;
    for (int i = wv; i < W_INST; i += NW)
      __builtin_amdgcn_global_load_lds(wc + (i * 64 + lane) * 4, sw + i * 256, 16, 0, 0);
  };
  f32x16 acc[MT][NT];
  for (int mt = 0; mt < MT; ++mt) for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x16{0};
  stage(0, 0);
  __syncthreads();
  for (int c = 0; c < 8; ++c) {
    if (c + 1 < 8) stage(c + 1, (c + 1) & 1);
    const float* si = smem + (c & 1) * (IN_F + W_F);
    const float* sw = si + IN_F;
#pragma unroll
    for (int tap = 0; tap < T2; ++tap) {
      const int ky = tap / 3, kx = tap % 3;
      f32x4 av[MT], bv[NT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) av[mt] = ld4(si + ((((wv * MT + mt) + ky) * 2 + hf) * HC + l32 + kx) * 4);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) bv[nt] = ld4(sw + ((tap * NT + nt) * 64 + lane) * 4);
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma32(av[mt][q], bv[nt][q], acc[mt][nt]);
    }
    __syncthreads();
  }
  float* o = out + (size_t)n * H * W * 64;
  const float* rs = res + (size_t)n * H * W * 64;
  for (int nt = 0; nt < NT; ++nt) {
    const int co = nt * 32 + l32;
    const float bv = bias[co];
    for (int mt = 0; mt < MT; ++mt) {
      const int y = oy0 + wv * MT + mt;
      for (int r = 0; r < 16; ++r) {
        const int x = ox0 + mfma_row(r, lane);
        const size_t p = ((size_t)y * W + x) * 64 + co;
        o[p] = rs[p] + acc[mt][nt][r] + bv;
      }
    }
  }
}

template <int MT, int NT, int NW>
void run2(const char* name, float* in, float* wpk, float* b, float* out, float* res, int N, int H, int W,
          const float* ref, std::vector<float>& hbuf) {
  dim3 grid((W / 32) * (H / (NW * MT)), 1, N);
  hipLaunchKernelGGL((k2<MT, NT, NW>), grid, dim3(NW * 64), 0, 0, in, wpk, b, out, res, N, H, W);
  CK(hipDeviceSynchronize());
  std::vector<float> got(hbuf.size());
  CK(hipMemcpy(got.data(), out, got.size() * 4, hipMemcpyDeviceToHost));
  double md = 0, mx = 0;
  for (size_t i = 0; i < got.size(); ++i) { md = fmax(md, fabs(got[i] - ref[i])); mx = fmax(mx, fabs(ref[i])); }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 20;
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) hipLaunchKernelGGL((k2<MT, NT, NW>), grid, dim3(NW * 64), 0, 0, in, wpk, b, out, res, N, H, W);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= iters;
  const double flops = 2.0 * 64 * 576 * (double)N * H * W;
  printf("%-40s %8.1f us  %6.1f TFLOP/s   maxdiff vs k %.3g (max %.3g)\n", name, ms * 1e3, flops / (ms * 1e-3) / 1e12, md, mx);
}


// Epilogue staged through LDS: per (mt, nt) a wave writes its 32 px x 32 cout accumulator tile
// into a private 4-KB LDS block ([px][co], 16-B slots XOR-swizzled by px&3), reads it back as
// float4 rows and issues coalesced 16-B residual loads / output stores (8 px x 128 B per instruction).
template <int MT, int NT, int NW>
__device__ __forceinline__ void epi_res_lds(f32x16 (&acc)[MT][NT], float* sbuf, const float* bias, float* o,
                                            const float* rs, int oy0, int ox0, int wv, int lane, int H, int W) {
  float* blk = sbuf + wv * 1024;
  const int l32 = lane & 31, hf = lane >> 5;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int y = oy0 + wv * MT + mt;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const float bv = bias[nt * 32 + l32];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int px = (r & 3) + 8 * (r >> 2) + 4 * hf;
        const int slot = (l32 >> 2) ^ (px & 3);
        blk[px * 32 + slot * 4 + (l32 & 3)] = acc[mt][nt][r] + bv;
      }
      // read back: lane -> (px = i*8 + lane/8, co4 = lane%8)
      f32x4 v[4], rv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int px = i * 8 + (lane >> 3), c4 = lane & 7;
        v[i] = ld4(blk + px * 32 + ((c4 ^ (px & 3)) * 4));
        rv[i] = ld4(rs + ((size_t)y * W + ox0 + px) * 64 + nt * 32 + c4 * 4);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int px = i * 8 + (lane >> 3), c4 = lane & 7;
        st4(o + ((size_t)y * W + ox0 + px) * 64 + nt * 32 + c4 * 4, v[i] + rv[i]);
      }
    }
  }
}

template <int MT, int NT, int NW>
__global__ __launch_bounds__(NW * 64) void k3(const float* in0, const float* wpk, const float* bias, float* out,
                                             const float* res, int nitems, int H, int W) {
  constexpr int TH = NW * MT, HR = TH + 2, HC = 34, T2 = 9, C0 = 64;
  constexpr int IN_EL = HR * 2 * HC;
  constexpr int IN_INST = (IN_EL + 63) / 64;
  constexpr int W_EL = T2 * NT * 64;
  constexpr int W_INST = W_EL / 64;
  constexpr int IN_F = IN_INST * 64 * 4, W_F = W_EL * 4;
  constexpr int SM = 2 * (IN_F + W_F) > NW * 1024 ? 2 * (IN_F + W_F) : NW * 1024;
  __shared__ __attribute__((aligned(16))) float smem[SM];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, l32 = lane & 31, hf = lane >> 5;
  const int tiles_x = (W + 31) >> 5;
  const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x, n = blockIdx.z;
  const float* inp = in0 + (size_t)n * H * W * C0;
  const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void*)inp, (short)0, H * W * C0 * 4, 0x00020000);
  const int oy0 = ty * TH, ox0 = tx * 32, iy0 = oy0 - 1, ix0 = ox0 - 1;
  auto stage = [&](int c, int buf) {
    float* si = smem + buf * (IN_F + W_F);
    float* sw = si + IN_F;
    for (int i = wv; i < IN_INST; i += NW) {
      const int e = i * 64 + lane;
      const int col = e % HC, rh = e / HC, h = rh & 1, row = rh >> 1;
      const int y = iy0 + row, x = ix0 + col;
      const bool ok = e < IN_EL && y >= 0 && y < H && x >= 0 && x < W;
      const unsigned voff = ok ? (unsigned)((((size_t)y * W + x) * C0 + c * 8 + h * 4) * 4) : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rin, si + i * 256, 16, voff, 0, 0, 0);
    }
    const float* wc = wpk + (size_t)c * W_EL * 4;
    for (int i = wv; i < W_INST; i += NW)
      __builtin_amdgcn_global_load_lds(wc + (i * 64 + lane) * 4, sw + i * 256, 16, 0, 0);
  };
  f32x16 acc[MT][NT];
  for (int mt = 0; mt < MT; ++mt) for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x16{0};
  stage(0, 0);
  __syncthreads();
  for (int c = 0; c < 8; ++c) {
    if (c + 1 < 8) stage(c + 1, (c + 1) & 1);
    const float* si = smem + (c & 1) * (IN_F + W_F);
    const float* sw = si + IN_F;
#pragma unroll
    for (int tap = 0; tap < T2; ++tap) {
      const int ky = tap / 3, kx = tap % 3;
      f32x4 av[MT], bv[NT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) av[mt] = ld4(si + ((((wv * MT + mt) + ky) * 2 + hf) * HC + l32 + kx) * 4);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) bv[nt] = ld4(sw + ((tap * NT + nt) * 64 + lane) * 4);
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma32(av[mt][q], bv[nt][q], acc[mt][nt]);
    }
    __syncthreads();
  }
  epi_res_lds<MT, NT, NW>(acc, smem, bias, out + (size_t)n * H * W * 64, res + (size_t)n * H * W * 64, oy0, ox0,
                          wv, lane, H, W);
}

// v1 staging + LDS epilogue
template <int MT, int NT>
__global__ __launch_bounds__(256) void k1e(const float* in0, const float* w, const float* bias, float* out,
                                         const float* res, int nitems, int H, int W) {
  constexpr int KS = 3, S = 1, TH = 4 * MT, HR = (TH - 1) * S + KS, HC = 31 * S + KS, PS = 12, T2 = 9,
                WS = T2 * 8 + 4, NJ = NT * 32, C0 = 64;
  __shared__ __attribute__((aligned(16))) float smem[HR * HC * PS + NJ * WS];
  float* s_in = smem;
  float* s_w = smem + HR * HC * PS;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, l32 = lane & 31, hf = lane >> 5;
  const int tiles_x = (W + 31) >> 5;
  const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x, n = blockIdx.z;
  const float* inp = in0 + (size_t)n * H * W * C0;
  const int oy0 = ty * TH, ox0 = tx * 32, iy0 = oy0 - 1, ix0 = ox0 - 1;
  f32x16 acc[MT][NT];
  for (int mt = 0; mt < MT; ++mt) for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x16{0};
  for (int c = 0; c < 8; ++c) {
    for (int e = tid; e < HR * HC * 2; e += 256) {
      const int half = e & 1, pix = e >> 1, r = pix / HC, cc = pix - r * HC, y = iy0 + r, x = ix0 + cc;
      f32x4 v = f32x4{0};
      if (y >= 0 && y < H && x >= 0 && x < W) v = ld4(inp + ((size_t)y * W + x) * C0 + c * 8 + half * 4);
      st4(s_in + pix * PS + half * 4, v);
    }
    const float* wc = w + (size_t)c * 64 * T2 * 8;
    for (int e = tid; e < NJ * T2 * 2; e += 256) {
      const int j = e / (T2 * 2), q = e - j * (T2 * 2);
      st4(s_w + j * WS + q * 4, ld4(wc + (size_t)j * T2 * 8 + q * 4));
    }
    __syncthreads();
#pragma unroll
    for (int tap = 0; tap < T2; ++tap) {
      const int ky = tap / KS, kx = tap % KS;
      f32x4 av[MT], bv[NT];
      for (int mt = 0; mt < MT; ++mt) av[mt] = ld4(s_in + (((wv * MT + mt) + ky) * HC + l32 + kx) * PS + hf * 4);
      for (int nt = 0; nt < NT; ++nt) bv[nt] = ld4(s_w + (nt * 32 + l32) * WS + tap * 8 + hf * 4);
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma32(av[mt][q], bv[nt][q], acc[mt][nt]);
    }
    __syncthreads();
  }
  epi_res_lds<MT, NT, 4>(acc, smem, bias, out + (size_t)n * H * W * 64, res + (size_t)n * H * W * 64, oy0, ox0, wv,
                         lane, H, W);
}

template <class KF>
void timeit(const char* name, KF launch, float* out, int N, int H, int W, const float* ref, size_t fm) {
  launch();
  CK(hipDeviceSynchronize());
  std::vector<float> got(fm);
  CK(hipMemcpy(got.data(), out, fm * 4, hipMemcpyDeviceToHost));
  double md = 0, mx = 0;
  for (size_t i = 0; i < fm; ++i) { md = fmax(md, fabs(got[i] - ref[i])); mx = fmax(mx, fabs(ref[i])); }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 20;
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= iters;
  const double flops = 2.0 * 64 * 576 * (double)N * H * W;
  printf("%-40s %8.1f us  %6.1f TFLOP/s   maxdiff %.3g (max %.3g)\n", name, ms * 1e3, flops / (ms * 1e-3) / 1e12, md, mx);
}

template <int MT, int NT, int ABL>
void run(const char* name, float* in, float* w, float* b, float* out, float* res, int N, int H, int W) {
  dim3 grid((W / 32) * (H / (4 * MT)), 1, N);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k<MT, NT, ABL>), grid, dim3(256), 0, 0, in, w, b, out, res, N, H, W);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 20;
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) hipLaunchKernelGGL((k<MT, NT, ABL>), grid, dim3(256), 0, 0, in, w, b, out, res, N, H, W);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= iters;
  const double flops = 2.0 * 64 * 576 * (double)N * H * W;
  printf("%-40s %8.1f us  %6.1f TFLOP/s\n", name, ms * 1e3, flops / (ms * 1e-3) / 1e12);
}

int main() {
  const int N = 18, H = 256, W = 256;
  size_t fm = (size_t)N * H * W * 64;
  float *in, *w, *b, *out, *res;
  CK(hipMalloc(&in, fm * 4));
  CK(hipMalloc(&res, fm * 4));
  CK(hipMalloc(&out, fm * 4));
  CK(hipMalloc(&w, 64 * 576 * 4));
  CK(hipMalloc(&b, 64 * 4));
  std::vector<float> h(fm);
  for (size_t i = 0; i < fm; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  CK(hipMemcpy(in, h.data(), fm * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(res, h.data(), fm * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(w, h.data(), 64 * 576 * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(b, h.data(), 64 * 4, hipMemcpyHostToDevice));
  run<2, 2, 0>("baseline MT2 NT2", in, w, b, out, res, N, H, W);
  run<2, 2, 1>("no weight restage", in, w, b, out, res, N, H, W);
  run<2, 2, 2>("no input restage", in, w, b, out, res, N, H, W);
  run<2, 2, 3>("no restage at all", in, w, b, out, res, N, H, W);
  run<2, 2, 4>("no epilogue store", in, w, b, out, res, N, H, W);
  run<2, 2, 7>("mfma + LDS reads only", in, w, b, out, res, N, H, W);
  run<2, 2, 8>("no mfma", in, w, b, out, res, N, H, W);
  run<4, 2, 0>("baseline MT4 NT2", in, w, b, out, res, N, H, W);
  run<1, 2, 0>("baseline MT1 NT2", in, w, b, out, res, N, H, W);

  // reference output of the baseline kernel
  run<2, 2, 0>("baseline (ref for v2)", in, w, b, out, res, N, H, W);
  std::vector<float> ref(fm);
  CK(hipMemcpy(ref.data(), out, fm * 4, hipMemcpyDeviceToHost));
  // repack weights [chunk][cout][tap][8] -> [chunk][tap][nt][lane][4]
  std::vector<float> wl(64 * 576), wp(64 * 576);
  CK(hipMemcpy(wl.data(), w, 64 * 576 * 4, hipMemcpyDeviceToHost));
  for (int c = 0; c < 8; ++c) for (int t = 0; t < 9; ++t) for (int nt = 0; nt < 2; ++nt) for (int l = 0; l < 64; ++l)
    for (int e = 0; e < 4; ++e)
      wp[((((size_t)c * 9 + t) * 2 + nt) * 64 + l) * 4 + e] = wl[(((size_t)c * 64 + nt * 32 + (l & 31)) * 9 + t) * 8 + 4 * (l >> 5) + e];
  float* wpk;
  CK(hipMalloc(&wpk, 64 * 576 * 4));
  CK(hipMemcpy(wpk, wp.data(), 64 * 576 * 4, hipMemcpyHostToDevice));
  run2<2, 2, 4>("v2 DMA dbuf MT2 NT2 NW4", in, wpk, b, out, res, N, H, W, ref.data(), h);
  run2<2, 2, 8>("v2 DMA dbuf MT2 NT2 NW8", in, wpk, b, out, res, N, H, W, ref.data(), h);
  run2<4, 2, 4>("v2 DMA dbuf MT4 NT2 NW4", in, wpk, b, out, res, N, H, W, ref.data(), h);
  run2<1, 2, 8>("v2 DMA dbuf MT1 NT2 NW8", in, wpk, b, out, res, N, H, W, ref.data(), h);
  run2<2, 2, 4>("v2 DMA dbuf MT2 NT2 NW4 (again)", in, wpk, b, out, res, N, H, W, ref.data(), h);
#define T3(MT, NT, NW) timeit("v3 DMA + LDS epi MT" #MT " NT" #NT " NW" #NW, [&]() { hipLaunchKernelGGL((k3<MT, NT, NW>), dim3((W / 32) * (H / (NW * MT)), 1, N), dim3(NW * 64), 0, 0, in, wpk, b, out, res, N, H, W); }, out, N, H, W, ref.data(), fm)
#define T1E(MT, NT) timeit("v1 staging + LDS epi MT" #MT " NT" #NT, [&]() { hipLaunchKernelGGL((k1e<MT, NT>), dim3((W / 32) * (H / (4 * MT)), 1, N), dim3(256), 0, 0, in, w, b, out, res, N, H, W); }, out, N, H, W, ref.data(), fm)
  T1E(2, 2); T1E(1, 2);
  T3(2, 2, 4); T3(1, 2, 4); T3(1, 2, 8); T3(2, 2, 8); T3(4, 2, 4);
  T1E(2, 2); T3(1, 2, 4);
  return 0;
}

