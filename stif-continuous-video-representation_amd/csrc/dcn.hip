// Modulated deformable convolution (DCNv2) for gfx950.
//
// 1. k_dcn: the fused STIF path (64 -> 64, 3x3, stride 1, pad 1, 8 deformable groups).
//    Reference: DCN_sep.forward (DCNv2/dcn_v2.py:127-140) -> dcn_v2_cuda_forward
//    (src/cuda/dcn_v2_cuda.cu:42-172) = im2col into an HBM columns buffer + batched
//    SGEMM.  Here each workgroup owns 4 rows x 32 columns of output pixels; for each
//    deformable group (= 8 input channels = one K chunk) it bilinearly samples the
//    group's 9 taps straight into an LDS A-tile (semantics of
//    modulated_deformable_im2col_gpu_kernel / dmcn_im2col_bilinear,
//    dcn_v2_im2col_cuda.cu:25-54,125-195), stages the group's weight slice, and
//    contracts with fp32 MFMA.  The columns buffer never exists.
// 2. stif_dcn_v2_forward: drop-in for `_ext.dcn_v2_forward` (NCHW, any shape): the STIF shape
//    runs k_dcn between NCHW <-> NHWC transposes (weights packed on the device); any other shape
//    an im2col kernel into a caller workspace + an fp32-MFMA GEMM with fused bias, per sample.
#include "stif_common.h"
#include "tuning.h"
#include "stif.h"
#include "abi_util.h"


namespace {

constexpr int OMC = 216;  // offmask channels per pixel: [group][tap][dy, dx, mask]

STIF_DEV f32x4 dcn_sample4(const float* __restrict__ img, int H, int W, float h, float w, int coff) {
  // dmcn_im2col_bilinear (dcn_v2_im2col_cuda.cu:25-54) on 4 channels of an NHWC 64-ch map.
  const int h_low = (int)floorf(h);
  const int w_low = (int)floorf(w);
  const int h_high = h_low + 1, w_high = w_low + 1;
  const float lh = h - (float)h_low, lw = w - (float)w_low;
  const float hh = 1.f - lh, hw = 1.f - lw;
  f32x4 v1 = f32x4{0}, v2 = f32x4{0}, v3 = f32x4{0}, v4 = f32x4{0};
  if (h_low >= 0 && w_low >= 0) v1 = ld4(img + ((size_t)h_low * W + w_low) * 64 + coff);
  if (h_low >= 0 && w_high <= W - 1) v2 = ld4(img + ((size_t)h_low * W + w_high) * 64 + coff);
  if (h_high <= H - 1 && w_low >= 0) v3 = ld4(img + ((size_t)h_high * W + w_low) * 64 + coff);
  if (h_high <= H - 1 && w_high <= W - 1) v4 = ld4(img + ((size_t)h_high * W + w_high) * 64 + coff);
  const float w1 = hh * hw, w2 = hh * lw, w3 = lh * hw, w4 = lh * lw;
  return w1 * v1 + w2 * v2 + w3 * v3 + w4 * v4;
}

// Workgroup: DCN_ROWS waves, MR output rows x 32 px per wave, all 64 output channels.  Per deformable
// group (= 8 input channels = one K chunk): the group's input tile with an M-pixel margin around the
// 3x3 footprint ([row][channel half][col][4], zero-filled outside the frame) and the group's
// weight fragments are LDS-DMA'd one chunk ahead (double-buffered).  Each lane then bilinearly
// samples its own MFMA A-fragment (pixel = lane & 31, channels 4h..4h+3) tap by tap from the
// tile -- falling back to global loads only when an offset leaves the margin -- so sampling
// (VALU + LDS) interleaves with the MFMAs and no sampled A tile ever round-trips memory.
// F16: the contraction on split-fp16 MFMA (stif_common.h split_f16x3): two taps per 32x32x16 MFMA,
// lane half h sampling tap 2p + h (tap 9 = 0) for all 8 channels of the group (elements 0..7), so
// each (pixel, tap) computes its bilinear weights once; weights packed STIF_PACK_PLAIN |
// STIF_PACK_F16X3 ([group][pair][nt][plane][lane][8 halves]).  On large maps each wave owns MR = 2
// output rows (two M-tiles): every B fragment read from LDS feeds both rows' MFMAs, which halves the
// weight traffic through LDS (the bilinear corner reads at data-dependent addresses conflict) and
// stages fewer halo pixels per output (with 8 waves: C0 L1 shape 342 -> 322 us); small maps keep
// MR = 1, where the halved grid would leave CUs idle.  The kernel is latency-bound (waves parked on
// memory waits and group barriers 43 % of their cycles, profiles/r02_dcn_sq_c0l1.txt), so two
// independent 4-wave workgroups per CU beat one 8-wave workgroup.
constexpr int DCN_ROWS = DCN_TH;   // waves per workgroup

// MR: output rows per wave (2 only with F16; the launcher picks it by grid size, see stif_dcn_nhwc)
template <int EPI, int F16, int MR = 1>
__global__ __launch_bounds__(64 * DCN_ROWS) void k_dcn(stif_dcn_args a) {
  static_assert(MR == 1 || F16, "two rows per wave: split-fp16 path only");
  constexpr int NW = DCN_ROWS, TH = NW * MR, M = DCN_M;
  constexpr int TR = TH + 2 + 2 * M, TC = 32 + 2 + 2 * M;   // tile rows / cols
  constexpr int TP = TC;                                     // column pitch of the staged tile (16-B slots)
  constexpr int T_EL = TR * 2 * TP;                          // 16-B elements
  constexpr int T_INST = (T_EL + 63) / 64;
  constexpr int T_F = T_INST * 256;
  constexpr int W_F = F16 ? 5 * 2 * 2 * 256 : 9 * 2 * 64 * 4;   // packed B fragments of one group
  constexpr int BUF_F = T_F + W_F;
  __shared__ __attribute__((aligned(16))) float smem[2 * BUF_F];

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, l32 = lane & 31, hf = lane >> 5;
  const int H = a.H, W = a.W;
  const int tiles_x = (W + 31) >> 5;
  const int bx = blockIdx.x;
  const int tx = bx % tiles_x, ty = bx / tiles_x;
  const int g = blockIdx.z / a.nitems, n = blockIdx.z - g * a.nitems;
  const float* in = a.in[g] + (size_t)n * a.in_item;
  const float* om = a.offmask[g] + (size_t)n * a.om_item;
  const float* wt = a.w[g];
  const int oy0 = ty * TH, ox0 = tx * 32;
  const int ty0 = oy0 - 1 - M, tx0 = ox0 - 1 - M;           // tile origin (frame coords)
  const int ox = ox0 + l32;                                  // this lane's output column
  int oy[MR];
  bool pix_ok[MR];
  const float* omp[MR];
#pragma unroll
  for (int mr = 0; mr < MR; ++mr) {                          // this wave's output rows
    oy[mr] = oy0 + wv * MR + mr;
    pix_ok[mr] = oy[mr] < H && ox < W;
    omp[mr] = om + ((size_t)min(oy[mr], H - 1) * W + min(ox, W - 1)) * OMC;
  }
  const __amdgpu_buffer_rsrc_t rin =
      __builtin_amdgcn_make_buffer_rsrc((void*)in, (short)0, (int)((size_t)H * W * 64 * 4), 0x00020000);

  auto stage = [&](int dg, int buf) {
    float* st = smem + buf * BUF_F;
    float* sw = st + T_F;
    for (int i = wv; i < T_INST; i += NW) {
      const int e = i * 64 + lane;
      const int col = e % TP, rh = e / TP, h = rh & 1, row = rh >> 1;
      const int y = ty0 + row, x = tx0 + col;
      const bool ok = e < T_EL && col < TC && y >= 0 && y < H && x >= 0 && x < W;
      const unsigned voff = ok ? (unsigned)((((size_t)y * W + x) * 64 + dg * 8 + h * 4) * 4) : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rin, st + i * 256, 16, voff, 0, 0, 0);
    }
    const float* wc = wt + (size_t)dg * W_F;   // packed [chunk][tap][nt][lane][4]
    for (int i = wv; i < W_F / 256; i += NW)
      __builtin_amdgcn_global_load_lds(wc + (i * 64 + lane) * 4, sw + i * 256, 16, 0, 0);
  };
  // offset/mask values of a group: all 27 (fp32 path), or (F16) the 5 taps 2p + h of this lane half
  // as [p][dy, dx, m] (tap 9 reads tap 8's values and is masked off)
  constexpr int NOM = F16 ? 15 : 27;
  auto om_load = [&](int dgi, int mr, float* o) {
#pragma unroll
    for (int k = 0; k < NOM; ++k) o[k] = omp[mr][dgi * 27 + k];
  };
  // F16 variant: a group's 27 offset/mask floats (108 B, dword-aligned) as 6 x 16-B + 1 x 12-B loads
  // per lane instead of 15 scalar loads; lane half h picks its taps 2p + h at the group switch
  typedef float f32x4u __attribute__((ext_vector_type(4), aligned(4)));
  typedef float f32x3u __attribute__((ext_vector_type(3), aligned(4)));
  auto om_raw = [&](int dgi, int mr, float* r) {
    const float* p = omp[mr] + dgi * 27;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const f32x4u v = *reinterpret_cast<const f32x4u*>(p + 4 * i);
      r[4 * i] = v[0]; r[4 * i + 1] = v[1]; r[4 * i + 2] = v[2]; r[4 * i + 3] = v[3];
    }
    const f32x3u v = *reinterpret_cast<const f32x3u*>(p + 24);
    r[24] = v[0]; r[25] = v[1]; r[26] = v[2];
  };
  auto om_pick = [&](const float* r, float* o) {
#pragma unroll
    for (int k = 0; k < 15; ++k) {
      const int i0 = 6 * (k / 3) + k % 3;
      o[k] = (k < 12 && hf) ? r[i0 + 3] : r[i0];
    }
  };
  float omr[MR][27];
  float omc[MR][NOM], omn[MR][NOM];
#pragma unroll
  for (int mr = 0; mr < MR; ++mr) {
    if constexpr (F16) {
      om_raw(0, mr, omr[mr]);
      om_pick(omr[mr], omc[mr]);
    } else {
      om_load(0, mr, omc[mr]);
    }
  }

  // bilinear sample (dmcn_im2col_bilinear semantics) of 8 channels (F16: a0 = channels 0-3, a1 = 4-7)
  // or of this lane half's 4 channels (fp32: a0) at tap `tap` of row mr, with the mask folded into
  // the corner weights and the `> -1` / `< H` gate; global-load fallback outside the staged margin
  auto sample = [&](const float* st, int dg, int mr, int tap, const float* oc, f32x4& a0, f32x4& a1) {
    const int ky = tap / 3, kx = tap - 3 * ky;
    const float h_im = (float)(oy[mr] - 1 + ky) + oc[0];
    const float w_im = (float)(ox - 1 + kx) + oc[1];
    const bool valid = pix_ok[mr] & (tap < 9) & (h_im > -1.f) & (w_im > -1.f) & (h_im < (float)H) & (w_im < (float)W);
    const float fh = floorf(h_im), fw = floorf(w_im);
    const float lh = h_im - fh, lw = w_im - fw, hh = 1.f - lh, hw = 1.f - lw;
    const int h_low = (int)fh, w_low = (int)fw;
    const int r0 = h_low - ty0, c0 = w_low - tx0;
    const bool in_tile = ((unsigned)r0 < (unsigned)(TR - 1)) & ((unsigned)c0 < (unsigned)(TC - 1));
    const float m = valid ? oc[2] : 0.f;
    const float hm = hh * m, lm = lh * m;
    const float w1 = hm * hw, w2 = hm * lw, w3 = lm * hw, w4 = lm * lw;
    const int hsel = F16 ? 0 : hf;
    const float* p0 = st + (((in_tile ? r0 : 0) * 2 + hsel) * TP + (in_tile ? c0 : 0)) * 4;
    const float* p1 = p0 + 2 * TP * 4;                                                 // next row
    a0 = w1 * ld4(p0) + w2 * ld4(p0 + 4) + w3 * ld4(p1) + w4 * ld4(p1 + 4);
    if (F16) a1 = w1 * ld4(p0 + TP * 4) + w2 * ld4(p0 + TP * 4 + 4) + w3 * ld4(p1 + TP * 4) + w4 * ld4(p1 + TP * 4 + 4);
    const bool fb = valid & !in_tile;
    if (__builtin_amdgcn_ballot_w64(fb)) {
      if (fb) {
        const int h_high = h_low + 1, w_high = w_low + 1, co = dg * 8 + hsel * 4;
        const bool b1 = h_low >= 0 && w_low >= 0, b2 = h_low >= 0 && w_high <= W - 1;
        const bool b3 = h_high <= H - 1 && w_low >= 0, b4 = h_high <= H - 1 && w_high <= W - 1;
        const float* q1 = in + ((size_t)h_low * W + w_low) * 64 + co;
        const float* q2 = in + ((size_t)h_low * W + w_high) * 64 + co;
        const float* q3 = in + ((size_t)h_high * W + w_low) * 64 + co;
        const float* q4 = in + ((size_t)h_high * W + w_high) * 64 + co;
        const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
        a0 = w1 * (b1 ? ld4(q1) : z) + w2 * (b2 ? ld4(q2) : z) + w3 * (b3 ? ld4(q3) : z) + w4 * (b4 ? ld4(q4) : z);
        if (F16)
          a1 = w1 * (b1 ? ld4(q1 + 4) : z) + w2 * (b2 ? ld4(q2 + 4) : z) + w3 * (b3 ? ld4(q3 + 4) : z) +
               w4 * (b4 ? ld4(q4 + 4) : z);
      }
    }
  };

  f32x16 acc0[MR], acc1[MR];
#pragma unroll
  for (int mr = 0; mr < MR; ++mr) acc0[mr] = acc1[mr] = f32x16{0};
  stage(0, 0);
  lds_dma_barrier();
  for (int dg = 0; dg < 8; ++dg) {
    if (dg + 1 < 8) {
      stage(dg + 1, (dg + 1) & 1);
#pragma unroll
      for (int mr = 0; mr < MR; ++mr) {
        if constexpr (F16) om_raw(dg + 1, mr, omr[mr]);
        else om_load(dg + 1, mr, omn[mr]);
      }
    }
    const float* st = smem + (dg & 1) * BUF_F;
    const float* sw = st + T_F;
    if constexpr (F16) {
      // tap pair p: lane half h samples tap 2p + h for all 8 channels of the group -- one bilinear
      // weight set per (pixel, tap) -- and supplies them as the 8 K values of its MFMA A operand; the
      // pair's B fragments (read once) feed both rows
#pragma unroll
      for (int pp = 0; pp < 5; ++pp) {
        f16x8 ah[MR], al[MR];
#pragma unroll
        for (int mr = 0; mr < MR; ++mr) {
          f32x4 a0, a1;
          sample(st, dg, mr, 2 * pp + hf, omc[mr] + pp * 3, a0, a1);
          split_f16x3(a0, a1, ah[mr], al[mr]);
        }
        const float* wp = sw + pp * 1024 + lane * 4;   // [pair][nt][plane][lane][8 halves]
        const f16x8 bh0 = ldh8(wp), bl0 = ldh8(wp + 256), bh1 = ldh8(wp + 512), bl1 = ldh8(wp + 768);
#pragma unroll
        for (int mr = 0; mr < MR; ++mr) {
          acc0[mr] = mfma16h(ah[mr], bh0, acc0[mr]);
          acc1[mr] = mfma16h(ah[mr], bh1, acc1[mr]);
          acc0[mr] = mfma16h(ah[mr], bl0, acc0[mr]);
          acc1[mr] = mfma16h(ah[mr], bl1, acc1[mr]);
          acc0[mr] = mfma16h(al[mr], bh0, acc0[mr]);
          acc1[mr] = mfma16h(al[mr], bh1, acc1[mr]);
        }
      }
    } else {
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        // modulated_deformable_im2col (dcn_v2_im2col_cuda.cu:158-192) for this lane's pixel / tap
        f32x4 av, unused;
        sample(st, dg, 0, tap, omc[0] + tap * 3, av, unused);
        const f32x4 b0 = ld4(sw + ((tap * 2 + 0) * 64 + lane) * 4);
        const f32x4 b1 = ld4(sw + ((tap * 2 + 1) * 64 + lane) * 4);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          acc0[0] = mfma32(av[q], b0[q], acc0[0]);
          acc1[0] = mfma32(av[q], b1[q], acc1[0]);
        }
      }
    }
    if (dg + 1 < 8) {
#pragma unroll
      for (int mr = 0; mr < MR; ++mr) {
        if constexpr (F16) {
          om_pick(omr[mr], omc[mr]);
        } else {
#pragma unroll
          for (int k = 0; k < NOM; ++k) omc[mr][k] = omn[mr][k];
        }
      }
    }
    lds_dma_barrier();
  }
  // epilogue through a per-wave LDS block -> coalesced 16-B stores (see tile_to_lds)
  float* out = a.out[g] + (size_t)n * a.out_item;
  const float* bias = a.bias[g];
  float* blk = smem + wv * 1024;
  const int rpx = lane >> 3, c4 = lane & 7;
#pragma unroll
  for (int mr = 0; mr < MR; ++mr) {
    const int y = oy[mr];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const float bv = bias[nt * 32 + l32];
      f32x16 v;
      bool bad = false;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float t = (nt ? acc1[mr][r] : acc0[mr][r]) * (F16 ? F16X3_UNSCALE : 1.f) + bv;
        if (F16) bad |= not_finite(t);
        if (EPI == STIF_EPI_LRELU) t = lrelu01(t);
        v[r] = t;
      }
      if (F16) report_range(a.status, bad);
      tile_to_lds(blk, v, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int px = i * 8 + rpx, x = ox0 + px;
        const f32x4 o = lds_row4(blk, px, c4);
        if (y < H && x < W) st4(out + ((size_t)y * W + x) * 64 + nt * 32 + c4 * 4, o);
      }
    }
  }
}

// ------------------------------------------------------------------ generic drop-in path
// columns[b][c*K + k][ho*Wo + wo], exactly the reference's im2col layout (dcn_v2_cuda.cu:90).
__global__ __launch_bounds__(256) void k_im2col(const float* __restrict__ im, const float* __restrict__ off,
                                                const float* __restrict__ msk, float* __restrict__ col,
                                                int B, int C, int H, int W, int Ho, int Wo, int kh, int kw,
                                                int sh, int sw, int ph, int pw, int dh, int dw, int dg) {
  const long long n = (long long)B * C * Ho * Wo;
  const int K = kh * kw;
  const int cpg = C / dg;
  for (long long idx = (long long)blockIdx.x * 256 + threadIdx.x; idx < n; idx += (long long)gridDim.x * 256) {
    const int wo = (int)(idx % Wo);
    const int ho = (int)((idx / Wo) % Ho);
    const int c = (int)((idx / ((long long)Wo * Ho)) % C);
    const int b = (int)(idx / ((long long)Wo * Ho * C));
    const int g = c / cpg;
    const int h_in = ho * sh - ph, w_in = wo * sw - pw;
    const float* img = im + ((size_t)b * C + c) * H * W;
    const float* o = off + ((size_t)b * dg + g) * 2 * K * Ho * Wo;
    const float* m = msk + ((size_t)b * dg + g) * K * Ho * Wo;
    float* cp = col + (((size_t)b * C + c) * K) * Ho * Wo + (size_t)ho * Wo + wo;
    for (int i = 0; i < kh; ++i)
      for (int j = 0; j < kw; ++j) {
        const int k = i * kw + j;
        const float oh = o[((size_t)2 * k * Ho + ho) * Wo + wo];
        const float ow = o[((size_t)(2 * k + 1) * Ho + ho) * Wo + wo];
        const float mk = m[((size_t)k * Ho + ho) * Wo + wo];
        const float h = (float)(h_in + i * dh) + oh;
        const float w = (float)(w_in + j * dw) + ow;
        float val = 0.f;
        if (h > -1.f && w > -1.f && h < (float)H && w < (float)W) {
          const int h_low = (int)floorf(h), w_low = (int)floorf(w);
          const int h_high = h_low + 1, w_high = w_low + 1;
          const float lh = h - (float)h_low, lw = w - (float)w_low, hh = 1.f - lh, hw = 1.f - lw;
          const float v1 = (h_low >= 0 && w_low >= 0) ? img[(size_t)h_low * W + w_low] : 0.f;
          const float v2 = (h_low >= 0 && w_high <= W - 1) ? img[(size_t)h_low * W + w_high] : 0.f;
          const float v3 = (h_high <= H - 1 && w_low >= 0) ? img[(size_t)h_high * W + w_low] : 0.f;
          const float v4 = (h_high <= H - 1 && w_high <= W - 1) ? img[(size_t)h_high * W + w_high] : 0.f;
          val = hh * hw * v1 + hh * lw * v2 + lh * hw * v3 + lh * lw * v4;
        }
        cp[(size_t)k * Ho * Wo] = val * mk;
      }
  }
}

// out[b][m][p] = bias[m] + sum_k A[m][k] * Bm[b][k][p]   (fp32 MFMA, 64x64 tile per workgroup)
__global__ __launch_bounds__(256) void k_gemm_bias(const float* __restrict__ A, const float* __restrict__ Bm,
                                                   const float* __restrict__ bias, float* __restrict__ out,
                                                   int M, int K, int N) {
  constexpr int LS = 12;
  __shared__ __attribute__((aligned(16))) float sA[64 * LS];
  __shared__ __attribute__((aligned(16))) float sB[64 * LS];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, l32 = lane & 31, hf = lane >> 5;
  const int m0 = blockIdx.y * 64, p0 = blockIdx.x * 64, b = blockIdx.z;
  const float* Bb = Bm + (size_t)b * K * N;
  const int mi = wv >> 1, ni = wv & 1;
  f32x16 acc = f32x16{0};
  for (int k0 = 0; k0 < K; k0 += 8) {
    for (int e = tid; e < 512; e += 256) {
      const int r = e >> 3, kk = e & 7;   // A: row r, k kk
      const int m = m0 + r, k = k0 + kk;
      sA[r * LS + kk] = (m < M && k < K) ? A[(size_t)m * K + k] : 0.f;
      const int kb = e >> 6, p = e & 63;  // B: k kb, col p
      const int kq = k0 + kb, pp = p0 + p;
      sB[p * LS + kb] = (kq < K && pp < N) ? Bb[(size_t)kq * N + pp] : 0.f;
    }
    __syncthreads();
    const f32x4 av = ld4(sA + (mi * 32 + l32) * LS + hf * 4);
    const f32x4 bv = ld4(sB + (ni * 32 + l32) * LS + hf * 4);
#pragma unroll
    for (int q = 0; q < 4; ++q) acc = mfma32(av[q], bv[q], acc);
    __syncthreads();
  }
  const int p = p0 + ni * 32 + l32;
  if (p >= N) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + mi * 32 + mfma_row(r, lane);
    if (m < M) out[((size_t)b * M + m) * N + p] = acc[r] + bias[m];
  }
}

// ------------------------------------------------------------------ drop-in, STIF shape
// [R][Cc] -> [Cc][R] per batch item (NCHW <-> NHWC of one item), 32 x 32 tiles through LDS
__global__ __launch_bounds__(256) void k_transpose(const float* __restrict__ src, float* __restrict__ dst, int R, int Cc) {
  __shared__ float t[32][33];
  const int b = blockIdx.z;
  const float* s = src + (size_t)b * R * Cc;
  float* d = dst + (size_t)b * R * Cc;
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 32 x 8
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int r = r0 + ty + 8 * k, c = c0 + tx;
    t[ty + 8 * k][tx] = (r < R && c < Cc) ? s[(size_t)r * Cc + c] : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = c0 + ty + 8 * k, r = r0 + tx;
    if (c < Cc && r < R) d[(size_t)c * R + r] = t[tx][ty + 8 * k];
  }
}

// offset [b][8*18][HW] + mask [b][8*9][HW] (NCHW, reference channel order: offset (g, tap k) at
// g*18 + 2k (+1 for w), mask at g*9 + k; dcn_v2_im2col_cuda.cu:160-167) -> the fused kernel's offmask
// [b][HW][216] = [group][tap][dy, dx, mask], 64 pixels per workgroup through LDS
__global__ __launch_bounds__(256) void k_offmask_nchw(const float* __restrict__ off, const float* __restrict__ msk,
                                                      float* __restrict__ om, int HW) {
  __shared__ float t[64 * 217];
  const int b = blockIdx.y, p0 = blockIdx.x * 64;
  const float* ob = off + (size_t)b * 144 * HW;
  const float* mb = msk + (size_t)b * 72 * HW;
  for (int i = threadIdx.x; i < 216 * 64; i += 256) {
    const int j = i >> 6, px = i & 63, p = p0 + px;   // packed channel j, pixel
    const int g = j / 27, k = (j % 27) / 3, e = j % 3;
    float v = 0.f;
    if (p < HW) v = e < 2 ? ob[(size_t)(g * 18 + 2 * k + e) * HW + p] : mb[(size_t)(g * 9 + k) * HW + p];
    t[px * 217 + j] = v;
  }
  __syncthreads();
  float* ow = om + ((size_t)b * HW + p0) * 216;
  const int npx = min(64, HW - p0);
  for (int i = threadIdx.x; i < npx * 216; i += 256) ow[i] = t[(i / 216) * 217 + i % 216];
}

// nn.Conv2d weight [64][64][3][3] + bias -> the STIF_PACK_PLAIN layout k_dcn<.., 0> reads:
// [chunk 8][tap 9][nt 2][lane 64][4], lane l of nt = cout nt*32 + (l & 31), channels chunk*8 + 4(l >> 5) + e
__global__ __launch_bounds__(256) void k_pack_dcn_w(const float* __restrict__ w, const float* __restrict__ b,
                                                    float* __restrict__ wp, float* __restrict__ bp) {
  const int i = blockIdx.x * 256 + threadIdx.x;   // 8 * 9 * 2 * 64 * 4 = 36864
  if (i < 36864) {
    const int e = i & 3, l = (i >> 2) & 63, nt = (i >> 8) & 1, t = (i >> 9) % 9, c = (i >> 9) / 9;
    const int co = nt * 32 + (l & 31), ci = c * 8 + 4 * (l >> 5) + e;
    wp[i] = w[(co * 64 + ci) * 9 + t];
  }
  if (i < 64) bp[i] = b[i];
}

// ------------------------------------------------------------------ backward (drop-in _ext.dcn_v2_backward)
// C[m][n] = sum_k A(m, k) B(k, n) (+ C[m][n] when acc): A(m, k) = A[m sam + k sak], B(k, n) = B[k sbk + n sbn];
// 64 x 64 tile per workgroup on fp32 MFMA (exact fp32 products, fp32 sums); the tile loads follow the
// unit-stride dimension of each operand so they coalesce.
__global__ __launch_bounds__(256) void k_sgemm(const float* __restrict__ A, long long sam, long long sak,
                                               const float* __restrict__ Bm, long long sbk, long long sbn,
                                               float* __restrict__ Cm, long long ldc, int M, int N, int K, int acc_c) {
  constexpr int LS = 12;
  __shared__ __attribute__((aligned(16))) float sA[64 * LS];
  __shared__ __attribute__((aligned(16))) float sB[64 * LS];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, l32 = lane & 31, hf = lane >> 5;
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  const int mi = wv >> 1, ni = wv & 1;
  const bool a_m = sam == 1, b_n = sbn == 1;
  f32x16 acc = f32x16{0};
  for (int k0 = 0; k0 < K; k0 += 8) {
    for (int e = tid; e < 512; e += 256) {
      const int r = a_m ? (e & 63) : (e >> 3), kk = a_m ? (e >> 6) : (e & 7);
      const int m = m0 + r, k = k0 + kk;
      sA[r * LS + kk] = (m < M && k < K) ? A[(long long)m * sam + (long long)k * sak] : 0.f;
      const int c = b_n ? (e & 63) : (e >> 3), kb = b_n ? (e >> 6) : (e & 7);
      const int n = n0 + c, kq = k0 + kb;
      sB[c * LS + kb] = (kq < K && n < N) ? Bm[(long long)kq * sbk + (long long)n * sbn] : 0.f;
    }
    __syncthreads();
    const f32x4 av = ld4(sA + (mi * 32 + l32) * LS + hf * 4);
    const f32x4 bv = ld4(sB + (ni * 32 + l32) * LS + hf * 4);
#pragma unroll
    for (int q = 0; q < 4; ++q) acc = mfma32(av[q], bv[q], acc);
    __syncthreads();
  }
  const int n = n0 + ni * 32 + l32;
  if (n >= N) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + mi * 32 + mfma_row(r, lane);
    if (m < M) {
      float* c = Cm + (long long)m * ldc + n;
      *c = acc_c ? *c + acc[r] : acc[r];
    }
  }
}

struct DcnGeom {
  int C, H, W, Ho, Wo, kh, kw, sh, sw, ph, pw, dh, dw, dg;
};

// sampling position of tap k at output pixel p and its (-1, H) x (-1, W) gate (dcn_v2_im2col_cuda.cu:173-176)
STIF_DEV bool dcn_pos(const DcnGeom& G, const float* off, int g, int k, int p, float& h, float& w) {
  const int K = G.kh * G.kw, P = G.Ho * G.Wo;
  const int ho = p / G.Wo, wo = p - ho * G.Wo, i = k / G.kw, j = k - i * G.kw;
  h = (float)(ho * G.sh - G.ph + i * G.dh) + off[((size_t)g * 2 * K + 2 * k) * P + p];
  w = (float)(wo * G.sw - G.pw + j * G.dw) + off[((size_t)g * 2 * K + 2 * k + 1) * P + p];
  return h > -1.f && w > -1.f && h < (float)G.H && w < (float)G.W;
}

// grad_offset / grad_mask of one sample (modulated_deformable_col2im_coord, dcn_v2_im2col_cuda.cu:256-327):
// one thread per (group, tap, pixel) computes both coordinate gradients and the mask gradient in one
// pass over the group's channels (the reference runs one thread per offset channel)
__global__ __launch_bounds__(256) void k_dcn_bwd_coord(const float* __restrict__ colg, const float* __restrict__ im,
                                                       const float* __restrict__ off, const float* __restrict__ msk,
                                                       float* __restrict__ goff, float* __restrict__ gmsk, DcnGeom G) {
  const int K = G.kh * G.kw, P = G.Ho * G.Wo, cpg = G.C / G.dg;
  const long long n = (long long)G.dg * K * P;
  for (long long idx = (long long)blockIdx.x * 256 + threadIdx.x; idx < n; idx += (long long)gridDim.x * 256) {
    const int p = (int)(idx % P), k = (int)((idx / P) % K), g = (int)(idx / ((long long)P * K));
    float h, w, vh = 0.f, vw = 0.f, vm = 0.f;
    if (dcn_pos(G, off, g, k, p, h, w)) {
      const int hl = (int)floorf(h), wl = (int)floorf(w);
      const float lh = h - (float)hl, lw = w - (float)wl, hh = 1.f - lh, hw = 1.f - lw;
      const bool b1 = hl >= 0 && wl >= 0, b2 = hl >= 0 && wl + 1 <= G.W - 1;
      const bool b3 = hl + 1 <= G.H - 1 && wl >= 0, b4 = hl + 1 <= G.H - 1 && wl + 1 <= G.W - 1;
      const size_t o1 = (size_t)hl * G.W + wl;
      for (int c = 0; c < cpg; ++c) {
        const float* img = im + (size_t)(g * cpg + c) * G.H * G.W;
        const float v1 = b1 ? img[o1] : 0.f, v2 = b2 ? img[o1 + 1] : 0.f;
        const float v3 = b3 ? img[o1 + G.W] : 0.f, v4 = b4 ? img[o1 + G.W + 1] : 0.f;
        const float col = colg[((size_t)(g * cpg + c) * K + k) * P + p];
        vh += col * (-hw * v1 - lw * v2 + hw * v3 + lw * v4);
        vw += col * (-hh * v1 + hh * v2 - lh * v3 + lh * v4);
        vm += col * (hh * hw * v1 + hh * lw * v2 + lh * hw * v3 + lh * lw * v4);
      }
    }
    const float m = msk[((size_t)g * K + k) * P + p];
    goff[((size_t)g * 2 * K + 2 * k) * P + p] = vh * m;
    goff[((size_t)g * 2 * K + 2 * k + 1) * P + p] = vw * m;
    gmsk[((size_t)g * K + k) * P + p] = vm;
  }
}

// grad_input of one sample (modulated_deformable_col2im, dcn_v2_im2col_cuda.cu:197-254): col * mask
// added into the in-bounds bilinear corners (hardware fp32 atomics; the reference uses atomicAdd too)
__global__ __launch_bounds__(256) void k_dcn_bwd_col2im(const float* __restrict__ colg, const float* __restrict__ off,
                                                        const float* __restrict__ msk, float* __restrict__ gin,
                                                        DcnGeom G) {
  const int K = G.kh * G.kw, P = G.Ho * G.Wo, cpg = G.C / G.dg;
  const long long n = (long long)G.C * K * P;
  for (long long idx = (long long)blockIdx.x * 256 + threadIdx.x; idx < n; idx += (long long)gridDim.x * 256) {
    const int p = (int)(idx % P), k = (int)((idx / P) % K), c = (int)(idx / ((long long)P * K));
    const int g = c / cpg;
    float h, w;
    if (!dcn_pos(G, off, g, k, p, h, w)) continue;
    const float coef = colg[idx] * msk[((size_t)g * K + k) * P + p];
    const int hl = (int)floorf(h), wl = (int)floorf(w);
    const float lh = h - (float)hl, lw = w - (float)wl, hh = 1.f - lh, hw = 1.f - lw;
    float* gi = gin + (size_t)c * G.H * G.W;
    if (hl >= 0 && wl >= 0) unsafeAtomicAdd(gi + (size_t)hl * G.W + wl, hh * hw * coef);
    if (hl >= 0 && wl + 1 <= G.W - 1) unsafeAtomicAdd(gi + (size_t)hl * G.W + wl + 1, hh * lw * coef);
    if (hl + 1 <= G.H - 1 && wl >= 0) unsafeAtomicAdd(gi + (size_t)(hl + 1) * G.W + wl, lh * hw * coef);
    if (hl + 1 <= G.H - 1 && wl + 1 <= G.W - 1) unsafeAtomicAdd(gi + (size_t)(hl + 1) * G.W + wl + 1, lh * lw * coef);
  }
}

// grad_bias[co] += sum_p grad_out[co][p] of one sample (dcn_v2_cuda.cu:320-326); one workgroup per co
__global__ __launch_bounds__(256) void k_dcn_bwd_bias(const float* __restrict__ go, float* __restrict__ gb, int P) {
  __shared__ float red[256];
  const int co = blockIdx.x;
  float s = 0.f;
  for (int p = threadIdx.x; p < P; p += 256) s += go[(size_t)co * P + p];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if (threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x == 0) gb[co] += red[0];
}

bool stif_dcn_shape(int channels, int channels_out, int kh, int kw, int sh, int sw, int ph, int pw, int dh, int dw,
                    int dg, int height, int width) {
  return channels == 64 && channels_out == 64 && kh == 3 && kw == 3 && sh == 1 && sw == 1 && ph == 1 && pw == 1 &&
         dh == 1 && dw == 1 && dg == 8 && (long long)height * width * 216 * 4 < 0x7fffffffLL;
}
constexpr size_t DCN_WPACK = 36864, DCN_BPACK = 64;


}  // namespace

extern "C" int stif_dcn_nhwc(const stif_dcn_args* pa, void* stream) {
  if (!pa) return stif_fail(STIF_E_INVALID, "stif_dcn_nhwc: null args");
  const stif_dcn_args& a = *pa;
  if (a.ngroups < 1 || a.ngroups > STIF_MAX_GROUPS || a.nitems < 1 || a.H < 1 || a.W < 1)
    return stif_fail(STIF_E_INVALID, "stif_dcn_nhwc: bad sizes");
  if ((long long)a.H * a.W * 64 * 4 >= 0x7fffffffLL)
    return stif_fail(STIF_E_INVALID, "stif_dcn_nhwc: item larger than 2 GB (buffer addressing)");
  const bool f16 = a.flags & STIF_CONV_F16X3;
  // two rows per wave (8-row workgroups, two per CU) when that still gives >= 4 workgroups per CU
  const long long wg2 = (long long)((a.W + 31) / 32) * ((a.H + 2 * DCN_ROWS - 1) / (2 * DCN_ROWS)) * a.ngroups * a.nitems;
  const bool mr2 = f16 && wg2 >= DCN_MR2_MIN;
  const int th = DCN_ROWS * (mr2 ? 2 : 1);   // output rows per workgroup
  dim3 grid(((a.W + 31) / 32) * ((a.H + th - 1) / th), 1, a.ngroups * a.nitems);
  if (a.epi == STIF_EPI_LRELU && mr2)
    hipLaunchKernelGGL((k_dcn<STIF_EPI_LRELU, 1, 2>), grid, dim3(64 * DCN_ROWS), 0, (hipStream_t)stream, a);
  else if (a.epi == STIF_EPI_NONE && mr2)
    hipLaunchKernelGGL((k_dcn<STIF_EPI_NONE, 1, 2>), grid, dim3(64 * DCN_ROWS), 0, (hipStream_t)stream, a);
  else if (a.epi == STIF_EPI_LRELU && f16)
    hipLaunchKernelGGL((k_dcn<STIF_EPI_LRELU, 1>), grid, dim3(64 * DCN_ROWS), 0, (hipStream_t)stream, a);
  else if (a.epi == STIF_EPI_NONE && f16)
    hipLaunchKernelGGL((k_dcn<STIF_EPI_NONE, 1>), grid, dim3(64 * DCN_ROWS), 0, (hipStream_t)stream, a);
  else if (a.epi == STIF_EPI_LRELU)
    hipLaunchKernelGGL((k_dcn<STIF_EPI_LRELU, 0>), grid, dim3(64 * DCN_ROWS), 0, (hipStream_t)stream, a);
  else if (a.epi == STIF_EPI_NONE)
    hipLaunchKernelGGL((k_dcn<STIF_EPI_NONE, 0>), grid, dim3(64 * DCN_ROWS), 0, (hipStream_t)stream, a);
  else
    return stif_fail(STIF_E_INVALID, "stif_dcn_nhwc: epilogue must be NONE or LRELU");
  return stif_check_launch("stif_dcn_nhwc");
}

static bool dcn_dims(int H, int W, int kh, int kw, int sh, int sw, int ph, int pw, int dh, int dw, int* Ho,
                     int* Wo) {
  *Ho = (H + 2 * ph - (dh * (kh - 1) + 1)) / sh + 1;
  *Wo = (W + 2 * pw - (dw * (kw - 1) + 1)) / sw + 1;
  return *Ho > 0 && *Wo > 0;
}

extern "C" size_t stif_dcn_v2_workspace_size(int batch, int channels, int height, int width, int channels_out,
                                             int kernel_h, int kernel_w, int stride_h, int stride_w, int pad_h,
                                             int pad_w, int dilation_h, int dilation_w, int deformable_group) {
  int Ho, Wo;
  if (!dcn_dims(height, width, kernel_h, kernel_w, stride_h, stride_w, pad_h, pad_w, dilation_h, dilation_w, &Ho,
                &Wo))
    return 0;
  if (stif_dcn_shape(channels, channels_out, kernel_h, kernel_w, stride_h, stride_w, pad_h, pad_w, dilation_h,
                     dilation_w, deformable_group, height, width))
    return ((size_t)batch * height * width * (64 + 216 + 64) + DCN_WPACK + DCN_BPACK) * sizeof(float);
  // generic: the reference's per-sample columns buffer [c * kh * kw][ho * wo] (dcn_v2_cuda.cu:90, one sample)
  return (size_t)channels * kernel_h * kernel_w * Ho * Wo * sizeof(float);
}

extern "C" int stif_dcn_v2_forward(const float* input, const float* weight, const float* bias, const float* offset,
                                   const float* mask, float* output, int batch, int channels, int height, int width,
                                   int channels_out, int kernel_h, int kernel_w, int stride_h, int stride_w,
                                   int pad_h, int pad_w, int dilation_h, int dilation_w, int deformable_group,
                                   void* workspace, size_t workspace_bytes, void* stream) {
  // argument checks mirror dcn_v2_cuda_forward's AT_ASSERTMs (dcn_v2_cuda.cu:60-84)
  if (!input || !weight || !bias || !offset || !mask || !output)
    return stif_fail(STIF_E_INVALID, "dcn_v2_forward: null tensor");
  if (batch < 1 || channels < 1 || channels_out < 1 || kernel_h < 1 || kernel_w < 1 || stride_h < 1 ||
      stride_w < 1 || dilation_h < 1 || dilation_w < 1 || deformable_group < 1 || channels % deformable_group)
    return stif_fail(STIF_E_INVALID, "dcn_v2_forward: invalid shape arguments");
  int Ho, Wo;
  if (!dcn_dims(height, width, kernel_h, kernel_w, stride_h, stride_w, pad_h, pad_w, dilation_h, dilation_w, &Ho,
                &Wo))
    return stif_fail(STIF_E_INVALID, "dcn_v2_forward: empty output");
  const size_t need = stif_dcn_v2_workspace_size(batch, channels, height, width, channels_out, kernel_h, kernel_w,
                                                 stride_h, stride_w, pad_h, pad_w, dilation_h, dilation_w,
                                                 deformable_group);
  if (!workspace || workspace_bytes < need)
    return stif_fail(STIF_E_WORKSPACE, "dcn_v2_forward: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  if (stif_dcn_shape(channels, channels_out, kernel_h, kernel_w, stride_h, stride_w, pad_h, pad_w, dilation_h,
                     dilation_w, deformable_group, height, width)) {
    // every DCN_sep of LunaTokis: NCHW -> NHWC, offset/mask -> offmask, weights packed on the device,
    // the fused im2col-free kernel (fp32 MFMA), NHWC -> NCHW
    const int HW = height * width;
    float* in_nhwc = (float*)workspace;
    float* om = in_nhwc + (size_t)batch * HW * 64;
    float* out_nhwc = om + (size_t)batch * HW * 216;
    float* wp = out_nhwc + (size_t)batch * HW * 64;
    float* bp = wp + DCN_WPACK;
    hipLaunchKernelGGL(k_transpose, dim3((HW + 31) / 32, 2, batch), dim3(256), 0, st, input, in_nhwc, 64, HW);
    hipLaunchKernelGGL(k_offmask_nchw, dim3((HW + 63) / 64, batch), dim3(256), 0, st, offset, mask, om, HW);
    hipLaunchKernelGGL(k_pack_dcn_w, dim3((unsigned)(DCN_WPACK / 256)), dim3(256), 0, st, weight, bias, wp, bp);
    int rc = stif_check_launch("dcn_v2_forward/layout");
    if (rc) return rc;
    stif_dcn_args a{};
    a.in[0] = in_nhwc;
    a.offmask[0] = om;
    a.w[0] = wp;
    a.bias[0] = bp;
    a.out[0] = out_nhwc;
    a.in_item = (long long)HW * 64;
    a.om_item = (long long)HW * 216;
    a.out_item = (long long)HW * 64;
    a.ngroups = 1;
    a.nitems = batch;
    a.H = height;
    a.W = width;
    a.epi = STIF_EPI_NONE;
    a.flags = 0;
    a.status = nullptr;
    rc = stif_dcn_nhwc(&a, stream);
    if (rc) return rc;
    hipLaunchKernelGGL(k_transpose, dim3(2, (HW + 31) / 32, batch), dim3(256), 0, st, out_nhwc, output, HW, 64);
    return stif_check_launch("dcn_v2_forward/out");
  }
  // any other shape: im2col + GEMM one sample at a time (dcn_v2_cuda_forward's per-sample columns)
  float* cols = (float*)workspace;
  const int K = channels * kernel_h * kernel_w, N = Ho * Wo;
  const long long n = (long long)channels * Ho * Wo;
  long long blocks = (n + 255) / 256;
  if (blocks > 1 << 20) blocks = 1 << 20;
  for (int b = 0; b < batch; ++b) {
    hipLaunchKernelGGL(k_im2col, dim3((unsigned)blocks), dim3(256), 0, st,
                       input + (size_t)b * channels * height * width,
                       offset + (size_t)b * deformable_group * 2 * kernel_h * kernel_w * N,
                       mask + (size_t)b * deformable_group * kernel_h * kernel_w * N, cols, 1, channels, height, width,
                       Ho, Wo, kernel_h, kernel_w, stride_h, stride_w, pad_h, pad_w, dilation_h, dilation_w,
                       deformable_group);
    int rc = stif_check_launch("dcn_v2_forward/im2col");
    if (rc) return rc;
    dim3 grid((N + 63) / 64, (channels_out + 63) / 64, 1);
    hipLaunchKernelGGL(k_gemm_bias, grid, dim3(256), 0, st, weight, cols, bias, output + (size_t)b * channels_out * N,
                       channels_out, K, N);
    rc = stif_check_launch("dcn_v2_forward/gemm");
    if (rc) return rc;
  }
  return STIF_OK;
}

extern "C" size_t stif_dcn_v2_backward_workspace_size(int batch, int channels, int height, int width,
                                                      int channels_out, int kernel_h, int kernel_w, int stride_h,
                                                      int stride_w, int pad_h, int pad_w, int dilation_h,
                                                      int dilation_w, int deformable_group) {
  (void)batch;
  (void)channels_out;
  (void)deformable_group;
  int Ho, Wo;
  if (!dcn_dims(height, width, kernel_h, kernel_w, stride_h, stride_w, pad_h, pad_w, dilation_h, dilation_w, &Ho,
                &Wo))
    return 0;
  // the reference's per-sample columns buffer (dcn_v2_cuda.cu:242): first the columns gradient, then
  // the forward columns for grad_weight
  return (size_t)channels * kernel_h * kernel_w * Ho * Wo * sizeof(float);
}

extern "C" int stif_dcn_v2_backward(const float* input, const float* weight, const float* bias, const float* offset,
                                    const float* mask, const float* grad_output, float* grad_input, float* grad_offset,
                                    float* grad_mask, float* grad_weight, float* grad_bias, int batch, int channels,
                                    int height, int width, int channels_out, int kernel_h, int kernel_w,
                                    int stride_h, int stride_w, int pad_h, int pad_w, int dilation_h, int dilation_w,
                                    int deformable_group, void* workspace, size_t workspace_bytes, void* stream) {
  // argument checks mirror dcn_v2_cuda_backward's (dcn_v2_cuda.cu:216-240)
  if (!input || !weight || !bias || !offset || !mask || !grad_output || !grad_input || !grad_offset || !grad_mask ||
      !grad_weight || !grad_bias)
    return stif_fail(STIF_E_INVALID, "dcn_v2_backward: null tensor");
  if (batch < 1 || channels < 1 || channels_out < 1 || kernel_h < 1 || kernel_w < 1 || stride_h < 1 ||
      stride_w < 1 || dilation_h < 1 || dilation_w < 1 || deformable_group < 1 || channels % deformable_group)
    return stif_fail(STIF_E_INVALID, "dcn_v2_backward: invalid shape arguments");
  int Ho, Wo;
  if (!dcn_dims(height, width, kernel_h, kernel_w, stride_h, stride_w, pad_h, pad_w, dilation_h, dilation_w, &Ho,
                &Wo))
    return stif_fail(STIF_E_INVALID, "dcn_v2_backward: empty output");
  const size_t need = stif_dcn_v2_backward_workspace_size(batch, channels, height, width, channels_out, kernel_h,
                                                          kernel_w, stride_h, stride_w, pad_h, pad_w, dilation_h,
                                                          dilation_w, deformable_group);
  if (!workspace || workspace_bytes < need) return stif_fail(STIF_E_WORKSPACE, "dcn_v2_backward: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const int K = kernel_h * kernel_w, P = Ho * Wo, CK = channels * K;
  const size_t in_n = (size_t)channels * height * width;
  if (hipMemsetAsync(grad_input, 0, (size_t)batch * in_n * sizeof(float), st) != hipSuccess ||
      hipMemsetAsync(grad_weight, 0, (size_t)channels_out * CK * sizeof(float), st) != hipSuccess ||
      hipMemsetAsync(grad_bias, 0, (size_t)channels_out * sizeof(float), st) != hipSuccess)
    return stif_fail(STIF_E_LAUNCH, "dcn_v2_backward: memset failed");
  const DcnGeom G{channels, height, width, Ho, Wo, kernel_h, kernel_w, stride_h, stride_w, pad_h, pad_w,
                  dilation_h, dilation_w, deformable_group};
  float* cols = (float*)workspace;
  auto blocks = [](long long n) { return (unsigned)std::min<long long>((n + 255) / 256, 1 << 20); };
  for (int b = 0; b < batch; ++b) {
    const float* in_b = input + (size_t)b * in_n;
    const float* off_b = offset + (size_t)b * deformable_group * 2 * K * P;
    const float* msk_b = mask + (size_t)b * deformable_group * K * P;
    const float* go_b = grad_output + (size_t)b * channels_out * P;
    // columns gradient [c*K + k][p] = sum_co W[co][c*K + k] grad_out[co][p] (dcn_v2_cuda.cu:274-277)
    hipLaunchKernelGGL(k_sgemm, dim3((P + 63) / 64, (CK + 63) / 64), dim3(256), 0, st, weight, 1LL, (long long)CK,
                       go_b, (long long)P, 1LL, cols, (long long)P, CK, P, channels_out, 0);
    hipLaunchKernelGGL(k_dcn_bwd_coord, dim3(blocks((long long)deformable_group * K * P)), dim3(256), 0, st, cols,
                       in_b, off_b, msk_b, grad_offset + (size_t)b * deformable_group * 2 * K * P,
                       grad_mask + (size_t)b * deformable_group * K * P, G);
    hipLaunchKernelGGL(k_dcn_bwd_col2im, dim3(blocks((long long)CK * P)), dim3(256), 0, st, cols, off_b, msk_b,
                       grad_input + (size_t)b * in_n, G);
    // forward columns, then grad_weight[co][c*K + k] += sum_p grad_out[co][p] cols[c*K + k][p] (:308-315)
    hipLaunchKernelGGL(k_im2col, dim3(blocks((long long)channels * P)), dim3(256), 0, st, in_b, off_b, msk_b, cols, 1,
                       channels, height, width, Ho, Wo, kernel_h, kernel_w, stride_h, stride_w, pad_h, pad_w,
                       dilation_h, dilation_w, deformable_group);
    hipLaunchKernelGGL(k_sgemm, dim3((CK + 63) / 64, (channels_out + 63) / 64), dim3(256), 0, st, go_b, (long long)P,
                       1LL, cols, 1LL, (long long)P, grad_weight, (long long)CK, channels_out, CK, P, 1);
    hipLaunchKernelGGL(k_dcn_bwd_bias, dim3(channels_out), dim3(256), 0, st, go_b, grad_bias, P);
    const int rc = stif_check_launch("dcn_v2_backward");
    if (rc) return rc;
  }
  return STIF_OK;
}
