// Fused DCN_sep for gfx950: conv_offset_mask (64 -> 216, 3x3) + chunk / cat / sigmoid + the
// modulated deformable conv (64 -> 64, 3x3, 8 deformable groups) in one kernel; the 216-channel
// offset/mask map never reaches HBM.
//
// Reference: DCN_sep.forward (DCNv2/dcn_v2.py:127-140) -> _DCNv2 -> dcn_v2_cuda_forward
// (src/cuda/dcn_v2_cuda.cu:42-172) with the sampling of modulated_deformable_im2col_gpu_kernel /
// dmcn_im2col_bilinear (dcn_v2_im2col_cuda.cu:25-54,125-195).
//
// Workgroup = 8 waves, tile = 8 output rows x 32 columns, wave w = output row w (lane & 31 = column).
//
// Phase 1, the offset/mask conv as a direct implicit GEMM with the WEIGHTS as the MFMA A operand:
// D[om row][pixel] += W[om row][k] X[k][pixel] on split-fp16 v_mfma_f32_32x32x16_f16 (f16x3, fp32
// accumulation).  Each deformable group's 27 offset/mask channels are one 32-row block whose rows
// are permuted at packing time (stif_pack_conv_weight, STIF_PACK_DCNSEP) so that the accumulator
// registers of lane (pixel p, half h) hold exactly the (dy, dx, mask) of the taps h, h + 2, ..., h + 8
// that lane half samples in phase 2 -- the offsets go from the MFMA accumulators straight into the
// bilinear sampling, with no exchange, no LDS round trip and no HBM traffic.  K = 36 steps
// (16-channel chunk c, tap t); per step a wave reads its pixels' 8 channels of the staged input
// halo (two ds_read_b128), splits them once and runs 3 MFMAs for each of the 8 groups (24 MFMAs per
// step; 128 accumulator VGPRs).  The input halo (10 x 34 pixels, one 16-channel chunk, 80-B pixel
// pitch: conflict-free reads) and the packed weights of each step (16 KB, a 3-slot ring) arrive by
// LDS-DMA ahead of use; one barrier per step.
//
// Phase 2, k_dcn's sampling + contraction with 8 waves x 1 row: per deformable group the input
// tile with a 2-px margin and the group's weight fragments are LDS-DMA'd one group ahead (group 0
// during phase 1), each lane samples its tap of every tap pair for the group's 8 channels (global
// fallback outside the margin) and runs 3 MFMAs per 32-cout half; epilogue through LDS as k_dcn.
#include "abi_util.h"
#include "stif.h"
#include "stif_common.h"

namespace {

constexpr int NW = 8;                         // waves = output rows per tile
constexpr int TW = 32;                        // output columns per tile
// phase 1
constexpr int HC1 = TW + 2;                   // halo columns (10 halo rows)
constexpr int PX_F = 20;                      // floats per staged halo pixel: 16 channels + 4 pad
constexpr int D_SLOTS = (NW + 2) * HC1 * 5;   // 16-B slots per data chunk (1700)
constexpr int D_INS = 32;                     // DMA instructions per data chunk (4 per wave; 27 carry data)
constexpr int D_F = D_INS * 256;              // floats per data buffer
constexpr int KSTEPS = 36;                    // k = 9 c + t: 16-channel chunk c, tap t
constexpr int WK_F = 8 * 2 * 256;             // packed weights of one step: [group][plane][lane][8 halves]
constexpr int RING = 3;
// phase 2 (k_dcn geometry, MR = 1)
constexpr int M = 2;                          // staged margin around the 3x3 footprint
constexpr int TR = NW + 2 + 2 * M, TC = TW + 2 + 2 * M, TP = TC;
constexpr int T_EL = TR * 2 * TP;             // 16-B elements of the staged tile
constexpr int T_INST = (T_EL + 63) / 64;      // 17
constexpr int T_F = T_INST * 256;
constexpr int W_F = 5 * 2 * 2 * 256;          // packed B fragments of one group
constexpr int G_INS = 40;                     // DMA instructions per group stage (17 tile + 20 weights + 3 pad)
constexpr int G_F = G_INS * 256;
static_assert(T_INST + W_F / 256 <= G_INS && G_INS % NW == 0 && D_INS % NW == 0 && 16 % NW == 0, "stage sizes");
static_assert(D_SLOTS <= D_INS * 64, "data chunk");
// LDS map (floats): [data 0][data 1][weight ring][phase-2 buffer 0]; phase-2 buffer 1 reuses the data
// buffers, the epilogue blocks the ring
constexpr int OFF_D = 0, OFF_W = 2 * D_F, OFF_G0 = OFF_W + RING * WK_F, OFF_G1 = 0;
constexpr int LDS_F = OFF_G0 + G_F;
static_assert(G_F <= 2 * D_F && NW * 1024 <= RING * WK_F && LDS_F * 4 <= 160 * 1024, "LDS map");
constexpr int DCN0_STEP = 28;
#ifndef DCNSEP_EXP
#define DCNSEP_EXP 0    // timing probes (wrong results): 1 no phase 1, 3 no phase 2, 4 no fallback loads
#endif
#ifndef DCNSEP_ROLL
#define DCNSEP_ROLL 0   // 1: phase 2 as a runtime loop over the groups (offsets rotated through registers)
#endif                 // phase-1 step that DMAs phase 2's first group

// vmcnt waits with an immediate operand (the counts are wave-uniform)
STIF_DEV void wait_vm(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}
// side DMA instructions a wave issues at step s after that step's weight DMA: the next data chunk
// (4) at steps 1, 10, 19 and phase 2's first group (5) at DCN0_STEP
STIF_DEV int side_dma(int s) {
  if (s < 0) return 0;
  if (s == DCN0_STEP) return G_INS / NW;
  return (s % 9 == 1 && s / 9 < 3) ? D_INS / NW : 0;
}

template <int EPI>
__global__ __launch_bounds__(64 * NW) void k_dcn_sep(stif_dcn_sep_args a) {
  __shared__ __attribute__((aligned(16))) float smem[LDS_F];
  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, hf = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.H, W = a.W;
  const int tiles_x = (W + TW - 1) / TW, tiles = tiles_x * ((H + NW - 1) / NW);
  // one flat grid over (weight set, item, tile), XCD-aware: each XCD walks a contiguous tile range, so
  // the halos neighbouring tiles share are fetched into one L2
  const int L = xcd_block(blockIdx.x, gridDim.x);
  const int z = L / tiles, tl = L - z * tiles;
  const int tx = tl % tiles_x, ty = tl / tiles_x;
  const int g = z / a.nitems, n = z - g * a.nitems;
  const float* fea = a.fea[g] + (size_t)n * a.fea_item;
  const float* in = a.in[g] + (size_t)n * a.in_item;
  const float* wom = a.w_om[g];
  const float* wt = a.w[g];
  const int oy0 = ty * NW, ox0 = tx * TW;
  const int oy = oy0 + wv, ox = ox0 + l32;
  const bool pix_ok = oy < H && ox < W;
  const unsigned img_bytes = (unsigned)((size_t)H * W * 64 * 4);
  const __amdgpu_buffer_rsrc_t rfea = __builtin_amdgcn_make_buffer_rsrc((void*)fea, (short)0, (int)img_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void*)in, (short)0, (int)img_bytes, 0x00020000);

  // ---------------------------------------------------------------- phase 1: offset/mask conv
  // data chunk c (channels 16c..16c+15) of the 10 x 34 halo: slot s = pixel * 5 + sub (sub 4 = pad)
  auto stage_data = [&](int c, float* dst) {
#pragma unroll
    for (int j = 0; j < D_INS / NW; ++j) {
      const int i = wv + j * NW;
      const int s = i * 64 + lane;
      const int px = s / 5, sub = s - 5 * px;
      const int row = px / HC1, col = px - HC1 * row;
      const int y = oy0 - 1 + row, x = ox0 - 1 + col;
      const bool ok = (s < D_SLOTS) & (sub < 4) & ((unsigned)y < (unsigned)H) & ((unsigned)x < (unsigned)W);
      const unsigned voff = ok ? (unsigned)((((size_t)y * W + x) * 64 + 16 * c + 4 * sub) * 4) : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rfea, dst + i * 256, 16, voff, 0, 0, 0);
    }
  };
  auto stage_w = [&](int k, int slot) {
    const float* src = wom + (size_t)k * WK_F;
    float* dst = smem + OFF_W + slot * WK_F;
#pragma unroll
    for (int j = 0; j < 16 / NW; ++j) {
      const int i = wv + j * NW;
      __builtin_amdgcn_global_load_lds(src + (i * 64 + lane) * 4, dst + i * 256, 16, 0, 0);
    }
  };
  // phase 2 stage of deformable group dg: [row][channel half][col][4] tile + the group's B fragments
  auto stage_group = [&](int dg, float* st) {
    const int ty0 = oy0 - 1 - M, tx0 = ox0 - 1 - M;
    const float* wc = wt + (size_t)dg * W_F;
#pragma unroll
    for (int j = 0; j < G_INS / NW; ++j) {
      const int i = wv + j * NW;   // wave-uniform
      if (i >= T_INST && i < T_INST + W_F / 256) {
        __builtin_amdgcn_global_load_lds(wc + ((i - T_INST) * 64 + lane) * 4, st + i * 256, 16, 0, 0);
      } else {
        const int e = i * 64 + lane;
        const int col = e % TP, rh = e / TP, h = rh & 1, row = rh >> 1;
        const int y = ty0 + row, x = tx0 + col;
        const bool ok = (i < T_INST) & (e < T_EL) & ((unsigned)y < (unsigned)H) & ((unsigned)x < (unsigned)W);
        const unsigned voff = ok ? (unsigned)((((size_t)y * W + x) * 64 + dg * 8 + h * 4) * 4) : 0x80000000u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rin, st + i * 256, 16, voff, 0, 0, 0);
      }
    }
  };

  f32x16 om[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) om[q] = f32x16{0};
#if DCNSEP_EXP == 1   // timing probe: no phase 1 (offsets = biases)
  if (false)
#endif
  {
  stage_data(0, smem + OFF_D);
  stage_w(0, 0);
  stage_w(1, 1);
#pragma unroll 1
  for (int k = 0; k < KSTEPS; ++k) {
    // this step's weights (and, at a chunk start, its data) landed in every wave: the DMA issued in the
    // last two steps may stay in flight
    wait_vm((k + 1 < KSTEPS ? 2 : 0) + side_dma(k - 1) + side_dma(k - 2));
    __syncthreads();
    if (k + 2 < KSTEPS) stage_w(k + 2, (k + 2) % RING);
    if (k % 9 == 1 && k / 9 < 3) stage_data(k / 9 + 1, smem + OFF_D + ((k / 9 + 1) & 1) * D_F);
    if (k == DCN0_STEP) stage_group(0, smem + OFF_G0);
    const int c = k / 9, t = k - 9 * c, ky = t / 3, kx = t - 3 * ky;
    const float* db = smem + OFF_D + (c & 1) * D_F + ((wv + ky) * HC1 + l32 + kx) * PX_F + hf * 8;
    f16x8 dh, dl;
    split_f16x3(ld4(db), ld4(db + 4), dh, dl);
    const float* wb = smem + OFF_W + (k % RING) * WK_F + lane * 4;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const f16x8 wh = ldh8(wb + (2 * q) * 256), wl = ldh8(wb + (2 * q + 1) * 256);
      om[q] = mfma16h(wh, dh, om[q]);
      om[q] = mfma16h(wh, dl, om[q]);
      om[q] = mfma16h(wl, dh, om[q]);
    }
  }
  }
#if DCNSEP_EXP == 1
  stage_group(0, smem + OFF_G0);
#endif
  // om[q][r] of lane (p, h): packed row (r & 3) + 8 (r >> 2) + 4 h of group q = component r % 3 (dy, dx,
  // mask) of tap 2 (r / 3) + h (r < 15); bias, unscale, sigmoid(mask) (dcn_v2.py:134-138)
  bool bad = false;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const f32x4 bq = ld4(a.b_om[g] + q * 32 + 8 * v + 4 * hf);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = 4 * v + e;
        if (r < 15) {
          float x = om[q][r] * F16X3_UNSCALE + bq[e];
          bad |= not_finite(x);
          if (r % 3 == 2) x = sigmoid_fast(x);
          om[q][r] = x;
        }
      }
    }
  }
  report_range(a.status, bad);

  // ---------------------------------------------------------------- phase 2: deformable conv
  const int ty0 = oy0 - 1 - M, tx0 = ox0 - 1 - M;
  // bilinear sample of the group's 8 channels (a0: 0-3, a1: 4-7) at tap `tap` with offset (dy, dx) and
  // modulation m folded into the corner weights; `> -1` / `< H` gate; global fallback outside the tile
  auto sample = [&](const float* st, int dg, int tap, float dy, float dx, float mk, f32x4& a0, f32x4& a1) {
    const int ky = tap / 3, kx = tap - 3 * ky;
    const float h_im = (float)(oy - 1 + ky) + dy;
    const float w_im = (float)(ox - 1 + kx) + dx;
    const bool valid = pix_ok & (tap < 9) & (h_im > -1.f) & (w_im > -1.f) & (h_im < (float)H) & (w_im < (float)W);
    const float fh = floorf(h_im), fw = floorf(w_im);
    const float lh = h_im - fh, lw = w_im - fw, hh = 1.f - lh, hw = 1.f - lw;
    const int h_low = (int)fh, w_low = (int)fw;
    const int r0 = h_low - ty0, c0 = w_low - tx0;
    const bool in_tile = ((unsigned)r0 < (unsigned)(TR - 1)) & ((unsigned)c0 < (unsigned)(TC - 1));
    const float m = valid ? mk : 0.f;
    const float hm = hh * m, lm = lh * m;
    const float w1 = hm * hw, w2 = hm * lw, w3 = lm * hw, w4 = lm * lw;
    const float* p0 = st + (((in_tile ? r0 : 0) * 2) * TP + (in_tile ? c0 : 0)) * 4;
    const float* p1 = p0 + 2 * TP * 4;
    a0 = w1 * ld4(p0) + w2 * ld4(p0 + 4) + w3 * ld4(p1) + w4 * ld4(p1 + 4);
    a1 = w1 * ld4(p0 + TP * 4) + w2 * ld4(p0 + TP * 4 + 4) + w3 * ld4(p1 + TP * 4) + w4 * ld4(p1 + TP * 4 + 4);
#if DCNSEP_EXP == 4   // timing probe: no global fallback outside the staged tile
    const bool fb = false;
#else
    const bool fb = valid & !in_tile;
#endif
    if (__builtin_amdgcn_ballot_w64(fb)) {
      if (fb) {
        const int h_high = h_low + 1, w_high = w_low + 1, co = dg * 8;
        const bool b1 = h_low >= 0 && w_low >= 0, b2 = h_low >= 0 && w_high <= W - 1;
        const bool b3 = h_high <= H - 1 && w_low >= 0, b4 = h_high <= H - 1 && w_high <= W - 1;
        const float* q1 = in + ((size_t)h_low * W + w_low) * 64 + co;
        const float* q2 = in + ((size_t)h_low * W + w_high) * 64 + co;
        const float* q3 = in + ((size_t)h_high * W + w_low) * 64 + co;
        const float* q4 = in + ((size_t)h_high * W + w_high) * 64 + co;
        const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
        a0 = w1 * (b1 ? ld4(q1) : z) + w2 * (b2 ? ld4(q2) : z) + w3 * (b3 ? ld4(q3) : z) + w4 * (b4 ? ld4(q4) : z);
        a1 = w1 * (b1 ? ld4(q1 + 4) : z) + w2 * (b2 ? ld4(q2 + 4) : z) + w3 * (b3 ? ld4(q3 + 4) : z) +
             w4 * (b4 ? ld4(q4 + 4) : z);
      }
    }
  };

  f32x16 acc0 = f32x16{0}, acc1 = f32x16{0};
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // group 0 staged (and the om biases loaded)
  __syncthreads();                                    // phase-1 buffers free for group 1
  auto dcn_group = [&](int dg, const f32x16& o) {
#if DCNSEP_EXP == 3   // timing probe: no phase 2 work
    return;
#endif
    if (dg + 1 < 8) stage_group(dg + 1, smem + (((dg + 1) & 1) ? OFF_G1 : OFF_G0));
    const float* st = smem + ((dg & 1) ? OFF_G1 : OFF_G0);
    const float* sw = st + T_F;
#pragma unroll
    for (int pp = 0; pp < 5; ++pp) {
      f32x4 a0, a1;
      sample(st, dg, 2 * pp + hf, o[3 * pp], o[3 * pp + 1], o[3 * pp + 2], a0, a1);
      f16x8 ah, al;
      split_f16x3(a0, a1, ah, al);
      const float* wp = sw + pp * 1024 + lane * 4;   // [pair][nt][plane][lane][8 halves]
      const f16x8 bh0 = ldh8(wp), bl0 = ldh8(wp + 256), bh1 = ldh8(wp + 512), bl1 = ldh8(wp + 768);
      acc0 = mfma16h(ah, bh0, acc0);
      acc1 = mfma16h(ah, bh1, acc1);
      acc0 = mfma16h(ah, bl0, acc0);
      acc1 = mfma16h(ah, bl1, acc1);
      acc0 = mfma16h(al, bh0, acc0);
      acc1 = mfma16h(al, bh1, acc1);
    }
    lds_dma_barrier();
  };
#if DCNSEP_ROLL
  // one loop body (smaller code): the next group's offsets rotate into om[0]
#pragma unroll 1
  for (int dg = 0; dg < 8; ++dg) {
    dcn_group(dg, om[0]);
#pragma unroll
    for (int q = 0; q < 7; ++q) om[q] = om[q + 1];
  }
#else
#pragma unroll
  for (int dg = 0; dg < 8; ++dg) dcn_group(dg, om[dg]);
#endif
  // epilogue through a per-wave LDS block -> coalesced 16-B stores (k_dcn's)
  float* out = a.out[g] + (size_t)n * a.out_item;
  const float* bias = a.bias[g];
  float* blk = smem + OFF_W + wv * 1024;
  const int rpx = lane >> 3, c4 = lane & 7;
  bool bad2 = false;
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const float bv = bias[nt * 32 + l32];
    f32x16 v;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float t = (nt ? acc1[r] : acc0[r]) * F16X3_UNSCALE + bv;
      bad2 |= not_finite(t);
      if (EPI == STIF_EPI_LRELU) t = lrelu01(t);
      v[r] = t;
    }
    tile_to_lds(blk, v, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int px = i * 8 + rpx, x = ox0 + px;
      const f32x4 o = lds_row4(blk, px, c4);
      if (oy < H && x < W) st4(out + ((size_t)oy * W + x) * 64 + nt * 32 + c4 * 4, o);
    }
  }
  report_range(a.status, bad2);
}

}  // namespace

extern "C" int stif_dcn_sep_nhwc(const stif_dcn_sep_args* pa, void* stream) {
  if (!pa) return stif_fail(STIF_E_INVALID, "stif_dcn_sep_nhwc: null args");
  const stif_dcn_sep_args& a = *pa;
  if (a.ngroups < 1 || a.ngroups > STIF_MAX_GROUPS || a.nitems < 1 || a.H < 1 || a.W < 1)
    return stif_fail(STIF_E_INVALID, "stif_dcn_sep_nhwc: bad sizes");
  if (!(a.flags & STIF_CONV_F16X3))
    return stif_fail(STIF_E_INVALID, "stif_dcn_sep_nhwc: split-fp16 operands only (flags = STIF_CONV_F16X3)");
  if ((long long)a.H * a.W * 64 * 4 >= 0x7fffffffLL)
    return stif_fail(STIF_E_INVALID, "stif_dcn_sep_nhwc: item larger than 2 GB (buffer addressing)");
  for (int i = 0; i < a.ngroups; ++i)
    if (!a.fea[i] || !a.in[i] || !a.w_om[i] || !a.b_om[i] || !a.w[i] || !a.bias[i] || !a.out[i])
      return stif_fail(STIF_E_INVALID, "stif_dcn_sep_nhwc: null tensor");
  const long long wgs = (long long)((a.W + TW - 1) / TW) * ((a.H + NW - 1) / NW) * a.ngroups * a.nitems;
  if (wgs > 0x7fffffff) return stif_fail(STIF_E_INVALID, "stif_dcn_sep_nhwc: grid too large");
  dim3 grid((unsigned)wgs);
  if (a.epi == STIF_EPI_LRELU)
    hipLaunchKernelGGL(k_dcn_sep<STIF_EPI_LRELU>, grid, dim3(64 * NW), 0, (hipStream_t)stream, a);
  else if (a.epi == STIF_EPI_NONE)
    hipLaunchKernelGGL(k_dcn_sep<STIF_EPI_NONE>, grid, dim3(64 * NW), 0, (hipStream_t)stream, a);
  else
    return stif_fail(STIF_E_INVALID, "stif_dcn_sep_nhwc: epilogue must be NONE or LRELU");
  return stif_check_launch("stif_dcn_sep_nhwc");
}
