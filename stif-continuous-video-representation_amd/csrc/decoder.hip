// Implicit SIREN decoder of LunaTokis.decoding (Sakuya_arch_test.py:364-459) for gfx950.
//
// The reference materialises, per query time t, ~2,300 floats per HR pixel of
// grid_sample gathers and torch.cat results and runs three nn.Linear stacks over
// them.  Here the work is split into:
//   (0) an LR projection (stif_conv2d_nhwc, 1x1, 200 -> 256 channels): every linear
//       input block that is gathered from the LR maps (feat 192 + inp 6) is projected
//       once per LR pixel -- nearest/bilinear sampling commutes with a linear map,
//       so the per-HR-pixel work gathers 64-wide projections instead of 198-wide
//       inputs (P1 nearest, P2 bilinear at the HR centre, P3/P4 bilinear at the
//       warped grids);
//   (1) k_dec1: per HR pixel feat_imnet -> HRfeat (64) and flow_imnet -> flow (4);
//   (2) k_dec2: per HR pixel warpgrid (warplayer.py:25-39) + bilinear HRfeat at both
//       warped grids + encode_imnet -> RGB.
// Each wave owns 32 HR pixels (one per lane, both lane halves hold the same pixel);
// every SIREN layer is a chain of v_mfma_f32_32x32x2_f32 with features in the
// accumulator registers (layout in dec_layout.h), sin(30 z) applied in registers.
#include "dec_layout.h"
#include "stif_common.h"
#include "tuning.h"
#include "stif.h"
#include "abi_util.h"

#include <algorithm>

namespace {

using namespace stif_dec;

// F16 (stif_pack_dec_mlp_ex with STIF_CONV_F16X3): every 32x32 weight tile is a split-fp16 tile
// ([m][plane h|l][lane][8 halves], W * 2^10) and every register tile that feeds one is split too
// (x * 2^4, split_f16x3), so MFMA accumulators hold values x 2^14 -- everything added into them
// (gathered projections, bias terms, the fp32 image tiles, packed x 2^14) is scaled to match and
// every consumer unscales (ACC_S).
template <int F16>
struct XT;   // a 32-feature register tile as an MFMA B operand
template <>
struct XT<0> {
  f32x16 v;
};
template <>
struct XT<1> {
  f16x8 h[2], l[2];
};
template <int F16>
STIF_DEV XT<F16> xop(const f32x16& x) {
  XT<F16> o;
  if constexpr (F16) {
#pragma unroll
    for (int m = 0; m < 2; ++m)
      split_f16x3(f32x4{x[8 * m], x[8 * m + 1], x[8 * m + 2], x[8 * m + 3]},
                  f32x4{x[8 * m + 4], x[8 * m + 5], x[8 * m + 6], x[8 * m + 7]}, o.h[m], o.l[m]);
  } else {
    o.v = x;
  }
  return o;
}
template <int F16>
constexpr float ACC_S = F16 ? F16X3_UNSCALE : 1.f;   // accumulator -> value
template <int F16>
constexpr float ACC_IN = F16 ? 16384.f : 1.f;        // value -> accumulator

// the 16 biases of one 32-feature register tile (features F(r, hf)) as 4 vector loads
struct Bias32 {
  f32x4 v[4];
};
STIF_DEV Bias32 bias_ld(const float* __restrict__ b, int hf) {
  Bias32 o;
#pragma unroll
  for (int v = 0; v < 4; ++v) o.v[v] = ld4(b + 8 * v + 4 * hf);
  return o;
}
// SineLayer: sin(30 * (z + b)) (SIREN.py:44-45, omega_0 = 30); the packed weights and biases of every
// sine layer carry the factor 30 (pack.cpp), so the kernel evaluates sin(z + b)
template <int F16>
STIF_DEV f32x16 bias_sin(f32x16 z, const Bias32& bb) {
#pragma unroll
  for (int v = 0; v < 4; ++v)
#pragma unroll
    for (int e = 0; e < 4; ++e) z[4 * v + e] = siren_sin<F16>(fmaf(z[4 * v + e], ACC_S<F16>, bb.v[v][e]));
  return z;
}
template <int F16>
STIF_DEV f32x16 bias_sin(f32x16 z, const float* __restrict__ b, int hf) {
  return bias_sin<F16>(z, bias_ld(b, hf));
}

template <int F16>
STIF_DEV f32x16 bias_add(f32x16 z, const float* __restrict__ b, int hf) {
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const f32x4 bb = ld4(b + 8 * v + 4 * hf);
#pragma unroll
    for (int e = 0; e < 4; ++e) z[4 * v + e] = fmaf(z[4 * v + e], ACC_S<F16>, bb[e]);
  }
  return z;
}

struct Bilin {  // grid_sample bilinear corners (align_corners=False, zeros padding)
  int o00, o01, o10, o11;      // element offsets (pixel index)
  float w00, w01, w10, w11;    // weights, 0 for out-of-range corners
};

// ATen grid_sampler_2d bilinear: ix = ((x + 1) * W - 1) / 2, corner weights
// nw = (ix_se - ix) * (iy_se - iy), ...; corners outside the map contribute 0.
STIF_DEV Bilin bilin(float gx, float gy, int Wd, int Hd) {
  const float ix = ((gx + 1.f) * (float)Wd - 1.f) / 2.f;
  const float iy = ((gy + 1.f) * (float)Hd - 1.f) / 2.f;
  const float fx0 = floorf(ix), fy0 = floorf(iy);
  const int x0 = (int)fx0, y0 = (int)fy0, x1 = x0 + 1, y1 = y0 + 1;
  const float wx1 = ix - fx0, wx0 = (fx0 + 1.f) - ix;
  const float wy1 = iy - fy0, wy0 = (fy0 + 1.f) - iy;
  const bool vx0 = x0 >= 0 && x0 < Wd, vx1 = x1 >= 0 && x1 < Wd;
  const bool vy0 = y0 >= 0 && y0 < Hd, vy1 = y1 >= 0 && y1 < Hd;
  const int cx0 = min(max(x0, 0), Wd - 1), cx1 = min(max(x1, 0), Wd - 1);
  const int cy0 = min(max(y0, 0), Hd - 1), cy1 = min(max(y1, 0), Hd - 1);
  Bilin b;
  b.o00 = cy0 * Wd + cx0; b.o01 = cy0 * Wd + cx1; b.o10 = cy1 * Wd + cx0; b.o11 = cy1 * Wd + cx1;
  b.w00 = (vx0 && vy0) ? wx0 * wy0 : 0.f;
  b.w01 = (vx1 && vy0) ? wx1 * wy0 : 0.f;
  b.w10 = (vx0 && vy1) ? wx0 * wy1 : 0.f;
  b.w11 = (vx1 && vy1) ? wx1 * wy1 : 0.f;
  return b;
}

// bilinear sample of channel block [c0, c0+64) of an NHWC map with `stride` channels,
// into two register tiles (features F(r, hf) of each 32-block)
STIF_DEV void gather64(f32x16* dst, const float* __restrict__ base, int stride, int c0, const Bilin& b, int hf) {
  // all 32 corner loads (8 channel groups x 4 corners, 128 VGPRs) are issued before the first blend,
  // so a gather waits for one memory latency, not one per channel group
  const int c = c0 + 4 * hf;
  const float* p00 = base + (size_t)b.o00 * stride + c;
  const float* p01 = base + (size_t)b.o01 * stride + c;
  const float* p10 = base + (size_t)b.o10 * stride + c;
  const float* p11 = base + (size_t)b.o11 * stride + c;
  f32x4 cr[8][4];
#pragma unroll
  for (int g = 0; g < 8; ++g) {   // group g = (ot, v) = (g >> 2, g & 3): channels 8 g + 4 hf ..
    cr[g][0] = ld4(p00 + 8 * g);
    cr[g][1] = ld4(p01 + 8 * g);
    cr[g][2] = ld4(p10 + 8 * g);
    cr[g][3] = ld4(p11 + 8 * g);
  }
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    f32x4 s = b.w00 * cr[g][0] + b.w01 * cr[g][1] + b.w10 * cr[g][2] + b.w11 * cr[g][3];
    // combine the corners here, in load order: otherwise the blend is sunk to the first use (past a
    // barrier) and all four corners of every channel stay live
    asm volatile("" : "+v"(s));
#pragma unroll
    for (int e = 0; e < 4; ++e) dst[g >> 2][4 * (g & 3) + e] = s[e];
  }
}

// gather64 with at most 8 corner loads (32 VGPRs) in flight: four memory latencies
STIF_DEV void gather64_q(f32x16* dst, const float* __restrict__ base, int stride, int c0, const Bilin& b, int hf) {
  const int c = c0 + 4 * hf;
  const float* p00 = base + (size_t)b.o00 * stride + c;
  const float* p01 = base + (size_t)b.o01 * stride + c;
  const float* p10 = base + (size_t)b.o10 * stride + c;
  const float* p11 = base + (size_t)b.o11 * stride + c;
#pragma unroll
  for (int qr = 0; qr < 4; ++qr) {
    f32x4 cr[2][4];
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const int o = 8 * (2 * qr + g);
      cr[g][0] = ld4(p00 + o);
      cr[g][1] = ld4(p01 + o);
      cr[g][2] = ld4(p10 + o);
      cr[g][3] = ld4(p11 + o);
    }
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      f32x4 s = b.w00 * cr[g][0] + b.w01 * cr[g][1] + b.w10 * cr[g][2] + b.w11 * cr[g][3];
      asm volatile("" : "+v"(s));
      const int gg = 2 * qr + g;
#pragma unroll
      for (int e = 0; e < 4; ++e) dst[gg >> 2][4 * (gg & 3) + e] = s[e];
    }
    asm volatile("" ::: "memory");
  }
}

// gather64 with at most 16 corner loads (64 VGPRs) in flight: two memory latencies instead of one, for
// kernels budgeted below the 128 VGPRs of the one-shot form
STIF_DEV void gather64_h(f32x16* dst, const float* __restrict__ base, int stride, int c0, const Bilin& b, int hf) {
  const int c = c0 + 4 * hf;
  const float* p00 = base + (size_t)b.o00 * stride + c;
  const float* p01 = base + (size_t)b.o01 * stride + c;
  const float* p10 = base + (size_t)b.o10 * stride + c;
  const float* p11 = base + (size_t)b.o11 * stride + c;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    f32x4 cr[4][4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int o = 8 * (4 * half + g);
      cr[g][0] = ld4(p00 + o);
      cr[g][1] = ld4(p01 + o);
      cr[g][2] = ld4(p10 + o);
      cr[g][3] = ld4(p11 + o);
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      f32x4 s = b.w00 * cr[g][0] + b.w01 * cr[g][1] + b.w10 * cr[g][2] + b.w11 * cr[g][3];
      asm volatile("" : "+v"(s));
#pragma unroll
      for (int e = 0; e < 4; ++e) dst[half][4 * g + e] = s[e];
    }
    asm volatile("" ::: "memory");
  }
}

// z[ot] += W_img . img: the 6 image channels (padded to 8) are one K chunk, so lane half h supplies
// channels 4h..4h+3 as the B operand of the first 4 MFMAs of a packed tile (features F(e, h), e < 4)
STIF_DEV void img_mma(f32x16* z, const float* __restrict__ wt, const f32x4 im4, int lane) {
#pragma unroll
  for (int ot = 0; ot < 2; ++ot) {
    const f32x4 w0 = ld4(wt + ot * T + lane * 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) z[ot] = mfma32(w0[e], im4[e], z[ot]);
  }
}

// bilinear sample of channels 4h..4h+3 of a [ih][iw][8] high-resolution image
STIF_DEV f32x4 img_sample(const float* __restrict__ I, const Bilin& b, int hf) {
  const float* c = I + 4 * hf;
  return b.w00 * ld4(c + b.o00 * IMG_C) + b.w01 * ld4(c + b.o01 * IMG_C) + b.w10 * ld4(c + b.o10 * IMG_C) +
         b.w11 * ld4(c + b.o11 * IMG_C);
}

// ---- weight streaming: a workgroup consumes its MLP weight tiles segment by segment; each segment
// (a few 4-KB tiles: one layer, or one output tile's K-tiles) is LDS-DMA'd while the previous one
// is being consumed (double-buffered, one barrier per segment), and every wave reads its A
// operands from LDS -- one tile feeds 16 MFMAs in each wave of the workgroup.
// waves per workgroup of k_dec1: 4-wave workgroups, DEC1_OCC per CU -- by default 4 (36 KB LDS, <= 128 VGPRs
// each; the HRIMG variants stay at 3: 52 KB, <= 168, and MODE 2 at 2: 69 KB): the waves sharing a SIMD come from different
// workgroups, so one's segment barrier, gather or sin stretch overlaps the others' MFMAs
constexpr int DEC2_NW = 4;   // k_dec2: 8 layer-3 accumulator tiles (128 VGPRs) live
constexpr int SEG = 10;      // max tiles per segment (k_dec2)
constexpr int SEG1 = 8;      // max tiles per segment (k_dec1)

// Buffer loads with the tile offset in SGPRs: the per-lane operand is the same lane*16 for every
// tile (flat global_load_lds would keep a 64-bit VGPR address per hoisted tile live).
// Probe DEC_EXP 3 issues every piece with an out-of-range offset (the same instructions, no memory traffic: the
// LDS receives zeros).  (A probe that issued no DMA at all, the former DEC_EXP 1, measured nothing: with the
// weight buffers never written the compiler folded most of the MFMAs, LDS reads and sines that read them.)
STIF_DEV void dec_dma(__amdgpu_buffer_rsrc_t rm, float* dst, int lane, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rm, dst, 16, DEC_EXP == 3 ? 0x80000000u : (unsigned)(lane * 16), soff, 0, 0);
}
template <int NW>
STIF_DEV void dma_tiles(float* dst, __amdgpu_buffer_rsrc_t rm, int src, int ntiles, int wv, int lane) {
  if ((ntiles * 4) % NW == 0) {
    // the same number of pieces per wave, known at compile time: the compiler counts them in vmcnt, so
    // waiting for a load issued before the DMA does not wait for the DMA
#pragma unroll
    for (int i = 0; i < ntiles * 4 / NW; ++i)
      dec_dma(rm, dst + (wv + i * NW) * 256, lane, (src + (wv + i * NW) * 256) * 4);
  } else {
    for (int k = wv; k < ntiles * 4; k += NW)
      dec_dma(rm, dst + k * 256, lane, (src + k * 256) * 4);
  }
}

// the segment barrier of the weight stream (lds_dma_barrier); probe DEC_EXP 2 skips its vmcnt(0) wait, i.e. the
// time the waves spend waiting for segments still in flight (wrong results)
STIF_DEV void dec_barrier() {
#if DEC_EXP == 2
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
#else
  lds_dma_barrier();
#endif
}

STIF_DEV __amdgpu_buffer_rsrc_t mlp_rsrc(const float* mlp) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)mlp, (short)0, (int)(MLP_FLOATS * 4), 0x00020000);
}

// acc += W_tile . x, tile in LDS ([v][lane][4]), x = one 32-feature register tile
template <int F16>
STIF_DEV void tile_mma(f32x16& acc, const float* t, const XT<F16>& xt, int lane) {
  const float* b = t + lane * 4;
  if constexpr (F16) {
    // tile [m][plane][lane][8 halves]: element e of half-tile m = feature F(8m + e, lane >> 5)
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const f16x8 ah = ldh8(b + (2 * m) * 256), al = ldh8(b + (2 * m + 1) * 256);
      acc = mfma16h(ah, xt.h[m], acc);
      acc = mfma16h(al, xt.h[m], acc);
      acc = mfma16h(ah, xt.l[m], acc);
    }
  } else {
    const f32x16& x = xt.v;
    const f32x4 w0 = ld4(b), w1 = ld4(b + 256), w2 = ld4(b + 512), w3 = ld4(b + 768);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc = mfma32(w0[e], x[e], acc);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc = mfma32(w1[e], x[4 + e], acc);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc = mfma32(w2[e], x[8 + e], acc);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc = mfma32(w3[e], x[12 + e], acc);
  }
  // keep the compiler from hoisting the LDS reads of many tiles ahead (VGPR budget)
  __builtin_amdgcn_sched_barrier(0);
}

// o[c] += W[c][32 kt + F(r, hf)] . x[r] over this lane's 16 features of register tile kt (W: plain
// [NO][256] rows in LDS; the two lane halves read two addresses per instruction, a broadcast)
template <int NO>
STIF_DEV void narrow_dot(float* o, const float* W, int kt, const f32x16& x, int hf) {
#pragma unroll
  for (int c = 0; c < NO; ++c)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const f32x4 w = ld4(W + c * 256 + kt * 32 + 8 * v + 4 * hf);
#pragma unroll
      for (int e = 0; e < 4; ++e) o[c] = fmaf(w[e], x[4 * v + e], o[c]);
    }
}

// MODE 0: feat_imnet + flow_imnet fused (the flow stage reads the pixel's own HRfeat);
// MODE 1: feat_imnet only; MODE 2: flow_imnet only, reading HRfeat at (hr_y, hr_x) of the query
// (local ensemble).  HRIMG: the flow stage's image input comes from the high-resolution image.
// DEC1_OCC = 3 (MODE 0 / 1): 6-tile segments (52 KB of LDS) and a 168-register budget, so three workgroups
// (three waves per SIMD) share a CU; flow layer 1's second output tile then arrives after the last feat step
// DEC1_OCC = 4: 4-tile segments (36 KB) and 128 registers; flow layer 1 then arrives after the last feat
// step and flow segment 0 after flow layer 0
// (the HRIMG variants, decoding_test's, stay at 3: at 128 registers their image gather spills)
template <int MODE, bool HRIMG>
constexpr int OCC1 = MODE == 2 ? 2 : (HRIMG && DEC1_OCC > 3) ? 3 : DEC1_OCC;
template <int MODE, bool HRIMG>
constexpr int S1 = OCC1<MODE, HRIMG> == 4 ? 4 : OCC1<MODE, HRIMG> == 3 ? 6 : SEG1;
// waves per workgroup: DEC1_NW for the four-per-SIMD variants (8: two 8-wave workgroups per CU stream each weight
// segment for 256 pixels instead of 128), 4 for the others
template <int MODE, bool HRIMG>
constexpr int NW1 = OCC1<MODE, HRIMG> == 4 ? DEC1_NW : 4;
template <int MODE, bool HRIMG, int F16>
__global__ __launch_bounds__((NW1<MODE, HRIMG> * 64)) __attribute__((amdgpu_waves_per_eu(OCC1<MODE, HRIMG>))) void k_dec1(const float* __restrict__ proj, const float* __restrict__ mlp,
                                                     stif_dec_tables tb, stif_dec_image im,
                                                     const float* __restrict__ tq, float* __restrict__ hrfeat,
                                                     float* __restrict__ flow, int n, int h, int w, int HH,
                                                     int WW) {
  // two segment buffers of SEG1 tiles + the flow's last layer (plain [4][256], resident)
  constexpr bool OCC3 = S1<MODE, HRIMG> != SEG1;             // 3 or 4 workgroups per CU
  constexpr bool OCC4 = OCC1<MODE, HRIMG> == 4;
  constexpr int DEC_NW = NW1<MODE, HRIMG>;
  __shared__ __attribute__((aligned(16))) float wbuf[2 * S1<MODE, HRIMG> * T + T];
  const int lane = threadIdx.x & 63, hf = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform
  float* const B0 = wbuf;
  float* const B1 = wbuf + S1<MODE, HRIMG> * T;
  float* const W3V = wbuf + 2 * S1<MODE, HRIMG> * T;
  const __amdgpu_buffer_rsrc_t rm = mlp_rsrc(mlp);
  if (MODE != 1) dma_tiles<DEC_NW>(W3V, rm, L_W3V, 1, wv, lane);
  // segment 0: feat layer 1 (4 tiles); segments 1..8: feat layer 2 tile kt + layer 3 (0, kt), (1, kt)
  if (MODE != 2) dma_tiles<DEC_NW>(B0, rm, F_W1, 4, wv, lane);
  else {   // flow only: flow layers 0 / 1 straight into B1
    dma_tiles<DEC_NW>(B1, rm, L_W0, 4, wv, lane);
    dma_tiles<DEC_NW>(B1 + 4 * T, rm, L_W1, 4, wv, lane);
  }
  const long long total = (long long)n * HH * WW;
  const long long p = ((long long)xcd_block(blockIdx.x, gridDim.x) * DEC_NW + wv) * 32 + (lane & 31);
  const bool valid = p < total;
  const long long pc = valid ? p : total - 1;
  const int item = (int)(pc / ((long long)HH * WW));
  const int rem = (int)(pc - (long long)item * HH * WW);
  const int py = rem / WW, px = rem - py * WW;
  const float t = tq[item];
  const float* P = proj + (size_t)item * h * w * PROJ_C;

  f32x16 hr[2] = {f32x16{0}, f32x16{0}};
  f32x16 x1[2];
  if constexpr (MODE != 2) {
  // ---- feat_imnet layer 0: z = P1[nearest] + w_rel . rel + w_t * t  (bias folded into P1)
  f32x16 x0[2];
  {
    const float ry = tb.rel_y[py], rx = tb.rel_x[px];
    const float* p1 = P + ((size_t)tb.near_y[py] * w + tb.near_x[px]) * PROJ_C;
#pragma unroll
    for (int ot = 0; ot < 2; ++ot)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int f = ot * 32 + 8 * v + 4 * hf;
        const f32x4 z = ld4(p1 + f) + ld4(mlp + F_WRY + f) * ry + ld4(mlp + F_WRX + f) * rx + ld4(mlp + F_WT + f) * t;
#pragma unroll
        for (int e = 0; e < 4; ++e) x0[ot][4 * v + e] = siren_sin<F16>(z[e]);
      }
  }
  auto seg_feat23 = [&](float* dst, int kt) {   // W2 rows kt (2 tiles), W3 (0, kt), (1, kt): 16 pieces, as one
    // loop with the same count on every wave (exact vmcnt bookkeeping for 4- and 8-wave workgroups)
#pragma unroll
    for (int r = 0; r < 16 / DEC_NW; ++r) {
      const int i = wv + r * DEC_NW, j = i >> 2;
      const int src = (j < 2 ? F_W2 + (kt * 2 + j) * T : F_W3 + ((j - 2) * 8 + kt) * T) + (i & 3) * 256;
      dec_dma(rm, dst + j * T + (i & 3) * 256, lane, src * 4);
    }
  };
  dec_barrier();
  const Bias32 fb1[2] = {bias_ld(mlp + F_B1, hf), bias_ld(mlp + F_B1 + 32, hf)};   // before the DMA
  __builtin_amdgcn_sched_barrier(0);
  seg_feat23(B1, 0);
  // ---- layer 1: 64 -> 64
  {
    const XT<F16> xs[2] = {xop<F16>(x0[0]), xop<F16>(x0[1])};
#pragma unroll
    for (int ot = 0; ot < 2; ++ot) {
      f32x16 acc = f32x16{0};
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) tile_mma<F16>(acc, B0 + (ot * 2 + kt) * T, xs[kt], lane);
      x1[ot] = bias_sin<F16>(acc, fb1[ot]);
    }
  }
  // ---- layer 2 (64 -> 256, sine) streamed into layer 3 (256 -> 64, linear)
  const XT<F16> x1s[2] = {xop<F16>(x1[0]), xop<F16>(x1[1])};
  // the streamed steps (kt = 7 peeled: its DMA differs, and the loop's steps must all issue the same
  // number of DMA pieces for the compiler's vmcnt bookkeeping to stay exact across the back edge)
  auto feat_step = [&](int kt, bool last) {
    dec_barrier();
    // this step's bias is loaded before the next segment's DMA is issued, so waiting for it does not
    // wait for the DMA (vmcnt counts in issue order)
    const Bias32 b2 = bias_ld(mlp + F_B2 + kt * 32, hf);
    __builtin_amdgcn_sched_barrier(0);
    float* cur = (kt & 1) ? B0 : B1;
    float* nxt = (kt & 1) ? B1 : B0;
    auto dma_next = [&]() {
      if (!last) seg_feat23(nxt, kt + 1);
      else {   // prefetch flow layer 0 (4 tiles) + layer 1 (4 tiles; OCC3: its first output tile)
        dma_tiles<DEC_NW>(nxt, rm, L_W0, 4, wv, lane);
        if (!OCC4) dma_tiles<DEC_NW>(nxt + 4 * T, rm, L_W1, OCC3 ? 2 : 4, wv, lane);
      }
    };
    if (!DEC_DMA_LATE) dma_next();
    f32x16 acc = f32x16{0};
    tile_mma<F16>(acc, cur, x1s[0], lane);
    tile_mma<F16>(acc, cur + T, x1s[1], lane);
    if (DEC_DMA_LATE) dma_next();
    const XT<F16> h2 = xop<F16>(bias_sin<F16>(acc, b2));
    tile_mma<F16>(hr[0], cur + 2 * T, h2, lane);
    tile_mma<F16>(hr[1], cur + 3 * T, h2, lane);
  };
#pragma unroll 1
  for (int kt = 0; kt < 7; ++kt) feat_step(kt, false);
  feat_step(7, true);
#pragma unroll
  for (int ot = 0; ot < 2; ++ot) hr[ot] = bias_add<F16>(hr[ot], mlp + F_B3 + ot * 32, hf);
  if (valid) {
    float* o = hrfeat + (size_t)pc * 64;
#pragma unroll
    for (int ot = 0; ot < 2; ++ot)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        f32x4 s;
#pragma unroll
        for (int e = 0; e < 4; ++e) s[e] = hr[ot][4 * v + e];
        st4(o + ot * 32 + 8 * v + 4 * hf, s);
      }
  }
  }   // MODE != 2
  if constexpr (MODE == 1) return;
  if constexpr (MODE == 2) {
    // the query's HRfeat operand: the HR pixel nearest to the shifted query (grid_sample nearest
    // of HRfeat at coord_, Sakuya_arch_test.py:1022-1025)
    Bilin b;
    b.o00 = b.o01 = b.o10 = b.o11 = tb.hr_y[py] * WW + tb.hr_x[px];
    b.w00 = 1.f;
    b.w01 = b.w10 = b.w11 = 0.f;
    gather64(hr, hrfeat + (size_t)item * HH * WW * 64, 64, 0, b, hf);
  }

  // ---- flow_imnet layer 0: W[:, :64] . HRfeat + bilinear(P2 at the HR centre) + w_t * t + b
  f32x16 z[2];
  {
    Bilin b;
    const int y0 = tb.by0[py], y1 = tb.by1[py], x0_ = tb.bx0[px], x1_ = tb.bx1[px];
    const float wy0 = tb.wy0[py], wy1 = tb.wy1[py], wx0 = tb.wx0[px], wx1 = tb.wx1[px];
    b.o00 = y0 * w + x0_; b.o01 = y0 * w + x1_; b.o10 = y1 * w + x0_; b.o11 = y1 * w + x1_;
    b.w00 = wx0 * wy0; b.w01 = wx1 * wy0; b.w10 = wx0 * wy1; b.w11 = wx1 * wy1;
    if (OCC4) gather64_q(z, P, PROJ_C, 64, b, hf);
    else if (OCC3) gather64_h(z, P, PROJ_C, 64, b, hf);
    else gather64(z, P, PROJ_C, 64, b, hf);
#pragma unroll
    for (int ot = 0; ot < 2; ++ot)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int f = ot * 32 + 8 * v + 4 * hf;
        const f32x4 wt = ld4(mlp + L_WT + f), bb = ld4(mlp + L_B0 + f);
#pragma unroll
        for (int e = 0; e < 4; ++e) z[ot][4 * v + e] = (z[ot][4 * v + e] + (wt[e] * t + bb[e])) * ACC_IN<F16>;
      }
    if constexpr (HRIMG) {   // q_inp from the high-resolution image (decoding_test :515-518)
      Bilin bi;
      const int y0 = im.by0[py], y1 = im.by1[py], x0_ = im.bx0[px], x1_ = im.bx1[px];
      const float wy0 = im.wy0[py], wy1 = im.wy1[py], wx0 = im.wx0[px], wx1 = im.wx1[px];
      bi.o00 = y0 * im.iw + x0_; bi.o01 = y0 * im.iw + x1_; bi.o10 = y1 * im.iw + x0_; bi.o11 = y1 * im.iw + x1_;
      bi.w00 = wx0 * wy0; bi.w01 = wx1 * wy0; bi.w10 = wx0 * wy1; bi.w11 = wx1 * wy1;
      img_mma(z, mlp + I_L, img_sample(im.img + (size_t)item * im.ih * im.iw * IMG_C, bi, hf), lane);
    }
  }
  // flow layers 0/1 live in B1 (prefetched during the last feat segment, or at the start)
  dec_barrier();
  const Bias32 lb1[2] = {bias_ld(mlp + L_B1, hf), bias_ld(mlp + L_B1 + 32, hf)};   // before the DMA
  __builtin_amdgcn_sched_barrier(0);
  auto seg_flow23 = [&](float* dst, int kt) {   // W2 rows kt (2 tiles); W3 is resident (W3V)
    dma_tiles<DEC_NW>(dst, rm, L_W2 + kt * 2 * T, 2, wv, lane);
  };
  // OCC3: layer 1's second output tile (2 tiles) into B0, segment 0 after it
  constexpr bool L1B0 = OCC3 && !OCC4 && MODE == 0;
  if (OCC4) dma_tiles<DEC_NW>(B0, rm, L_W1, 4, wv, lane);   // all of layer 1 into B0; segment 0 later
  else {
    if (L1B0) dma_tiles<DEC_NW>(B0, rm, L_W1 + 2 * T, 2, wv, lane);
    seg_flow23(B0 + (L1B0 ? 2 * T : 0), 0);
  }
  {
    const XT<F16> hs[2] = {xop<F16>(hr[0]), xop<F16>(hr[1])};
#pragma unroll
    for (int ot = 0; ot < 2; ++ot) {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) tile_mma<F16>(z[ot], B1 + (ot * 2 + kt) * T, hs[kt], lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) z[ot][r] = siren_sin<F16>(z[ot][r] * ACC_S<F16>);
    }
  }
  if (L1B0 || OCC4) dec_barrier();   // layer 1 (OCC3: its second output tile) landed in B0
  if (OCC4) seg_flow23(B1, 0);             // every wave is done with layer 0's B1
  {
    const XT<F16> zs[2] = {xop<F16>(z[0]), xop<F16>(z[1])};
#pragma unroll
    for (int ot = 0; ot < 2; ++ot) {
      f32x16 acc = f32x16{0};
      const float* w1t = OCC4 ? B0 + ot * 2 * T : (L1B0 && ot == 1) ? B0 : B1 + (4 + ot * 2) * T;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) tile_mma<F16>(acc, w1t + kt * T, zs[kt], lane);
      x1[ot] = bias_sin<F16>(acc, lb1[ot]);
    }
  }
  const XT<F16> x1f[2] = {xop<F16>(x1[0]), xop<F16>(x1[1])};
  float fl[4] = {0.f, 0.f, 0.f, 0.f};
  auto flow_step = [&](int kt, bool last) {   // kt = 7 peeled (see feat_step)
    dec_barrier();
    const Bias32 b2 = bias_ld(mlp + L_B2 + kt * 32, hf);   // before the DMA (see feat_step)
    __builtin_amdgcn_sched_barrier(0);
    // OCC4: segment 0 sits in B1, so the buffers alternate the other way round
    float* cur = OCC4 ? ((kt & 1) ? B0 : B1) : (kt & 1) ? B1 : (L1B0 && kt == 0 ? B0 + 2 * T : B0);
    float* nxt = OCC4 ? ((kt & 1) ? B1 : B0) : (kt & 1) ? B0 : B1;
    if (!last && !DEC_DMA_LATE) seg_flow23(nxt, kt + 1);
    f32x16 acc = f32x16{0};
    tile_mma<F16>(acc, cur, x1f[0], lane);
    tile_mma<F16>(acc, cur + T, x1f[1], lane);
    if (!last && DEC_DMA_LATE) seg_flow23(nxt, kt + 1);
    const f32x16 h2 = bias_sin<F16>(acc, b2);
    narrow_dot<4>(fl, W3V, kt, h2, hf);   // flow_imnet.net.3 (256 -> 4, linear)
  };
#pragma unroll 1
  for (int kt = 0; kt < 7; ++kt) flow_step(kt, false);
  flow_step(7, true);
#pragma unroll
  for (int c = 0; c < 4; ++c) fl[c] += __shfl_xor(fl[c], 32);   // the other lane half's 128 features
  if (valid && hf == 0) {
    const f32x4 bb = ld4(mlp + L_B3);
    f32x4 s;
#pragma unroll
    for (int e = 0; e < 4; ++e) s[e] = fl[e] + bb[e];
    st4(flow + (size_t)pc * 4, s);
  }
}

// ---------------------------------------------------------------------------------------------
// Stage 1 with resident weights (DEC1_RES, split-fp16, LR-image inputs; measured, not the default): the streamed
// k_dec1 has every 128-pixel workgroup stream all 244 KB of its weights through LDS behind per-segment barriers.
// Here the stage runs as two persistent kernels, one 16-wave workgroup per CU, that load their network's weights
// into LDS once and then walk 32-pixel blocks with no barrier and no stream:
//   k_dec1f: feat_imnet (W1 | W2 | W3 = 36 tiles, 144 KB) -> HRfeat (64 per HR pixel, stored);
//   k_dec1l: flow_imnet (W0 | W1 | W2 = 24 tiles + the plain [4][256] W3, 100 KB), its HRfeat operand read back
//            from HBM (256 B per HR pixel) -> flow.
// Same arithmetic, same order as k_dec1<0, false, 1> (bit-identical outputs), but 372 + 430 us vs 655 us at C0
// (profiles/r06_dec_res.log): without stream and barriers k_dec1f runs at 0.37 and k_dec1l at 0.21 of their MFMA
// time, so neither was what bounds stage 1.
constexpr int RW = 16;   // waves per resident workgroup
__global__ __launch_bounds__(RW * 64) __attribute__((amdgpu_waves_per_eu(4))) void k_dec1f(
    const float* __restrict__ proj, const float* __restrict__ mlp, stif_dec_tables tb, const float* __restrict__ tq,
    float* __restrict__ hrfeat, int n, int h, int w, int HH, int WW) {
  __shared__ __attribute__((aligned(16))) float wr[36 * T];   // W1 (ot * 2 + kt) | W2 (kt * 2 + j) | W3 (ot * 8 + kt)
  const int lane = threadIdx.x & 63, hf = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const __amdgpu_buffer_rsrc_t rm = mlp_rsrc(mlp);
  dma_tiles<RW>(wr, rm, F_W1, 4, wv, lane);
  dma_tiles<RW>(wr + 4 * T, rm, F_W2, 16, wv, lane);
  dma_tiles<RW>(wr + 20 * T, rm, F_W3, 16, wv, lane);
  lds_dma_barrier();
  const long long total = (long long)n * HH * WW;
  const long long nblk = (total + 31) / 32;
  for (long long blk = (long long)blockIdx.x * RW + wv; blk < nblk; blk += (long long)gridDim.x * RW) {
    // the weights in LDS are loop-invariant to the compiler, which would hoist their reads out of the block loop
    // (and spill them): a memory clobber per block keeps every read next to its MFMAs
    asm volatile("" ::: "memory");
    const long long p = blk * 32 + (lane & 31);
    const bool valid = p < total;
    const long long pc = valid ? p : total - 1;
    const int item = (int)(pc / ((long long)HH * WW));
    const int rem = (int)(pc - (long long)item * HH * WW);
    const int py = rem / WW, px = rem - py * WW;
    const float t = tq[item];
    const float* P = proj + (size_t)item * h * w * PROJ_C;
    // layer 0: z = P1[nearest] + w_rel . rel + w_t * t (bias folded into P1)
    f32x16 x0[2];
    {
      const float ry = tb.rel_y[py], rx = tb.rel_x[px];
      const float* p1 = P + ((size_t)tb.near_y[py] * w + tb.near_x[px]) * PROJ_C;
#pragma unroll
      for (int ot = 0; ot < 2; ++ot)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int f = ot * 32 + 8 * v + 4 * hf;
          const f32x4 z = ld4(p1 + f) + ld4(mlp + F_WRY + f) * ry + ld4(mlp + F_WRX + f) * rx + ld4(mlp + F_WT + f) * t;
#pragma unroll
          for (int e = 0; e < 4; ++e) x0[ot][4 * v + e] = siren_sin<1>(z[e]);
        }
    }
    // layer 1: 64 -> 64
    f32x16 x1[2];
    {
      const Bias32 fb1[2] = {bias_ld(mlp + F_B1, hf), bias_ld(mlp + F_B1 + 32, hf)};
      const XT<1> xs[2] = {xop<1>(x0[0]), xop<1>(x0[1])};
#pragma unroll
      for (int ot = 0; ot < 2; ++ot) {
        f32x16 acc = f32x16{0};
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) tile_mma<1>(acc, wr + (ot * 2 + kt) * T, xs[kt], lane);
        x1[ot] = bias_sin<1>(acc, fb1[ot]);
      }
    }
    // layer 2 (64 -> 256, sine) tile by tile into layer 3 (256 -> 64, linear)
    const XT<1> x1s[2] = {xop<1>(x1[0]), xop<1>(x1[1])};
    f32x16 hr[2] = {f32x16{0}, f32x16{0}};
#pragma unroll 1
    for (int kt = 0; kt < 8; ++kt) {
      const Bias32 b2 = bias_ld(mlp + F_B2 + kt * 32, hf);
      f32x16 acc = f32x16{0};
      tile_mma<1>(acc, wr + (4 + kt * 2) * T, x1s[0], lane);
      tile_mma<1>(acc, wr + (5 + kt * 2) * T, x1s[1], lane);
      const XT<1> h2 = xop<1>(bias_sin<1>(acc, b2));
      tile_mma<1>(hr[0], wr + (20 + kt) * T, h2, lane);
      tile_mma<1>(hr[1], wr + (28 + kt) * T, h2, lane);
    }
#pragma unroll
    for (int ot = 0; ot < 2; ++ot) hr[ot] = bias_add<1>(hr[ot], mlp + F_B3 + ot * 32, hf);
    if (valid) {
      float* o = hrfeat + (size_t)pc * 64;
#pragma unroll
      for (int ot = 0; ot < 2; ++ot)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          f32x4 s4;
#pragma unroll
          for (int e = 0; e < 4; ++e) s4[e] = hr[ot][4 * v + e];
          st4(o + ot * 32 + 8 * v + 4 * hf, s4);
        }
    }
  }
}

__global__ __launch_bounds__(RW * 64) __attribute__((amdgpu_waves_per_eu(4))) void k_dec1l(
    const float* __restrict__ proj, const float* __restrict__ mlp, stif_dec_tables tb, const float* __restrict__ tq,
    const float* __restrict__ hrfeat, float* __restrict__ flow, int n, int h, int w, int HH, int WW) {
  __shared__ __attribute__((aligned(16))) float wr[25 * T];   // W0 (ot * 2 + kt) | W1 | W2 (kt * 2 + j) | W3 [4][256]
  const int lane = threadIdx.x & 63, hf = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const __amdgpu_buffer_rsrc_t rm = mlp_rsrc(mlp);
  dma_tiles<RW>(wr, rm, L_W0, 4, wv, lane);
  dma_tiles<RW>(wr + 4 * T, rm, L_W1, 4, wv, lane);
  dma_tiles<RW>(wr + 8 * T, rm, L_W2, 16, wv, lane);
  dma_tiles<RW>(wr + 24 * T, rm, L_W3V, 1, wv, lane);
  lds_dma_barrier();
  const float* const W3V = wr + 24 * T;
  const long long total = (long long)n * HH * WW;
  const long long nblk = (total + 31) / 32;
  for (long long blk = (long long)blockIdx.x * RW + wv; blk < nblk; blk += (long long)gridDim.x * RW) {
    // the weights in LDS are loop-invariant to the compiler, which would hoist their reads out of the block loop
    // (and spill them): a memory clobber per block keeps every read next to its MFMAs
    asm volatile("" ::: "memory");
    const long long p = blk * 32 + (lane & 31);
    const bool valid = p < total;
    const long long pc = valid ? p : total - 1;
    const int item = (int)(pc / ((long long)HH * WW));
    const int rem = (int)(pc - (long long)item * HH * WW);
    const int py = rem / WW, px = rem - py * WW;
    const float t = tq[item];
    const float* P = proj + (size_t)item * h * w * PROJ_C;
    // the pixel's own HRfeat (k_dec1f's output), in the register-tile order
    f32x16 hr[2];
    {
      const float* hp = hrfeat + (size_t)pc * 64 + 4 * hf;
#pragma unroll
      for (int ot = 0; ot < 2; ++ot)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const f32x4 q = ld4(hp + ot * 32 + 8 * v);
#pragma unroll
          for (int e = 0; e < 4; ++e) hr[ot][4 * v + e] = q[e];
        }
    }
    // layer 0: W[:, :64] . HRfeat + bilinear(P2 at the HR centre) + w_t * t + b
    f32x16 z[2];
    {
      Bilin b;
      const int y0 = tb.by0[py], y1 = tb.by1[py], x0_ = tb.bx0[px], x1_ = tb.bx1[px];
      const float wy0 = tb.wy0[py], wy1 = tb.wy1[py], wx0 = tb.wx0[px], wx1 = tb.wx1[px];
      b.o00 = y0 * w + x0_; b.o01 = y0 * w + x1_; b.o10 = y1 * w + x0_; b.o11 = y1 * w + x1_;
      b.w00 = wx0 * wy0; b.w01 = wx1 * wy0; b.w10 = wx0 * wy1; b.w11 = wx1 * wy1;
      gather64_q(z, P, PROJ_C, 64, b, hf);
#pragma unroll
      for (int ot = 0; ot < 2; ++ot)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int f = ot * 32 + 8 * v + 4 * hf;
          const f32x4 wt = ld4(mlp + L_WT + f), bb = ld4(mlp + L_B0 + f);
#pragma unroll
          for (int e = 0; e < 4; ++e) z[ot][4 * v + e] = (z[ot][4 * v + e] + (wt[e] * t + bb[e])) * ACC_IN<1>;
        }
    }
    {
      const XT<1> hs[2] = {xop<1>(hr[0]), xop<1>(hr[1])};
#pragma unroll
      for (int ot = 0; ot < 2; ++ot) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) tile_mma<1>(z[ot], wr + (ot * 2 + kt) * T, hs[kt], lane);
#pragma unroll
        for (int r = 0; r < 16; ++r) z[ot][r] = siren_sin<1>(z[ot][r] * ACC_S<1>);
      }
    }
    f32x16 x1[2];
    {
      const Bias32 lb1[2] = {bias_ld(mlp + L_B1, hf), bias_ld(mlp + L_B1 + 32, hf)};
      const XT<1> zs[2] = {xop<1>(z[0]), xop<1>(z[1])};
#pragma unroll
      for (int ot = 0; ot < 2; ++ot) {
        f32x16 acc = f32x16{0};
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) tile_mma<1>(acc, wr + (4 + ot * 2 + kt) * T, zs[kt], lane);
        x1[ot] = bias_sin<1>(acc, lb1[ot]);
      }
    }
    const XT<1> x1f[2] = {xop<1>(x1[0]), xop<1>(x1[1])};
    float fl[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int kt = 0; kt < 8; ++kt) {
      const Bias32 b2 = bias_ld(mlp + L_B2 + kt * 32, hf);
      f32x16 acc = f32x16{0};
      tile_mma<1>(acc, wr + (8 + kt * 2) * T, x1f[0], lane);
      tile_mma<1>(acc, wr + (9 + kt * 2) * T, x1f[1], lane);
      const f32x16 h2 = bias_sin<1>(acc, b2);
      narrow_dot<4>(fl, W3V, kt, h2, hf);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) fl[c] += __shfl_xor(fl[c], 32);
    if (valid && hf == 0) {
      const f32x4 bb = ld4(mlp + L_B3);
      f32x4 s4;
#pragma unroll
      for (int e = 0; e < 4; ++e) s4[e] = fl[e] + bb[e];
      st4(flow + (size_t)pc * 4, s4);
    }
  }
}

template <bool HRIMG, int F16>
__global__ __launch_bounds__(DEC2_NW * 64) __attribute__((amdgpu_waves_per_eu(DEC2_WPE))) void k_dec2(const float* __restrict__ proj, const float* __restrict__ mlp,
                                                     const float* __restrict__ hrfeat, const float* __restrict__ flow,
                                                     stif_dec_tables tb, stif_dec_image im,
                                                     const float* __restrict__ tq, float* __restrict__ out, int n,
                                                     int h, int w, int HH, int WW, int* status) {
  __shared__ __attribute__((aligned(16))) float wbuf[2 * SEG * T];
  const int lane = threadIdx.x & 63, hf = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform
  float* const B0 = wbuf;
  float* const B1 = wbuf + SEG * T;
  const __amdgpu_buffer_rsrc_t rm = mlp_rsrc(mlp);
  // segments: [L0: 8 tiles] [L1: 4] then per layer-2 tile kt: [W2 rows kt (2) + W3 column kt (8)],
  // then [W4: 8]
  dma_tiles<DEC2_NW>(B0, rm, E_W0, 8, wv, lane);
  const long long total = (long long)n * HH * WW;
  const long long p = ((long long)xcd_block(blockIdx.x, gridDim.x) * DEC2_NW + wv) * 32 + (lane & 31);
  const bool valid = p < total;
  const long long pc = valid ? p : total - 1;
  const int item = (int)(pc / ((long long)HH * WW));
  const int rem = (int)(pc - (long long)item * HH * WW);
  const int py = rem / WW, px = rem - py * WW;
  const float t = tq[item];
  const float* P = proj + (size_t)item * h * w * PROJ_C;
  const float* HRF = hrfeat + (size_t)item * HH * WW * 64;

  // warpgrid (warplayer.py:25-39): linspace grid + flow / ((n - 1) / 2), then the decoder's
  // clamp to (-1 + 1e-6, 1 - 1e-6) (Sakuya_arch_test.py:428,441)
  const f32x4 fv = ld4(flow + (size_t)pc * 4);
  const float lo = -1.f + 1e-6f, hi = 1.f - 1e-6f;
  const float dx = ((float)WW - 1.f) / 2.f, dy = ((float)HH - 1.f) / 2.f;
  const float bx = tb.lin_x[px], by = tb.lin_y[py];
  const float g1x = fminf(fmaxf(bx + fv[0] / dx, lo), hi), g1y = fminf(fmaxf(by + fv[1] / dy, lo), hi);
  const float g2x = fminf(fmaxf(bx + fv[2] / dx, lo), hi), g2y = fminf(fmaxf(by + fv[3] / dy, lo), hi);

  // ---- encode_imnet layer 0: W[:, :128] . [q_feat1 | q_feat2] + P3(grid1) + P4(grid2) + w_t t + b
  f32x16 x0[2];
  {
    // four 64-channel bilinear gathers (32 x 16-B loads per lane each), consumed one at a time so
    // at most two 64-wide register tiles are live (2 waves/SIMD fit in 256 VGPRs); the compiler
    // barriers keep it from hoisting the next gather's loads over the current one
    f32x16 z[2], q[2];
    gather64(z, P, PROJ_C, 128, bilin(g1x, g1y, w, h), hf);
    asm volatile("" ::: "memory");
    gather64(q, P, PROJ_C, 192, bilin(g2x, g2y, w, h), hf);
#pragma unroll
    for (int ot = 0; ot < 2; ++ot)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int f = ot * 32 + 8 * v + 4 * hf;
        const f32x4 wt = ld4(mlp + E_WT + f), bb = ld4(mlp + E_B0 + f);
#pragma unroll
        for (int e = 0; e < 4; ++e) z[ot][4 * v + e] = (z[ot][4 * v + e] + (q[ot][4 * v + e] + wt[e] * t + bb[e])) * ACC_IN<F16>;
      }
    if constexpr (HRIMG) {   // q_img1 / q_img2 from the high-resolution image (decoding_test :558-583)
      const float* I = im.img + (size_t)item * im.ih * im.iw * IMG_C;
      img_mma(z, mlp + I_E1, img_sample(I, bilin(g1x, g1y, im.iw, im.ih), hf), lane);
      img_mma(z, mlp + I_E2, img_sample(I, bilin(g2x, g2y, im.iw, im.ih), hf), lane);
    }
    asm volatile("" ::: "memory");
    gather64(q, HRF, 64, 0, bilin(g1x, g1y, WW, HH), hf);   // q_feat1 -> W0 columns 0..63
    dec_barrier();
    dma_tiles<DEC2_NW>(B1, rm, E_W1, 4, wv, lane);
    {
      const XT<F16> qs[2] = {xop<F16>(q[0]), xop<F16>(q[1])};
#pragma unroll
      for (int ot = 0; ot < 2; ++ot)
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) tile_mma<F16>(z[ot], B0 + (ot * 4 + kt) * T, qs[kt], lane);
    }
    asm volatile("" ::: "memory");
    gather64(q, HRF, 64, 0, bilin(g2x, g2y, WW, HH), hf);   // q_feat2 -> W0 columns 64..127
    const XT<F16> qs[2] = {xop<F16>(q[0]), xop<F16>(q[1])};
#pragma unroll
    for (int ot = 0; ot < 2; ++ot) {
#pragma unroll
      for (int kt = 2; kt < 4; ++kt) tile_mma<F16>(z[ot], B0 + (ot * 4 + kt) * T, qs[kt - 2], lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) x0[ot][r] = siren_sin<F16>(z[ot][r] * ACC_S<F16>);
    }
  }
  dec_barrier();
  const Bias32 eb1[2] = {bias_ld(mlp + E_B1, hf), bias_ld(mlp + E_B1 + 32, hf)};   // before the DMA
  __builtin_amdgcn_sched_barrier(0);
  auto seg_l23_first = [&](float* dst) {
    dma_tiles<DEC2_NW>(dst, rm, E_W2, 2, wv, lane);
#pragma unroll
    for (int ot = 0; ot < 8; ++ot) dma_tiles<DEC2_NW>(dst + (2 + ot) * T, rm, E_W3 + ot * 8 * T, 1, wv, lane);
  };
  seg_l23_first(B0);
  f32x16 x1[2];
  {
    const XT<F16> xs[2] = {xop<F16>(x0[0]), xop<F16>(x0[1])};
#pragma unroll
    for (int ot = 0; ot < 2; ++ot) {
      f32x16 acc = f32x16{0};
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) tile_mma<F16>(acc, B1 + (ot * 2 + kt) * T, xs[kt], lane);
      x1[ot] = bias_sin<F16>(acc, eb1[ot]);
    }
  }
  const XT<F16> x1s[2] = {xop<F16>(x1[0]), xop<F16>(x1[1])};
  // layer 2 (64 -> 256, sine) streamed tile by tile into the 8 accumulators of layer 3 (256 -> 256):
  // segment kt = W2 rows of tile kt (2 tiles) + column kt of W3 (8 tiles)
  auto seg_l23 = [&](float* dst, int kt) {
    dma_tiles<DEC2_NW>(dst, rm, E_W2 + kt * 2 * T, 2, wv, lane);
#pragma unroll
    for (int ot = 0; ot < 8; ++ot) dma_tiles<DEC2_NW>(dst + (2 + ot) * T, rm, E_W3 + (ot * 8 + kt) * T, 1, wv, lane);
  };
  f32x16 a3[8];
#pragma unroll
  for (int ot = 0; ot < 8; ++ot) a3[ot] = f32x16{0};
  auto l23_step = [&](int kt, bool last) {   // kt = 7 peeled (see k_dec1's feat_step)
    dec_barrier();
    const Bias32 b2 = bias_ld(mlp + E_B2 + kt * 32, hf);   // before the DMA (see k_dec1)
    __builtin_amdgcn_sched_barrier(0);
    float* cur = (kt & 1) ? B1 : B0;
    float* nxt = (kt & 1) ? B0 : B1;
    if (!last) seg_l23(nxt, kt + 1);
    else dma_tiles<DEC2_NW>(nxt, rm, E_W4V, 1, wv, lane);
    f32x16 acc = f32x16{0};
    tile_mma<F16>(acc, cur, x1s[0], lane);
    tile_mma<F16>(acc, cur + T, x1s[1], lane);
    const XT<F16> h2 = xop<F16>(bias_sin<F16>(acc, b2));
#pragma unroll
    for (int ot = 0; ot < 8; ++ot) tile_mma<F16>(a3[ot], cur + (2 + ot) * T, h2, lane);
  };
#pragma unroll 1
  for (int kt = 0; kt < 7; ++kt) l23_step(kt, false);
  l23_step(7, true);
  // layer 3 sine streamed into layer 4 (256 -> 3, linear, VALU dot products); W4 sits in B0 as
  // plain rows, followed by the layer-3 biases (E_W4V_B3; kt = 7 prefetch)
  dec_barrier();
  float o4[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int kt = 0; kt < 8; ++kt) {
    const f32x16 h3 = bias_sin<F16>(a3[kt], B0 + (E_W4V_B3 - E_W4V) + kt * 32, hf);
    narrow_dot<3>(o4, B0, kt, h3, hf);
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) o4[c] += __shfl_xor(o4[c], 32);   // the other lane half's 128 features
  if (valid && hf == 0) {
    const size_t plane = (size_t)HH * WW;
    float* o = out + (size_t)item * 3 * plane + (size_t)py * WW + px;
    // stage 1's flow counts too: the warpgrid clamp above maps a NaN flow to a finite grid, so an
    // out-of-range flow_imnet operand would otherwise leave a finite but wrong pixel
    bool bad = not_finite((fv[0] + fv[1]) + (fv[2] + fv[3]));
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float v = o4[c] + mlp[E_B4 + c];
      bad |= not_finite(v);
      o[c * plane] = v;
    }
    if (F16) report_range(status, bad);
  }
}


// ---------------------------------------------------------------------------------------------
// k_dec2q: stage 2 (split-fp16, LR-projection image inputs) at 16 pixels per wave on
// v_mfma_f32_16x16x32_f16.  Lane l = (p = l & 15: the wave's pixel, q = l >> 4).  A 32-feature register
// tile is two 16x16 accumulators: lane (p, q) holds features 16 s + 4 q + i (s = 0, 1; i = 0..3) of pixel
// p -- which is also the B-operand order of the next layer's K (dec_layout.h Q_*), so features stay in
// registers between layers as in k_dec2.  The layer-3 state halves (8 tiles x 8 floats = 64 VGPRs): 128 VGPRs,
// four waves per SIMD.
// Weight streaming (round 6): every workgroup streams the whole 372-KB weight set through its LDS, so the
// stream is paid once per workgroup; its memory traffic costs ~10 % of the kernel (pieces issued out of range,
// DEC_EXP 3: profiles/r06_dec_probe3.log).  Workgroups are
// DEC2Q_NW waves (8: 128 pixels, two per CU; 16: 256 pixels, one per CU) and a segment is the layer-2 / -3
// weights of DEC2Q_KTS whole layer-2 tiles kt (W2 rows kt + W3 column kt: 10 tiles each), double-buffered in
// 2 x 40 KB (KTS 1) or 2 x 80 KB (KTS 2): the weight bytes per pixel halve / quarter and one barrier per kt
// (or per two) replaces two.  Every wave issues the same number of LDS-DMA pieces per segment (5), so the
// compiler's vmcnt bookkeeping stays exact.
// Gathers: each lane fetches its own quarter of a 64-channel block (16 corner loads in flight).
constexpr int DEC2Q_NWV = DEC2Q_NW;
#if DEC_TRACE
// diagnostic (stif_dec_trace_set): per k_dec2q wave 8 u32 -- life, gathers (incl. the flow load), segment-barrier
// waits, layer-2/3 span (its barriers included) -- s_memtime ticks
__device__ unsigned* g_dtrace;
#endif
constexpr int KTS = DEC2Q_KTS;            // layer-2 tiles per segment
constexpr int SEGQ = 10 * KTS;            // tiles per segment
static_assert(40 * KTS % DEC2Q_NWV == 0 && 32 % DEC2Q_NWV == 0 && 16 % DEC2Q_NWV == 0 && 8 % KTS == 0,
              "k_dec2q: every wave issues the same number of LDS-DMA pieces");
static_assert((DEC2Q_NWV == 8 || DEC2Q_NWV == 16) && 2 * SEGQ * T * 4 * (16 / DEC2Q_NWV) <= 160 * 1024,
              "k_dec2q: 16 waves per CU (four per SIMD) in 8- or 16-wave workgroups, their LDS within 160 KB");
struct R32 {
  f32x4 s[2];
};
struct XQ {
  f16x8 h, l;
};
STIF_DEV XQ xq(const R32& x) {
  XQ o;
  split_f16x3(x.s[0], x.s[1], o.h, o.l);
  return o;
}
STIF_DEV void tile_q(R32& acc, const float* t, const XQ& x, int lane) {
  const float* b = t + lane * 4;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const f16x8 ah = ldh8(b + (2 * s) * 256), al = ldh8(b + (2 * s + 1) * 256);
    acc.s[s] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, x.h, acc.s[s], 0, 0, 0);
    acc.s[s] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, x.h, acc.s[s], 0, 0, 0);
    acc.s[s] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, x.l, acc.s[s], 0, 0, 0);
  }
  __builtin_amdgcn_sched_barrier(0);
}
// this lane's biases of a register tile whose features start at b (they carry omega_0 / 2 pi, pack.cpp)
STIF_DEV R32 bias_q(const float* __restrict__ b, int q) {
  R32 o;
#pragma unroll
  for (int s = 0; s < 2; ++s) o.s[s] = ld4(b + 16 * s + 4 * q);
  return o;
}
// sin(z * 2^-14 + b) of a register tile, biases preloaded (bias_q)
STIF_DEV R32 bias_sin_q(const R32& z, const R32& bb) {
  R32 o;
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int e = 0; e < 4; ++e) o.s[s][e] = siren_sin<1>(fmaf(z.s[s][e], ACC_S<1>, bb.s[s][e]));
  return o;
}
STIF_DEV R32 bias_sin_q(const R32& z, const float* __restrict__ b, int q) { return bias_sin_q(z, bias_q(b, q)); }
// bilinear sample of this lane's channels c0 + 32 ot + 16 s + 4 q .. + 3 (ot, s = 0, 1) of an NHWC map
STIF_DEV void gather_q(R32* dst, const float* __restrict__ base, int stride, int c0, const Bilin& b, int q) {
  const int c = c0 + 4 * q;
  const float* p00 = base + (size_t)b.o00 * stride + c;
  const float* p01 = base + (size_t)b.o01 * stride + c;
  const float* p10 = base + (size_t)b.o10 * stride + c;
  const float* p11 = base + (size_t)b.o11 * stride + c;
  f32x4 cr[4][4];
#pragma unroll
  for (int g = 0; g < 4; ++g) {   // g = 2 ot + s: channel offset 16 g
    cr[g][0] = ld4(p00 + 16 * g);
    cr[g][1] = ld4(p01 + 16 * g);
    cr[g][2] = ld4(p10 + 16 * g);
    cr[g][3] = ld4(p11 + 16 * g);
  }
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    f32x4 v = b.w00 * cr[g][0] + b.w01 * cr[g][1] + b.w10 * cr[g][2] + b.w11 * cr[g][3];
    asm volatile("" : "+v"(v));
    dst[g >> 1].s[g & 1] = v;
  }
}

__global__ __launch_bounds__(DEC2Q_NWV * 64) __attribute__((amdgpu_waves_per_eu(4))) void k_dec2q(
    const float* __restrict__ proj, const float* __restrict__ mlp, const float* __restrict__ hrfeat,
    const float* __restrict__ flow, stif_dec_tables tb, const float* __restrict__ tq, float* __restrict__ out, int n,
    int h, int w, int HH, int WW, int* status) {
  __shared__ __attribute__((aligned(16))) float wbuf[2 * SEGQ * T];
#if DEC_TRACE
  const unsigned tr0 = (unsigned)__builtin_amdgcn_s_memtime();
  unsigned tr_g = 0, tr_b = 0, tr_l23 = 0, tr_x;
#define DTR_BEGIN() tr_x = (unsigned)__builtin_amdgcn_s_memtime()
#define DTR_END(acc) acc += (unsigned)__builtin_amdgcn_s_memtime() - tr_x
#else
#define DTR_BEGIN()
#define DTR_END(acc)
#endif
  const int lane = threadIdx.x & 63, q = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  constexpr int NW = DEC2Q_NWV;
  float* const B0 = wbuf;
  float* const B1 = wbuf + SEGQ * T;
  const __amdgpu_buffer_rsrc_t rm = mlp_rsrc(mlp);
  // segments: [L0: 8 tiles] in B0, [L1: 4 tiles] in B1, then per segment s the tiles of kt = KTS s .. KTS s + KTS - 1
  // ([W2 rows kt (2) | W3 column kt, ot 0-7 (8)] each) alternating B0 / B1, then [W4 rows + B3]
  dma_tiles<NW>(B0, rm, Q_W0, 8, wv, lane);   // tile index 4 ot + kt
  auto seg_l23 = [&](float* dst, int sg) {
#pragma unroll
    for (int r = 0; r < 40 * KTS / NW; ++r) {
      const int i = wv + r * NW;                // piece i: tile j = i / 4 of the segment, quarter i % 4
      const int j = i >> 2, k = j / 10, jj = j - 10 * k, kt = sg * KTS + k;
      const int src = (jj < 2 ? Q_W2 + (kt * 2 + jj) * T : Q_W3 + ((jj - 2) * 8 + kt) * T) + (i & 3) * 256;
      dec_dma(rm, dst + j * T + (i & 3) * 256, lane, src * 4);
    }
  };
  const long long total = (long long)n * HH * WW;
  const long long pix = ((long long)xcd_block(blockIdx.x, gridDim.x) * NW + wv) * 16 + (lane & 15);
  const bool valid = pix < total;
  const long long pc = valid ? pix : total - 1;
  const int item = (int)(pc / ((long long)HH * WW));
  const int rem = (int)(pc - (long long)item * HH * WW);
  const int py = rem / WW, px = rem - py * WW;
  const float t = tq[item];
  const float* P = proj + (size_t)item * h * w * PROJ_C;
  const float* HRF = hrfeat + (size_t)item * HH * WW * 64;

  // warpgrid (warplayer.py:25-39) and the decoder's clamp (Sakuya_arch_test.py:428,441), as k_dec2
  DTR_BEGIN();
  const f32x4 fv = ld4(flow + (size_t)pc * 4);
  const float lo = -1.f + 1e-6f, hi = 1.f - 1e-6f;
  const float dx = ((float)WW - 1.f) / 2.f, dy = ((float)HH - 1.f) / 2.f;
  const float bx = tb.lin_x[px], by = tb.lin_y[py];
  const float g1x = fminf(fmaxf(bx + fv[0] / dx, lo), hi), g1y = fminf(fmaxf(by + fv[1] / dy, lo), hi);
  const float g2x = fminf(fmaxf(bx + fv[2] / dx, lo), hi), g2y = fminf(fmaxf(by + fv[3] / dy, lo), hi);

  // ---- encode_imnet layer 0: W[:, :128] . [q_feat1 | q_feat2] + P3(grid1) + P4(grid2) + w_t t + b
  R32 x0[2];
  {
    R32 z[2], g[2];
    gather_q(z, P, PROJ_C, 128, bilin(g1x, g1y, w, h), q);
    asm volatile("" ::: "memory");
    gather_q(g, P, PROJ_C, 192, bilin(g2x, g2y, w, h), q);
#pragma unroll
    for (int ot = 0; ot < 2; ++ot)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int f = 32 * ot + 16 * s + 4 * q;
        const f32x4 wt = ld4(mlp + E_WT + f), bb = ld4(mlp + E_B0 + f);
#pragma unroll
        for (int e = 0; e < 4; ++e)
          z[ot].s[s][e] = (z[ot].s[s][e] + (g[ot].s[s][e] + wt[e] * t + bb[e])) * ACC_IN<1>;
      }
    asm volatile("" ::: "memory");
    gather_q(g, HRF, 64, 0, bilin(g1x, g1y, WW, HH), q);   // q_feat1 -> W0 columns 0..63
    DTR_END(tr_g);
    DTR_BEGIN();
    dec_barrier();                                      // layer 0 landed in B0
    DTR_END(tr_b);
    dma_tiles<NW>(B1, rm, Q_W1, 4, wv, lane);
    {
      const XQ qs[2] = {xq(g[0]), xq(g[1])};
#pragma unroll
      for (int ot = 0; ot < 2; ++ot)
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) tile_q(z[ot], B0 + (ot * 4 + kt) * T, qs[kt], lane);
    }
    asm volatile("" ::: "memory");
    DTR_BEGIN();
    gather_q(g, HRF, 64, 0, bilin(g2x, g2y, WW, HH), q);   // q_feat2 -> W0 columns 64..127
    DTR_END(tr_g);
    const XQ qs[2] = {xq(g[0]), xq(g[1])};
#pragma unroll
    for (int ot = 0; ot < 2; ++ot) {
#pragma unroll
      for (int kt = 2; kt < 4; ++kt) tile_q(z[ot], B0 + (ot * 4 + kt) * T, qs[kt - 2], lane);
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int e = 0; e < 4; ++e) x0[ot].s[s][e] = siren_sin<1>(z[ot].s[s][e] * ACC_S<1>);
    }
  }
  DTR_BEGIN();
  dec_barrier();   // layer 1 landed in B1; every wave is done with layer 0's B0
  DTR_END(tr_b);
  // layer-1 biases before the next segment's LDS-DMA: vmcnt counts in issue order, so a bias load issued
  // after the DMA would wait for the DMA too (as k_dec1 / k_dec2 do)
  const R32 eb1[2] = {bias_q(mlp + E_B1, q), bias_q(mlp + E_B1 + 32, q)};
  __builtin_amdgcn_sched_barrier(0);
  seg_l23(B0, 0);
  R32 x1[2];
  {
    const XQ xs[2] = {xq(x0[0]), xq(x0[1])};
#pragma unroll
    for (int ot = 0; ot < 2; ++ot) {
      R32 acc;
      acc.s[0] = acc.s[1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) tile_q(acc, B1 + (ot * 2 + kt) * T, xs[kt], lane);
      x1[ot] = bias_sin_q(acc, eb1[ot]);
    }
  }
  const XQ x1s[2] = {xq(x1[0]), xq(x1[1])};
  // layer 2 (64 -> 256, sine) streamed tile by tile into the 8 register tiles of layer 3 (256 -> 256)
  R32 a3[8];
#pragma unroll
  for (int ot = 0; ot < 8; ++ot) a3[ot].s[0] = a3[ot].s[1] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int NSEG = 8 / KTS;
  auto l23_step = [&](int sg, bool last) {
    DTR_BEGIN();
    dec_barrier();   // segment sg landed; every wave is done with the other buffer
    DTR_END(tr_b);
    R32 b2[KTS];
#pragma unroll
    for (int k = 0; k < KTS; ++k) b2[k] = bias_q(mlp + E_B2 + (sg * KTS + k) * 32, q);   // before the DMA
    __builtin_amdgcn_sched_barrier(0);
    float* cur = (sg & 1) ? B1 : B0;
    float* nxt = (sg & 1) ? B0 : B1;
    auto dma_next = [&]() {
      if (!last) seg_l23(nxt, sg + 1);
      else dma_tiles<NW>(nxt, rm, E_W4V, 1, wv, lane);
    };
    if (!DEC_DMA_LATE) dma_next();
#pragma unroll
    for (int k = 0; k < KTS; ++k) {
      const float* sk = cur + k * 10 * T;
      R32 acc;
      acc.s[0] = acc.s[1] = f32x4{0.f, 0.f, 0.f, 0.f};
      tile_q(acc, sk, x1s[0], lane);
      tile_q(acc, sk + T, x1s[1], lane);
      if (DEC_DMA_LATE && k == 0) dma_next();
      const XQ h2 = xq(bias_sin_q(acc, b2[k]));
#pragma unroll
      for (int ot = 0; ot < 8; ++ot) tile_q(a3[ot], sk + (2 + ot) * T, h2, lane);
    }
  };
#if DEC_TRACE
  const unsigned tr_l0 = (unsigned)__builtin_amdgcn_s_memtime();
#endif
#pragma unroll 1
  for (int sg = 0; sg < NSEG - 1; ++sg) l23_step(sg, false);
  l23_step(NSEG - 1, true);
#if DEC_TRACE
  tr_l23 = (unsigned)__builtin_amdgcn_s_memtime() - tr_l0;
#endif
  // layer 3 sine streamed into layer 4 (256 -> 3, VALU dot products over this lane's 64 features); W4 rows
  // and the layer-3 biases in the buffer the last segment did not use (k_dec2's tile)
  dec_barrier();
  float* const B4 = ((NSEG - 1) & 1) ? B0 : B1;
  float o4[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int kt = 0; kt < 8; ++kt) {
    const R32 h3 = bias_sin_q(a3[kt], B4 + (E_W4V_B3 - E_W4V) + kt * 32, q);
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const f32x4 wr = ld4(B4 + c * 256 + kt * 32 + 16 * s + 4 * q);
#pragma unroll
        for (int e = 0; e < 4; ++e) o4[c] = fmaf(wr[e], h3.s[s][e], o4[c]);
      }
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) {   // the other three lane groups' features
    o4[c] += __shfl_xor(o4[c], 16);
    o4[c] += __shfl_xor(o4[c], 32);
  }
  if (valid && q == 0) {
    const size_t plane = (size_t)HH * WW;
    float* o = out + (size_t)item * 3 * plane + (size_t)py * WW + px;
    bool bad = not_finite((fv[0] + fv[1]) + (fv[2] + fv[3]));
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float v = o4[c] + mlp[E_B4 + c];
      bad |= not_finite(v);
      o[c * plane] = v;
    }
    report_range(status, bad);
  }
#if DEC_TRACE
  if (g_dtrace && lane == 0) {
    typedef unsigned u32x4t __attribute__((ext_vector_type(4)));
    *reinterpret_cast<u32x4t*>(g_dtrace + ((size_t)blockIdx.x * NW + wv) * 8) =
        u32x4t{(unsigned)__builtin_amdgcn_s_memtime() - tr0, tr_g, tr_b, tr_l23};
  }
#endif
#undef DTR_BEGIN
#undef DTR_END
}

__global__ __launch_bounds__(256) void k_pack_lr(const float* __restrict__ f0, const float* __restrict__ f1,
                                                 const float* __restrict__ f2, const float* __restrict__ x,
                                                 float* __restrict__ out, int n, int h, int w) {
  const long long npix = (long long)n * h * w;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < npix * 50; e += (long long)gridDim.x * 256) {
    const long long pix = e / 50;
    const int q = (int)(e - pix * 50);
    f32x4 v;
    if (q < 48) {
      const float* src = q < 16 ? f0 : (q < 32 ? f1 : f2);
      v = ld4(src + pix * 64 + (q & 15) * 4);
    } else {
      const int item = (int)(pix / ((long long)h * w));
      const long long yx = pix - (long long)item * h * w;
      const float* xi = x + (size_t)item * 6 * h * w + yx;   // [2][3][h][w] of this item
      const size_t pl = (size_t)h * w;
      if (q == 48) { v[0] = xi[0]; v[1] = xi[pl]; v[2] = xi[2 * pl]; v[3] = xi[3 * pl]; }
      else { v[0] = xi[4 * pl]; v[1] = xi[5 * pl]; v[2] = 0.f; v[3] = 0.f; }
    }
    st4(out + pix * SRC_C + q * 4, v);
  }
}

__global__ __launch_bounds__(256) void k_blend4(const float* __restrict__ p0, const float* __restrict__ p1,
                                                const float* __restrict__ p2, const float* __restrict__ p3,
                                                const float* __restrict__ w0, const float* __restrict__ w1,
                                                const float* __restrict__ w2, const float* __restrict__ w3,
                                                float* __restrict__ out, long long total, int plane) {
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const int q = (int)(e % plane);
    float r = p0[e] * w0[q];   // ret = 0 + pred_0 * w_0 + ... in the reference's order (:1082-1084)
    r += p1[e] * w1[q];
    r += p2[e] * w2[q];
    r += p3[e] * w3[q];
    out[e] = r;
  }
}

bool tables_ok(const stif_dec_tables* t) {
  return t && t->near_y && t->rel_y && t->by0 && t->by1 && t->wy0 && t->wy1 && t->lin_y && t->near_x &&
         t->rel_x && t->bx0 && t->bx1 && t->wx0 && t->wx1 && t->lin_x;
}

}  // namespace

extern "C" int stif_dec_pack_lr(const float* f0, const float* f1, const float* f2, const float* x, float* out,
                                int n, int h, int w, void* stream) {
  if (!f0 || !f1 || !f2 || !x || !out || n < 1 || h < 1 || w < 1)
    return stif_fail(STIF_E_INVALID, "stif_dec_pack_lr: bad arguments");
  const long long work = (long long)n * h * w * 50;
  long long blocks = (work + 255) / 256;
  if (blocks > 1 << 16) blocks = 1 << 16;
  hipLaunchKernelGGL(k_pack_lr, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, f0, f1, f2, x, out, n, h,
                     w);
  return stif_check_launch("stif_dec_pack_lr");
}

namespace {

bool image_ok(const stif_dec_image* im) {
  return !im || (im->img && im->ih > 0 && im->iw > 0 && im->by0 && im->by1 && im->wy0 && im->wy1 && im->bx0 &&
                 im->bx1 && im->wx0 && im->wx1);
}

template <int MODE, bool HRIMG>
void launch_dec1(bool f16, long long total, hipStream_t st, const float* proj, const float* mlp,
                 const stif_dec_tables& tb, const stif_dec_image& im, const float* t, float* hrfeat, float* flow, int n,
                 int h, int w, int HH, int WW) {
  constexpr int nw = NW1<MODE, HRIMG>;
  const long long blocks = (total + nw * 32 - 1) / (nw * 32);
  if (f16)
    hipLaunchKernelGGL((k_dec1<MODE, HRIMG, 1>), dim3((unsigned)blocks), dim3(nw * 64), 0, st, proj, mlp, tb, im,
                       t, hrfeat, flow, n, h, w, HH, WW);
  else
    hipLaunchKernelGGL((k_dec1<MODE, HRIMG, 0>), dim3((unsigned)blocks), dim3(nw * 64), 0, st, proj, mlp, tb, im,
                       t, hrfeat, flow, n, h, w, HH, WW);
}

}  // namespace

extern "C" int stif_dec_stage1_ex(const float* proj, const float* mlp, const stif_dec_tables* tab,
                                  const stif_dec_image* img, const float* t, float* hrfeat, float* flow, int n, int h,
                                  int w, int HH, int WW, int flags, int* status, void* stream) {
  (void)status;   // stage 2 checks both stage-1 outputs it reads (flow, and HRfeat through the RGB; stif.h)
  const bool f16 = flags & STIF_CONV_F16X3;
  if (!proj || !mlp || !tables_ok(tab) || !image_ok(img) || !t || !hrfeat || !flow || n < 1 || h < 1 || w < 1 ||
      HH < 2 || WW < 2 || (!tab->hr_y) != (!tab->hr_x))
    return stif_fail(STIF_E_INVALID, "stif_dec_stage1: bad arguments");
  const long long total = (long long)n * HH * WW;
  hipStream_t st = (hipStream_t)stream;
  const stif_dec_image im = img ? *img : stif_dec_image{};
  if (tab->hr_y) {   // remapped HRfeat operand: the whole HRfeat map first, then the flow stage
    launch_dec1<1, false>(f16, total, st, proj, mlp, *tab, im, t, hrfeat, flow, n, h, w, HH, WW);
    if (img) launch_dec1<2, true>(f16, total, st, proj, mlp, *tab, im, t, hrfeat, flow, n, h, w, HH, WW);
    else launch_dec1<2, false>(f16, total, st, proj, mlp, *tab, im, t, hrfeat, flow, n, h, w, HH, WW);
  } else if (img) {
    launch_dec1<0, true>(f16, total, st, proj, mlp, *tab, im, t, hrfeat, flow, n, h, w, HH, WW);
  } else if (DEC1_RES && f16) {   // resident-weight feat and flow kernels (persistent, one workgroup per CU)
    const long long nblk = (total + 31) / 32;
    const unsigned grid = (unsigned)std::max<long long>(1, std::min<long long>(stif_num_cus(), (nblk + RW - 1) / RW));
    hipLaunchKernelGGL(k_dec1f, dim3(grid), dim3(RW * 64), 0, st, proj, mlp, *tab, t, hrfeat, n, h, w, HH, WW);
    hipLaunchKernelGGL(k_dec1l, dim3(grid), dim3(RW * 64), 0, st, proj, mlp, *tab, t, hrfeat, flow, n, h, w, HH, WW);
  } else {
    launch_dec1<0, false>(f16, total, st, proj, mlp, *tab, im, t, hrfeat, flow, n, h, w, HH, WW);
  }
  return stif_check_launch("stif_dec_stage1");
}

extern "C" int stif_dec_stage1(const float* proj, const float* mlp, const stif_dec_tables* tab,
                               const stif_dec_image* img, const float* t, float* hrfeat, float* flow, int n, int h,
                               int w, int HH, int WW, void* stream) {
  return stif_dec_stage1_ex(proj, mlp, tab, img, t, hrfeat, flow, n, h, w, HH, WW, 0, nullptr, stream);
}

extern "C" int stif_dec_stage2_ex(const float* proj, const float* mlp, const float* hrfeat, const float* flow,
                                  const stif_dec_tables* tab, const stif_dec_image* img, const float* t, float* out,
                                  int n, int h, int w, int HH, int WW, int flags, int* status, void* stream) {
  const bool f16 = flags & STIF_CONV_F16X3;
  if (!proj || !mlp || !hrfeat || !flow || !tables_ok(tab) || !image_ok(img) || !t || !out || n < 1 || h < 1 ||
      w < 1 || HH < 2 || WW < 2)
    return stif_fail(STIF_E_INVALID, "stif_dec_stage2: bad arguments");
  const long long total = (long long)n * HH * WW;
  const long long blocks = (total + DEC2_NW * 32 - 1) / (DEC2_NW * 32);
  const stif_dec_image im = img ? *img : stif_dec_image{};
  hipStream_t st = (hipStream_t)stream;
  if (DEC2_Q16 && f16 && !img) {
    const long long qblocks = (total + DEC2Q_NWV * 16 - 1) / (DEC2Q_NWV * 16);
    hipLaunchKernelGGL(k_dec2q, dim3((unsigned)qblocks), dim3(DEC2Q_NWV * 64), 0, st, proj, mlp, hrfeat, flow, *tab, t,
                       out, n, h, w, HH, WW, status);
    return stif_check_launch("stif_dec_stage2");
  }
  const dim3 g((unsigned)blocks), b(DEC2_NW * 64);
  if (img && f16) hipLaunchKernelGGL((k_dec2<true, 1>), g, b, 0, st, proj, mlp, hrfeat, flow, *tab, im, t, out, n, h, w, HH, WW, status);
  else if (img) hipLaunchKernelGGL((k_dec2<true, 0>), g, b, 0, st, proj, mlp, hrfeat, flow, *tab, im, t, out, n, h, w, HH, WW, status);
  else if (f16) hipLaunchKernelGGL((k_dec2<false, 1>), g, b, 0, st, proj, mlp, hrfeat, flow, *tab, im, t, out, n, h, w, HH, WW, status);
  else hipLaunchKernelGGL((k_dec2<false, 0>), g, b, 0, st, proj, mlp, hrfeat, flow, *tab, im, t, out, n, h, w, HH, WW, status);
  return stif_check_launch("stif_dec_stage2");
}

extern "C" int stif_dec_stage2(const float* proj, const float* mlp, const float* hrfeat, const float* flow,
                               const stif_dec_tables* tab, const stif_dec_image* img, const float* t, float* out, int n,
                               int h, int w, int HH, int WW, void* stream) {
  return stif_dec_stage2_ex(proj, mlp, hrfeat, flow, tab, img, t, out, n, h, w, HH, WW, 0, nullptr, stream);
}

#if DEC_TRACE
extern "C" int stif_dec_trace_set(unsigned* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_dtrace), &p, sizeof(p)) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int stif_dec_blend4(const float* const* pred, const float* const* wgt, float* out, int n, int HH, int WW,
                               void* stream) {
  if (!pred || !wgt || !out || n < 1 || HH < 1 || WW < 1) return stif_fail(STIF_E_INVALID, "stif_dec_blend4: bad arguments");
  for (int k = 0; k < 4; ++k)
    if (!pred[k] || !wgt[k]) return stif_fail(STIF_E_INVALID, "stif_dec_blend4: null input");
  const long long total = (long long)n * 3 * HH * WW;
  const long long blocks = std::min<long long>((total + 255) / 256, 1 << 16);
  hipLaunchKernelGGL(k_blend4, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, pred[0], pred[1], pred[2],
                     pred[3], wgt[0], wgt[1], wgt[2], wgt[3], out, total, HH * WW);
  return stif_check_launch("stif_dec_blend4");
}
