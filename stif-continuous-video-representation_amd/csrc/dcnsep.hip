// Fused DCN_sep for gfx950: conv_offset_mask (64 -> 216, 3x3) + chunk / cat / sigmoid + the
// modulated deformable conv (64 -> 64, 3x3, 8 deformable groups) in one kernel; the 216-channel
// offset/mask map never reaches HBM.
//
// Reference: DCN_sep.forward (DCNv2/dcn_v2.py:127-140) -> _DCNv2 -> dcn_v2_cuda_forward
// (src/cuda/dcn_v2_cuda.cu:42-172) with the sampling of modulated_deformable_im2col_gpu_kernel /
// dmcn_im2col_bilinear (dcn_v2_im2col_cuda.cu:25-54,125-195).
//
// Workgroup = NW waves (default 4: two 80-KB workgroups per CU), tile = NW output rows x 32 columns,
// wave w = output row w (lane & 31 = column).  Lane half h works on the deformable groups h, h + 2,
// h + 4, h + 6 throughout.
//
// Phase 1, the offset/mask conv as a direct implicit GEMM with the WEIGHTS as the MFMA A operand:
// D[om row][pixel] += W[om row][k] X[k][pixel] on split-fp16 v_mfma_f32_32x32x16_f16 (f16x3, fp32
// accumulation), 216 rows in 7 M-tiles.  The rows are permuted at packing time (stif_pack_conv_weight,
// STIF_PACK_DCNSEP) so that the accumulator registers of lane (pixel p, half h) hold exactly the
// (dy, dx, mask) of every tap of its four groups -- the offsets go from the MFMA accumulators
// straight into the bilinear sampling, with no exchange, no LDS round trip and no HBM traffic.
// K = 36 steps (16-channel chunk c, tap t); per step a wave reads its pixels' 8 channels of the staged
// input halo (two ds_read_b128), splits them once and runs 3 MFMAs per M-tile (21 MFMAs per step;
// 112 accumulator VGPRs).  The input halo ((NW + 2) x 34 pixels, one 16-channel chunk, 80-B pixel pitch:
// conflict-free reads) and the packed weights of each step (a 3-slot ring) arrive by LDS-DMA ahead of
// use; one barrier per step.
//
// Phase 2, the deformable conv, two groups per K step: per group pair (2a, 2a + 1) the 16-channel input
// tile with a 2-px margin and the pair's weight fragments are LDS-DMA'd (NW 8: one pair ahead, pair 0
// during phase 1; NW 4: into one buffer while the CU's other workgroup computes); for every tap t lane
// half h samples group 2a + h's 8 channels at its pixel (global fallback outside the margin) -- the 16
// K values of one 32x32x16 MFMA -- and runs 3 MFMAs per 32-cout half:
// 9 K steps per pair instead of 10 for two single groups (tap pairs); epilogue through LDS as k_dcn.
#include "abi_util.h"
#include "stif.h"
#include "stif_common.h"
#include "tuning.h"

#include <algorithm>

namespace {

// NW = 4 (tuning.h): 4 output rows per tile, two 80-KB workgroups per CU; NW = 8: one 152-KB workgroup per
// CU with the next group pair staged ahead (slower)
constexpr int NW = DCNSEP_NW;                 // waves = output rows per tile
constexpr int TW = 32;                        // output columns per tile
// phase 1
constexpr int MT = 7;                         // offset/mask M-tiles (224 rows >= 216)
constexpr int HC1 = TW + 2;                   // halo columns (NW + 2 halo rows)
constexpr int PX_F = 20;                      // floats per staged halo pixel: 16 channels + 4 pad
constexpr int D_SLOTS = (NW + 2) * HC1 * 5;   // 16-B slots per data chunk
constexpr int D_INS = NW == 8 ? 32 : 16;      // DMA instructions per data chunk (the last ones partly pad)
constexpr int D_F = D_INS * 256;              // floats per data buffer
constexpr int KSTEPS = 36;                    // k = 9 c + t: 16-channel chunk c, tap t
constexpr int WK_F = MT * 2 * 256;            // packed weights of one step: [M-tile][plane][lane][8 halves]
constexpr int WK_INS = 16;                    // DMA instructions per step (14 carry data)
constexpr int RING = 3;
// phase 2
constexpr int M = 2;                          // staged margin around the 3x3 footprint
constexpr int TR = NW + 2 + 2 * M, TC = TW + 2 + 2 * M, TP = TC;
constexpr int T_EL = TR * 4 * TP;             // 16-B elements of the staged tile: [row][channel quad][col]
constexpr int T_INST = (T_EL + 63) / 64;      // 34 (NW 8), 24 (NW 4)
constexpr int WP_F = 9 * 2 * 2 * 256;         // packed B fragments of one group pair (36 KB)
constexpr int P_INS = ((T_INST + WP_F / 256 + NW - 1) / NW) * NW;   // pair stage (tile + weights + pad)
constexpr bool PAIR_AHEAD = NW == 8;          // phase 2 double-buffered (pair 0 staged during phase 1)
static_assert(P_INS % NW == 0 && D_INS % NW == 0 && WK_INS % NW == 0, "stage sizes");
static_assert(D_SLOTS <= D_INS * 64 && MT * 2 <= WK_INS, "phase-1 stages");
// LDS map (floats).  NW 8 -- phase 1: data chunks D0, D1 and the weight ring; the stage of group pair 0
// (tile X, weights XW) lands in D0 (free once chunk 2 is done) and above the ring; phase 2: pairs
// alternate between X and Y (tile Y over D1, weights YW over the ring).  NW 4 -- phase 1: D0, D1, ring
// (80 KB); phase 2: one pair buffer X over them.  The epilogue blocks reuse D0.
constexpr int PW_PAD_F = (P_INS - T_INST) * 256;    // pair weight region incl. the pad instructions
constexpr int OFF_D0 = 0, OFF_D1 = PAIR_AHEAD ? T_INST * 256 : D_F, OFF_W = OFF_D1 + D_F;
constexpr int OFF_XT = 0, OFF_XW = PAIR_AHEAD ? OFF_W + RING * 4096 : T_INST * 256;
constexpr int OFF_YT = T_INST * 256, OFF_YW = OFF_YT + T_INST * 256;
constexpr int LDS_F = PAIR_AHEAD ? OFF_XW + PW_PAD_F : OFF_W + RING * 4096;
static_assert(D_F <= OFF_D1 && WK_F <= 4096 && NW * 1024 <= D_F && LDS_F * 4 <= (NW == 8 ? 160 : 80) * 1024 &&
              (PAIR_AHEAD ? OFF_YW + PW_PAD_F <= OFF_XW : OFF_XW + PW_PAD_F <= LDS_F), "LDS map");

#if DCNSEP_TP_DUMP
// diagnostic dump target (stif_dcnsep_dump_set): per thread 4 pairs x (9 taps x 8 blended samples + 32 accumulators),
// then the 112 phase-1 results phase 2 reads (offsets, sigmoid(mask)), then 4 pairs x 9 taps x the 4 corner weights
__device__ float* g_tp_dump;
// + pair 0 tap 0's eight corner vectors and four weights stored right before the blend (TP_DUMP 2: before, else after)
constexpr int TPD_F = 4 * (9 * 8 + 32) + 112 + 4 * 9 * 4 + 32;
#endif

#if DCNSEP_TRACE
// per wave 8 u32: start (low bits), phase-1 end, phase-2 end, end (relative to start), phase-1 vmcnt-wait sum,
// phase-1 barrier sum, phase-2 stage + wait sum, workgroup id
__device__ unsigned* g_trace;
STIF_DEV unsigned tstamp() { return (unsigned)__builtin_amdgcn_s_memtime(); }
#endif

// vmcnt waits with an immediate operand (the counts are wave-uniform)
STIF_DEV void wait_vm(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

template <int EPI>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(DCNSEP_WPE))) void k_dcn_sep(stif_dcn_sep_args a) {
  __shared__ __attribute__((aligned(16))) float smem[LDS_F];
#if DCNSEP_SOLO   // diagnostic: 48 KB of unused LDS, so only one workgroup fits on a CU
  __shared__ float solo_pad[12288];
  if (a.H < 0) reinterpret_cast<volatile float*>(solo_pad)[threadIdx.x] = 0.f;
#endif
  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, hf = lane >> 5;
#if DCNSEP_TRACE
  const unsigned tr_t0 = tstamp();
  unsigned tr_vm = 0, tr_bar = 0, tr_p2w = 0, tr_p1e = 0, tr_p2e = 0;
#endif
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
  const float* wt = a.w[g];
  const int oy0 = ty * NW, ox0 = tx * TW;
  const int oy = oy0 + wv, ox = ox0 + l32;
  const bool pix_ok = oy < H && ox < W;
  const unsigned img_bytes = (unsigned)((size_t)H * W * 64 * 4);
  const __amdgpu_buffer_rsrc_t rfea = __builtin_amdgcn_make_buffer_rsrc((void*)fea, (short)0, (int)img_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void*)in, (short)0, (int)img_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rwom =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.w_om[g], (short)0, KSTEPS * WK_F * 4, 0x00020000);

  // ---------------------------------------------------------------- stages (LDS-DMA)
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
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rfea, dst + i * 256, 16, voff, 0, 0, DCNSEP_NT);
    }
  };
  // the packed weights of step k (the instructions past the step's 14 KB load zeros)
  // DCNSEP_WTRIM: only the 14 pieces that carry data are issued (waves 0-1: 4, waves 2-3: 3, wave-uniform counts the
  // phase-1 waits follow); else 16 with two all-pad pieces (every wave 4)
  auto stage_w = [&](int k, int slot) {
    float* dst = smem + OFF_W + slot * 4096;
#pragma unroll
    for (int j = 0; j < WK_INS / NW; ++j) {
      const int i = wv + j * NW;
      if (DCNSEP_WTRIM && i >= MT * 2) continue;   // wave-uniform
      const unsigned voff = i < MT * 2 ? (unsigned)((k * WK_F + i * 256) * 4 + lane * 16) : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rwom, dst + i * 256, 16, voff, 0, 0, 0);
    }
  };
  // phase-2 stage of group pair pa: the [row][channel quad][col][4] tile of channels 16 pa .. 16 pa + 15
  // and the pair's B fragments (instructions 0..33 tile, 34..69 weights, 70..71 pad)
  const int ty0 = oy0 - 1 - M, tx0 = ox0 - 1 - M;
  auto stage_pair = [&](int pa, float* st, float* sw) {
    const float* wc = wt + (size_t)pa * WP_F;
#pragma unroll 1
    for (int j = 0; j < P_INS / NW; ++j) {
      const int i = wv + j * NW;   // wave-uniform
      if (i >= T_INST && i < T_INST + WP_F / 256) {
        __builtin_amdgcn_global_load_lds(wc + ((i - T_INST) * 64 + lane) * 4, sw + (i - T_INST) * 256, 16, 0, 0);
      } else {
        const int e = i * 64 + lane;
        const int col = e % TP, rq = e / TP, q = rq & 3, row = rq >> 2;
        const int y = ty0 + row, x = tx0 + col;
        const bool ok = (i < T_INST) & (e < T_EL) & ((unsigned)y < (unsigned)H) & ((unsigned)x < (unsigned)W);
        const unsigned voff = ok ? (unsigned)((((size_t)y * W + x) * 64 + pa * 16 + q * 4) * 4) : 0x80000000u;
        float* dst = i < T_INST ? st + i * 256 : sw + (i - T_INST) * 256;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rin, dst, 16, voff, 0, 0, DCNSEP_NT);   // tile (pad pieces load nothing)
      }
    }
  };

  // ---------------------------------------------------------------- phase 1: offset/mask conv
  // the accumulators start at bias x 2^14 (the f16x3 scale): no bias pass between the phases.  Slot s =
  // 16 m + r of lane half h is packed row (r & 3) + 8 (r >> 2) + 4 h of M-tile m (stif_pack_conv_weight,
  // STIF_PACK_DCNSEP: bias [M-tile][32 rows], zero on the padding rows)
  f32x16 om[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const f32x4 bq = ld4(a.b_om[g] + m * 32 + 8 * v + 4 * hf) * (1.0f / F16X3_UNSCALE);
#pragma unroll
      for (int e = 0; e < 4; ++e) om[m][4 * v + e] = bq[e];
    }
#if DCNSEP_EXP == 1   // timing probe: no phase 1 (offsets = biases)
  if (false)
#endif
  {
#if DCNSEP_PRIO == 2
  __builtin_amdgcn_s_setprio(2);   // phase 1 (MFMA stream) ahead of a co-resident phase-2 wave
#endif
  stage_data(0, smem + OFF_D0);
  stage_w(0, 0);
  stage_w(1, 1);
  // chunk loop at run time, taps unrolled: tap offsets, ring slots ((9 c + t) % 3 = t % 3) and the waits
  // are compile-time; the next tap's data fragment is read and split while this tap's MFMAs run, each
  // M-tile's weight fragments one M-tile ahead (scheduling barriers pin that order: the compiler would
  // sink each read next to its MFMAs and wait for it there)
  f16x8 dh, dl;
#pragma unroll 1
  for (int c = 0; c < KSTEPS / 9; ++c) {
    const float* dbuf = smem + ((c & 1) ? OFF_D1 : OFF_D0) + (wv * HC1 + l32) * PX_F + hf * 8;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int k = 9 * c + t;
      // this step's weights (and, at a chunk start, its data) landed in every wave; the DMA issued in the
      // last two steps (weights of k + 1, the side stage of tap 1) may stay in flight
      // weight DMA instructions per wave and step (DCNSEP_WTRIM: wave-uniform, 4 or 3)
      const int WQ = (DCNSEP_WTRIM && NW == 4) ? (wv < MT * 2 - 3 * NW ? 4 : 3) : WK_INS / NW;
#if DCNSEP_TRACE
      const unsigned tr_a = tstamp();
#endif
      if (t == 2 || t == 3) wait_vm(c < 3 ? WQ + D_INS / NW : (PAIR_AHEAD ? WQ + P_INS / NW : WQ));
      else if (t == 8 && c == 3) wait_vm(0);
      else wait_vm(WQ);
#if DCNSEP_TRACE
      const unsigned tr_b = tstamp();
      tr_vm += tr_b - tr_a;
#endif
      // a bare s_barrier: __syncthreads()'s workgroup fence would wait for vmcnt(0), i.e. for the DMA of
      // the next two steps too.  Every LDS read of the step that frees a ring slot has returned (its
      // MFMAs consumed it), and LDS-DMA visibility is the vmcnt wait above.
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#if DCNSEP_P1_SAFE   // diagnostic: every phase-1 step behind a full drain (vmcnt(0) lgkmcnt(0)) and __syncthreads
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
#endif
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
#if DCNSEP_TRACE
      tr_bar += tstamp() - tr_b;
#endif
      // the first weight fragments right after the barrier; this step's data fragment was read and split
      // during the previous step (a chunk's first tap: read now), so the MFMAs start at once, and the
      // next steps' LDS-DMA is issued behind the first M-tile's MFMAs
      const float* wb = smem + OFF_W + (t % RING) * 4096 + lane * 4;
      f16x8 wh[2], wl[2];
      wh[0] = ldh8(wb);
      wl[0] = ldh8(wb + 256);
      if (t == 0) {
        split_f16x3(ld4(dbuf), ld4(dbuf + 4), dh, dl);
      }
      f32x4 x0, x1;
#pragma unroll
      for (int q = 0; q < MT; ++q) {
        if (q + 1 < MT) {
          wh[(q + 1) & 1] = ldh8(wb + (2 * q + 2) * 256);
          wl[(q + 1) & 1] = ldh8(wb + (2 * q + 3) * 256);
        }
        __builtin_amdgcn_sched_barrier(0);
        om[q] = mfma16h(wh[q & 1], dh, om[q]);
        om[q] = mfma16h(wh[q & 1], dl, om[q]);
        om[q] = mfma16h(wl[q & 1], dh, om[q]);
        if (q == 0) {
          if ((t < 7 || c < 3) && DCNSEP_EXP != 7) stage_w(k + 2, (t + 2) % RING);
          if (t == 1) {
            if (c < 3) stage_data(c + 1, smem + (((c + 1) & 1) ? OFF_D1 : OFF_D0));
            else if (PAIR_AHEAD) stage_pair(0, smem + OFF_XT, smem + OFF_XW);   // D0 is free: chunk 2 is done
          }
        }
        if (q == 1 && t < 8) {   // the next tap of the same chunk: its buffer is stable until the chunk ends
          const float* nb = dbuf + (((t + 1) / 3) * HC1 + (t + 1) % 3) * PX_F;
          x0 = ld4(nb);
          x1 = ld4(nb + 4);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if (t < 8) split_f16x3(x0, x1, dh, dl);   // the next step's B operand
    }
  }
  }
#if DCNSEP_EXP == 1
  if (PAIR_AHEAD) stage_pair(0, smem + OFF_XT, smem + OFF_XW);
#endif
#if DCNSEP_TRACE
  tr_p1e = tstamp() - tr_t0;
#endif
  // slot s = 16 m + r of lane half h = component s % 3 (dy, dx, mask) of tap (s % 27) / 3 of group
  // 2 (s / 27) + h, packed row (r & 3) + 8 (r >> 2) + 4 h of M-tile m; bias, unscale, sigmoid(mask)
  // (dcn_v2.py:134-138)
  // unscale, sigmoid(mask) (dcn_v2.py:134-138); the range check is one sum (a non-finite value makes it
  // non-finite) -- a per-value compare would hold 108 lane masks in SGPRs
  float chk = 0.f;
#pragma unroll
  for (int m = 0; m < MT; ++m) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int s = 16 * m + r;
      if (s < 108) {
        float x = om[m][r] * F16X3_UNSCALE;
        chk += x;
        if (s % 3 == 2) x = sigmoid_fast(x);
        om[m][r] = x;
      }
    }
  }
  const bool bad = not_finite(chk);
  report_range(a.status, bad);
#if DCNSEP_TP_DUMP
  if (g_tp_dump) {
    float* d = g_tp_dump + ((size_t)blockIdx.x * (64 * NW) + tid) * TPD_F + 4 * (9 * 8 + 32);
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int r = 0; r < 16; r += 4) st4(d + 16 * m + r, f32x4{om[m][r], om[m][r + 1], om[m][r + 2], om[m][r + 3]});
  }
#endif

  // ---------------------------------------------------------------- phase 2: deformable conv
  // bilinear sample of this lane half's group (channels 16 pa + 8 h .. + 7: a0 = quad 2h, a1 = quad 2h + 1)
  // at tap `tap` with offset (dy, dx) and modulation m folded into the corner weights; `> -1` / `< H`
  // gate; global fallback outside the tile
  auto sample = [&](const float* st, int pa, int tap, float dy, float dx, float mk, f32x4& a0, f32x4& a1) {
    const int ky = tap / 3, kx = tap - 3 * ky;
#if DCNSEP_EXP == 6   // timing probe: sampling positions without the learned offsets (regular LDS addresses)
    const float h_im = (float)(oy - 1 + ky) + 0.25f + 0.f * dy;
    const float w_im = (float)(ox - 1 + kx) + 0.25f + 0.f * dx;
#else
    const float h_im = (float)(oy - 1 + ky) + dy;
    const float w_im = (float)(ox - 1 + kx) + dx;
#endif
    const bool valid = pix_ok & (h_im > -1.f) & (w_im > -1.f) & (h_im < (float)H) & (w_im < (float)W);
    const float fh = floorf(h_im), fw = floorf(w_im);
    const float lh = h_im - fh, lw = w_im - fw, hh = 1.f - lh, hw = 1.f - lw;
    const int h_low = (int)fh, w_low = (int)fw;
    const int r0 = h_low - ty0, c0 = w_low - tx0;
    const bool in_tile = ((unsigned)r0 < (unsigned)(TR - 1)) & ((unsigned)c0 < (unsigned)(TC - 1));
    const float m = valid ? mk : 0.f;
    const float hm = hh * m, lm = lh * m;
    const float w1 = hm * hw, w2 = hm * lw, w3 = lm * hw, w4 = lm * lw;
    const float* p0 = st + (((in_tile ? r0 : 0) * 4 + 2 * hf) * TP + (in_tile ? c0 : 0)) * 4;
    const float* p1 = p0 + 4 * TP * 4;   // next row
    a0 = w1 * ld4(p0) + w2 * ld4(p0 + 4) + w3 * ld4(p1) + w4 * ld4(p1 + 4);
    a1 = w1 * ld4(p0 + TP * 4) + w2 * ld4(p0 + TP * 4 + 4) + w3 * ld4(p1 + TP * 4) + w4 * ld4(p1 + TP * 4 + 4);
    const bool fb = valid & !in_tile;
    if (__builtin_amdgcn_ballot_w64(fb)) {
      if (fb) {
        const int h_high = h_low + 1, w_high = w_low + 1, co = pa * 16 + hf * 8;
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

  // accumulators start at the DCN bias x 2^14 (lane = output channel)
  f32x16 acc0, acc1;
  {
    const float b0 = a.bias[g][l32] * (1.0f / F16X3_UNSCALE), b1 = a.bias[g][32 + l32] * (1.0f / F16X3_UNSCALE);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      acc0[r] = b0;
      acc1[r] = b1;
    }
  }
#if DCNSEP_TP_CHECK
  int tp_bad = 0, tp_badw = 0, tp_first = -1, tp_tap = 0;
#endif
#if DCNSEP_PRIO == 1
  __builtin_amdgcn_s_setprio(2);   // phase 2 (VALU / latency-bound sampling) ahead of a co-resident phase-1 wave
#elif DCNSEP_PRIO == 2
  __builtin_amdgcn_s_setprio(0);
#endif
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // pair 0 staged (NW 8) and the om biases loaded
  __syncthreads();                                    // phase-1 buffers free
#pragma unroll
  for (int pa = 0; pa < 4; ++pa) {
#if DCNSEP_EXP == 3   // timing probe: no phase 2 work
    break;
#endif
    if (PAIR_AHEAD) {
      if (pa + 1 < 4) {
        if ((pa + 1) & 1) stage_pair(pa + 1, smem + OFF_YT, smem + OFF_YW);
        else stage_pair(pa + 1, smem + OFF_XT, smem + OFF_XW);
      }
    } else {
      // one buffer: this pair's stage lands while the other workgroup on the CU computes
#if DCNSEP_EXP == 5   // timing probe: pair 0's stage reused for every pair (no restaging)
      if (pa == 0) {
        stage_pair(pa, smem + OFF_XT, smem + OFF_XW);
        lds_dma_barrier();
      }
#else
#if DCNSEP_TRACE
      const unsigned tr_c = tstamp();
#endif
      if (pa) __syncthreads();   // every wave is done with the previous pair's buffer
      stage_pair(pa, smem + OFF_XT, smem + OFF_XW);
      if (!DCNSEP_P2PROG) lds_dma_barrier();   // else per tap group in the tap loop
#if DCNSEP_TRACE
      tr_p2w += tstamp() - tr_c;
#endif
#endif
    }
    const float* st = smem + ((PAIR_AHEAD && (pa & 1)) ? OFF_YT : OFF_XT);
    const float* sw = smem + ((PAIR_AHEAD && (pa & 1)) ? OFF_YW : OFF_XW);
#if DCNSEP_TAPPIPE
    // diagnostic variant (round-5 review item 4): tap t + 1's eight corner reads issued before tap t's blend
    struct Samp {
      f32x4 v[8];
      float w1, w2, w3, w4;
      int h_low, w_low;
      bool fb;
      bool it;
    };
    auto prep = [&](int tap, float dy, float dx, float mk, Samp& o) {
      const int ky = tap / 3, kx = tap - 3 * ky;
      const float h_im = (float)(oy - 1 + ky) + dy;
      const float w_im = (float)(ox - 1 + kx) + dx;
      const bool valid = pix_ok & (h_im > -1.f) & (w_im > -1.f) & (h_im < (float)H) & (w_im < (float)W);
      const float fh = floorf(h_im), fw = floorf(w_im);
      const float lh = h_im - fh, lw = w_im - fw, hh = 1.f - lh, hw = 1.f - lw;
      o.h_low = (int)fh;
      o.w_low = (int)fw;
      const int r0 = o.h_low - ty0, c0 = o.w_low - tx0;
      const bool in_tile = ((unsigned)r0 < (unsigned)(TR - 1)) & ((unsigned)c0 < (unsigned)(TC - 1));
      const float m = valid ? mk : 0.f;
      const float hm = hh * m, lm = lh * m;
      o.w1 = hm * hw;
      o.w2 = hm * lw;
      o.w3 = lm * hw;
      o.w4 = lm * lw;
      o.fb = DCNSEP_TP_NOFB ? false : (valid & !in_tile);
      o.it = in_tile;
      const float* p0 = st + (((in_tile ? r0 : 0) * 4 + 2 * hf) * TP + (in_tile ? c0 : 0)) * 4;
      const float* p1 = p0 + 4 * TP * 4;
      o.v[0] = ld4(p0);
      o.v[1] = ld4(p0 + 4);
      o.v[2] = ld4(p1);
      o.v[3] = ld4(p1 + 4);
      o.v[4] = ld4(p0 + TP * 4);
      o.v[5] = ld4(p0 + TP * 4 + 4);
      o.v[6] = ld4(p1 + TP * 4);
      o.v[7] = ld4(p1 + TP * 4 + 4);
    };
    auto finish = [&](const Samp& o, f32x4& a0, f32x4& a1) {
#if DCNSEP_TP_CHECK
      // diagnostic guard: every staged corner this lane read from LDS against the input map in HBM
      if (o.it) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int y = o.h_low + ((k >> 1) & 1), x = o.w_low + (k & 1), qd = 2 * hf + (k >> 2);
          const bool inimg = ((unsigned)y < (unsigned)H) & ((unsigned)x < (unsigned)W);
          const f32x4 g = inimg ? ld4(in + ((size_t)y * W + x) * 64 + pa * 16 + qd * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (__builtin_bit_cast(unsigned, g[e]) != __builtin_bit_cast(unsigned, o.v[k][e])) {
              ++tp_bad;
              if (tp_first < 0) tp_first = (pa * 16 + tp_tap) * 8 + k;
            }
        }
      }
#endif
      a0 = o.w1 * o.v[0] + o.w2 * o.v[1] + o.w3 * o.v[2] + o.w4 * o.v[3];
      a1 = o.w1 * o.v[4] + o.w2 * o.v[5] + o.w3 * o.v[6] + o.w4 * o.v[7];
      if (__builtin_amdgcn_ballot_w64(o.fb)) {
        if (o.fb) {
          const int h_low = o.h_low, w_low = o.w_low, h_high = h_low + 1, w_high = w_low + 1, co = pa * 16 + hf * 8;
          const bool b1 = h_low >= 0 && w_low >= 0, b2 = h_low >= 0 && w_high <= W - 1;
          const bool b3 = h_high <= H - 1 && w_low >= 0, b4 = h_high <= H - 1 && w_high <= W - 1;
          const float* q1 = in + ((size_t)h_low * W + w_low) * 64 + co;
          const float* q2 = in + ((size_t)h_low * W + w_high) * 64 + co;
          const float* q3 = in + ((size_t)h_high * W + w_low) * 64 + co;
          const float* q4 = in + ((size_t)h_high * W + w_high) * 64 + co;
          const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
          a0 = o.w1 * (b1 ? ld4(q1) : z) + o.w2 * (b2 ? ld4(q2) : z) + o.w3 * (b3 ? ld4(q3) : z) +
               o.w4 * (b4 ? ld4(q4) : z);
          a1 = o.w1 * (b1 ? ld4(q1 + 4) : z) + o.w2 * (b2 ? ld4(q2 + 4) : z) + o.w3 * (b3 ? ld4(q3 + 4) : z) +
               o.w4 * (b4 ? ld4(q4 + 4) : z);
        }
      }
    };
    Samp cur, nxt;
    {
      const int s = 27 * pa;
      prep(0, om[s / 16][s % 16], om[(s + 1) / 16][(s + 1) % 16], om[(s + 2) / 16][(s + 2) % 16], cur);
    }
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const float* wp = sw + t * 1024 + lane * 4;
      const f16x8 bh0 = ldh8(wp), bl0 = ldh8(wp + 256), bh1 = ldh8(wp + 512), bl1 = ldh8(wp + 768);
      if (t < 8) {
        const int s = 27 * pa + 3 * (t + 1);
        prep(t + 1, om[s / 16][s % 16], om[(s + 1) / 16][(s + 1) % 16], om[(s + 2) / 16][(s + 2) % 16], nxt);
      }
      if (DCNSEP_TP_WAIT) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      f32x4 a0, a1;
#if DCNSEP_TP_CHECK
      tp_tap = t;
      {   // the B fragments of this tap against the packed weights in HBM
        const float* gw = wt + (size_t)pa * WP_F + t * 1024 + lane * 4;
        const f16x8 g0 = ldh8(gw), g1 = ldh8(gw + 256), g2 = ldh8(gw + 512), g3 = ldh8(gw + 768);
        typedef unsigned u32x4c __attribute__((ext_vector_type(4)));
        const u32x4c d = __builtin_bit_cast(u32x4c, g0) ^ __builtin_bit_cast(u32x4c, bh0);
        const u32x4c d1 = __builtin_bit_cast(u32x4c, g1) ^ __builtin_bit_cast(u32x4c, bl0);
        const u32x4c d2 = __builtin_bit_cast(u32x4c, g2) ^ __builtin_bit_cast(u32x4c, bh1);
        const u32x4c d3 = __builtin_bit_cast(u32x4c, g3) ^ __builtin_bit_cast(u32x4c, bl1);
        if ((d[0] | d[1] | d[2] | d[3] | d1[0] | d1[1] | d1[2] | d1[3] | d2[0] | d2[1] | d2[2] | d2[3] | d3[0] | d3[1] |
             d3[2] | d3[3]) != 0u) {
          tp_badw++;
          if (tp_first < 0) tp_first = 100000 + pa * 16 + t;
        }
      }
#endif
#if DCNSEP_TP_DUMP == 2
      if (g_tp_dump && pa == 0 && t == 0) {
        float* d = g_tp_dump + ((size_t)blockIdx.x * (64 * NW) + tid) * TPD_F;
#pragma unroll
        for (int k = 0; k < 8; ++k) st4(d + TPD_F - 32 + 4 * k, cur.v[k]);
        st4(d + 4 * (9 * 8 + 32) + 112, f32x4{cur.w1, cur.w2, cur.w3, cur.w4});
      }
#endif
      finish(cur, a0, a1);
#if DCNSEP_TP_DUMP
      if (g_tp_dump) {
        float* d = g_tp_dump + ((size_t)blockIdx.x * (64 * NW) + tid) * TPD_F + pa * (9 * 8 + 32) + t * 8;
        st4(d, a0);
        st4(d + 4, a1);
        if (DCNSEP_TP_DUMP == 1 || pa || t)
          st4(g_tp_dump + ((size_t)blockIdx.x * (64 * NW) + tid) * TPD_F + 4 * (9 * 8 + 32) + 112 + (pa * 9 + t) * 4,
              f32x4{cur.w1, cur.w2, cur.w3, cur.w4});
        if (DCNSEP_TP_DUMP == 1 && pa == 0 && t == 0)
#pragma unroll
          for (int k = 0; k < 8; ++k) st4(g_tp_dump + ((size_t)blockIdx.x * (64 * NW) + tid) * TPD_F + TPD_F - 32 + 4 * k, cur.v[k]);
      }
#endif
      f16x8 ah, al;
      split_f16x3(a0, a1, ah, al);
      acc0 = mfma16h(ah, bh0, acc0);
      acc1 = mfma16h(ah, bh1, acc1);
      acc0 = mfma16h(ah, bl0, acc0);
      acc1 = mfma16h(ah, bl1, acc1);
      acc0 = mfma16h(al, bh0, acc0);
      acc1 = mfma16h(al, bh1, acc1);
      __builtin_amdgcn_sched_barrier(0);
      if (t < 8) cur = nxt;
    }
#if DCNSEP_TP_DUMP
    if (g_tp_dump) {
      float* d = g_tp_dump + ((size_t)blockIdx.x * (64 * NW) + tid) * TPD_F + pa * (9 * 8 + 32) + 72;
#pragma unroll
      for (int r = 0; r < 16; r += 4) {
        st4(d + r, f32x4{acc0[r], acc0[r + 1], acc0[r + 2], acc0[r + 3]});
        st4(d + 16 + r, f32x4{acc1[r], acc1[r + 1], acc1[r + 2], acc1[r + 3]});
      }
    }
#endif
#else
    // a tap-level software pipeline (tap t + 1's corner reads issued before tap t's blend, one more
    // sample set live) measured 4 % faster in the C0 step but made the outputs depend on the launch's
    // timing at two waves per SIMD; not kept
    // DCNSEP_P2PROG (NW 4): each wave issued its stage pieces as 6 tile pieces, then one weight piece per tap in tap
    // order (stage_pair: instruction wv + 4 j), so "tile + taps <= u landed" is vmcnt(8 - u) per wave, published to the
    // other waves by the barrier after it (the reads follow the barrier)
    static_assert(DCNSEP_P2PROG == 0 || (!PAIR_AHEAD && NW == 4 && T_INST == 24 && P_INS == 60 &&
                                         (DCNSEP_P2PROG == 3 || DCNSEP_P2PROG == 9)), "DCNSEP_P2PROG");
    constexpr int P2G = DCNSEP_P2PROG ? 9 / DCNSEP_P2PROG : 9;   // taps per wait group
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      if (DCNSEP_P2PROG && !PAIR_AHEAD && t % P2G == 0) {
        wait_vm(8 - (t + P2G - 1));
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
      const int s = 27 * pa + 3 * t;   // this lane half's group 2 pa + h, tap t: slots s .. s + 2
      f32x4 a0, a1;
      sample(st, pa, t, om[s / 16][s % 16], om[(s + 1) / 16][(s + 1) % 16], om[(s + 2) / 16][(s + 2) % 16], a0, a1);
      f16x8 ah, al;
      split_f16x3(a0, a1, ah, al);
      const float* wp = sw + t * 1024 + lane * 4;   // [tap][nt][plane][lane][8 halves]
      const f16x8 bh0 = ldh8(wp), bl0 = ldh8(wp + 256), bh1 = ldh8(wp + 512), bl1 = ldh8(wp + 768);
      acc0 = mfma16h(ah, bh0, acc0);
      acc1 = mfma16h(ah, bh1, acc1);
      acc0 = mfma16h(ah, bl0, acc0);
      acc1 = mfma16h(ah, bl1, acc1);
      acc0 = mfma16h(al, bh0, acc0);
      acc1 = mfma16h(al, bh1, acc1);
      __builtin_amdgcn_sched_barrier(0);   // one tap's operands live at a time (VGPR budget)
    }
#endif
    if (PAIR_AHEAD) lds_dma_barrier();
  }
#if DCNSEP_TP_CHECK
  if (__builtin_amdgcn_ballot_w64(tp_bad > 0 || tp_badw > 0)) {
    const unsigned long long m = __builtin_amdgcn_ballot_w64(tp_bad > 0 || tp_badw > 0);
    if (lane == __builtin_ctzll(m))
      printf("TPCHECK block %d wave %d tile (%d,%d) g %d n %d H %d: lanes %d, corner mismatches %d, weight mismatches %d, "
             "first %d\n", (int)blockIdx.x, wv, oy0, ox0, g, n, H, __builtin_popcountll(m), tp_bad, tp_badw, tp_first);
  }
#endif
#if DCNSEP_TRACE
  tr_p2e = tstamp() - tr_t0;
#endif
  if (!PAIR_AHEAD) __syncthreads();   // the epilogue blocks overwrite the pair buffer
  // epilogue through a per-wave LDS block -> coalesced 16-B stores (k_dcn's)
  float* out = a.out[g] + (size_t)n * a.out_item;
  float* blk = smem + OFF_D0 + wv * 1024;
  const int rpx = lane >> 3, c4 = lane & 7;
  float chk2 = 0.f;
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    f32x16 v;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float t = (nt ? acc1[r] : acc0[r]) * F16X3_UNSCALE;
      chk2 += t;
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
  report_range(a.status, not_finite(chk2));
#if DCNSEP_TRACE
  if (g_trace && lane == 0) {
    const unsigned tr_end = tstamp() - tr_t0;
    unsigned* d = g_trace + ((size_t)blockIdx.x * NW + wv) * 8;
    typedef unsigned u32x4t __attribute__((ext_vector_type(4)));
    *reinterpret_cast<u32x4t*>(d) = u32x4t{tr_t0, tr_p1e, tr_p2e, tr_end};
    *reinterpret_cast<u32x4t*>(d + 4) = u32x4t{tr_vm, tr_bar, tr_p2w, blockIdx.x};
  }
#endif
}

}  // namespace

#if DCNSEP_TRACE
extern "C" int stif_dcnsep_trace_set(unsigned* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_trace), &p, sizeof(p)) == hipSuccess ? 0 : -1;
}
#endif

#if DCNSEP_TP_DUMP
extern "C" int stif_dcnsep_dump_set(float* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_tp_dump), &p, sizeof(p)) == hipSuccess ? 0 : -1;
}
#endif

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
