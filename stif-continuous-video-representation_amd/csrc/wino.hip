// 3x3 stride-1 convolution on NHWC fp32 maps by Winograd F(2x2, 3x3) with fp32 MFMA.
//
// Same operator as k_conv for the 3x3 / stride-1 shapes of the STIF encoder (feature
// extraction and recon_trunk ResidualBlock_noBN convs, module_util.py:48-52; PCD / Easy_PCD
// feature convs, Sakuya_arch_test.py:29-67,136-141; the 1x1-free cat convs): Y = A^T [(G g G^T)
// . (B^T d B)] A per 2x2 output tile (Lavin & Gray's F(2x2,3x3)).  The transformed-domain
// products are 16 GEMMs [tiles x cin] x [cin x cout], 16 MACs per 2x2 outputs per (ci, co)
// instead of 36: 2.25x fewer MFMAs than the direct implicit GEMM, all arithmetic fp32.
// The transforms only add/subtract (B, A) and the weight transform G g G^T is done once on the
// host in double (stif_pack_conv_wino); fp32 error stays ~1e-7 relative per layer.
//
// Workgroup = 4 waves, output tile = 4 rows x 32 columns x 64 couts (one slice): 2 x 16
// Winograd tiles = one 32-row MFMA M-tile.  Wave i owns transform row i (xi = 4i + j, j = 0..3),
// which is what makes the kernel cheap:
//   * the input transform row i needs only rows r_A(i), r_B(i) of each 4x4 patch, and the
//     values wave i computes (tile = lane & 31, channels 4h..4h+3 with h = lane >> 5) are
//     exactly its MFMA A operands (permuted-K layout, see conv.hip) -- no LDS round trip;
//   * the B operands U[xi] (packed [slice][chunk][i][j][nt][lane][4]) are per-wave, so they are
//     loaded straight from L2 into registers, one 8-channel chunk ahead;
//   * the output transform's sum over j happens in registers (P_i = M_i A), only the sum over
//     i crosses waves (an LDS exchange per 32-cout half, balanced over all 4 waves).
// Input halo tiles (6 rows x 34 columns x 32 channels per phase) are LDS-DMA'd, double-buffered,
// even and odd columns in separate runs, a pixel's channel chunks consecutive (coalesced loads) at an
// odd pitch (conflict-free transform reads).
#include "abi_util.h"
#include "stif.h"
#include "stif_common.h"
#include "tuning.h"

#include <algorithm>
#include <array>
#include <mutex>
#include <unordered_map>

namespace {

constexpr int WR = 4;      // output rows per tile
constexpr int HR = 6;      // halo rows
constexpr int HC = 34;     // halo columns
constexpr int PSUB = 4;    // 8-channel chunks per staging phase
constexpr int XREAD_J = 3; // F16: block j after whose split the next pair's first chunk is read
// phase image: [halo row][column slot][16-B channel chunk: 2 * PSUB of them + 1 pad], halo rows
// OM_RP chunks apart.  A pixel's chunks are consecutive (8 lanes of an LDS-DMA instruction read one
// pixel's 128 B); the odd pixel pitch (9 slots) keeps 16 consecutive pixels in 16 distinct bank
// groups for the transform's ds_read_b128, and OM_RP = 0 mod 8 keeps the two patch rows a lane
// group spans (lanes of tile rows 0 and 1 share a 16-lane group) conflict-free as well.
constexpr int PITCH = 2 * PSUB + 1;
constexpr int OM_RP = 320;                     // 16-B chunks per staged halo row (35 x PITCH + 5)
constexpr int EX_F = 2 * 2 * 2 * 1024;         // epilogue exchange: [wave 1|2][nt][b][32 tiles][32 co]
constexpr int BUF_F = EX_F;                    // floats per buffer (32 KB)
constexpr int WG_PER_CU = 2;
static_assert(HR * OM_RP * 4 <= BUF_F && OM_RP % 8 == 0 && 35 * PITCH <= OM_RP, "staging image");

// slot of halo column c in its (row, chunk, half) run: even columns first, then odd
STIF_DEV int col_slot(int c) { return (c & 1) ? 17 + (c >> 1) : (c >> 1); }

// LDS-DMA of one staging phase (2 * PSUB 16-B chunks = 32 channels from channel cbase of a
// Cs-channel NHWC map) of the 6 x 34 halo at (iy0, ix0) into `dst`: 30 instructions, (r, m) =
// (halo row, run of 7 column slots); lane -> column slot 7 m + lane / 9, chunk lane % 9 (8 = pad).
// Lane 63 lands on the next run's first chunk with that same pixel's data (or in the row pad), so
// the overlap is benign.  Wave w of nw issues instructions w, w + nw, ...  No divisions per lane.
STIF_DEV void stage_image(__amdgpu_buffer_rsrc_t rs, float* dst, int iy0, int ix0, int H, int W, int Cs, int cbase,
                          int w, int nw, int lpx, int lck) {
  // lane constants: the chunk's byte offset within a pixel, and an x bias that fails the range test
  // for the pad chunk (lck = 8); 24-bit multiplies (pixel index < 2^24, host-checked 2-GB items)
  const unsigned cb = (unsigned)(cbase + lck * 4) * 4u;
  const int xpad = lck < 2 * PSUB ? 0 : (1 << 28);
  const unsigned cs4 = (unsigned)Cs * 4u;
  for (int ins = w; ins < 30; ins += nw) {
    const int r = ins / 5, m = ins - 5 * (ins / 5);   // wave-uniform
    const int y = iy0 + r;
    const int slot = 7 * m + lpx;
    // column of the slot (even columns 0..32 in slots 0..16, odd 1..33 in 17..33; slots >= HC out of
    // range), as shift-and-mask arithmetic so the compiler emits no divergent branch
    const int xo = 2 * slot - (((16 - slot) >> 31) & 33) + (((HC - 1 - slot) >> 31) & (1 << 28)) + xpad;
    const int x = ix0 + xo;
    const unsigned off = __umul24((unsigned)(y * W + x), cs4) + cb;
    // select, not branch: every lane's offset is computed, out-of-range ones replaced
    const unsigned voff = (((unsigned)y < (unsigned)H) & ((unsigned)x < (unsigned)W)) ? off : 0x80000000u;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, dst + (r * OM_RP + 63 * m) * 4, 16, voff, 0, 0, WINO_NT);
  }
}

// IN1 = 2 (the PCD cat(x, s * up2(c)) convs): the second input is the coarse map c [H/2][W/2][C1]; its
// phases stage the 4 x 18 coarse pixels under a tile's 6 x 34 halo (coarse rows oy0/2 - 1 .. +2,
// columns ox0/2 - 1 .. +16) into a scratch area by LDS-DMA, and between phases the workgroup expands
// them into the phase image with F.interpolate(scale_factor=2, bilinear, align_corners=False)
// arithmetic (k_up2's expression) times s -- the upsampled map is never written to HBM.
constexpr int UP_R = 4, UP_C = 18;                    // coarse rows / columns per tile
constexpr int SCR_F = UP_R * UP_C * 2 * PSUB * 4;      // scratch floats: [row][col][chunk][4]
constexpr int SCR_INS = (UP_R * UP_C * 2 * PSUB + 63) / 64;

struct Tile {
  int oy0, ox0, slice, g, n;
  const float* src0;   // the item's input maps (k_wino: in0 and in1 of group g, item n), loaded from the
  const float* src1;   // kernel arguments once per tile, not per staging phase
};

// Persistent: WG_PER_CU workgroups per CU walk the tiles (tile = 4 output rows x 32 columns x one
// 64-cout slice of one item), and the last staging phase of a tile already LDS-DMAs the first
// phase of the next tile and the last chunk prefetches the next tile's first B operands, so a
// workgroup's MFMA stream only pauses at the per-phase barriers and the short epilogue exchange.
// Wave i = transform row i for both 32-cout halves (2 waves per SIMD, ~250 VGPRs).
// dynamic schedule: the value each XCD counter holds before the launch (the host keeps the counters'
// running totals, so nothing resets them at the end of a launch)
#if WINO_TRACE
// diagnostic (stif_wino_trace_set): per wave of the RELU-epilogue f16x3 k_wino (the ResidualBlock conv1) 4 u32 --
// life, phase-end waits (vmcnt + barrier), epilogue (output-transform exchange + stores), tiles -- s_memtime ticks
__device__ unsigned* g_wtrace;
#endif
struct SchedBase {
  unsigned b[8];
};

template <int IN1, int EPI, int F16>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_wino(stif_conv_args a, int ntiles,
                                                                                      SchedBase sb) {
  __shared__ __attribute__((aligned(16))) float smem[2 * BUF_F + (IN1 == 2 ? SCR_F : 0)];
  float* const scr = smem + 2 * BUF_F;                       // IN1 = 2: coarse patch of the next phase
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wi = __builtin_amdgcn_readfirstlane(tid >> 6);   // transform row i of this wave
  const int hf = lane >> 5;
  const int tl = lane & 31;                                  // Winograd tile of this lane
  const int tyl = tl >> 4, txl = tl & 15;

  const int tiles_x = (a.Wo + 31) >> 5;
  const int tiles_y = (a.Ho + WR - 1) / WR;
  const int slices = (a.cout + 63) >> 6;
  const int H = a.H, W = a.W, C0 = a.C0, C1 = a.C1;
  const int NC0 = C0 >> 3;
  const int NC = NC0 + (IN1 ? (C1 >> 3) : 0);
  const int NP = NC / PSUB;   // host guarantees NC % PSUB == 0
  const int NQ = NC >> 1;     // F16: 16-channel chunk pairs

  // tile order: cout slice fastest (the slices of one spatial tile share its input), then x, y, item
  auto tile_of = [&](int T) {
    Tile t;
    t.slice = T % slices;
    int r = T / slices;
    const int x = r % tiles_x;
    r /= tiles_x;
    const int y = r % tiles_y;
    r /= tiles_y;
    t.g = r / a.nitems;
    t.n = r - t.g * a.nitems;
    t.oy0 = y * WR;
    t.ox0 = x * 32;
    t.src0 = a.in0[t.g] + (size_t)t.n * a.in0_item;
    t.src1 = IN1 ? a.in1[t.g] + (size_t)t.n * a.in1_item : t.src0;
    return t;
  };
  // packed U: [slice][chunk][i][j][nt][lane][4]; B fragment (j, local half u) at wsl + (j*2 + u)*256
  // F16 (STIF_PACK_F16X3): [slice][pair][i][j][u][plane h|l][lane][8 halves]; fragment (j, u, plane)
  // of pair q at wsl + q * 16384 + ((j * 2 + u) * 2 + plane) * 256 (float offsets)
  auto wbase = [&](const Tile& t) {
    return F16 ? a.w[t.g] + (size_t)t.slice * NC * 8192 + wi * 4096 + lane * 4
               : a.w[t.g] + (size_t)t.slice * NC * 8192 + wi * 2048 + lane * 4;
  };

  // staging image (stage_image): DMA instruction (r, m) = wave wi's ins = wi, wi + 4, ... of 30
  const int lpx = lane / 9, lck = lane - 9 * (lane / 9);
  const int h1 = H >> 1, w1 = W >> 1;   // IN1 = 2: the coarse map's size
  auto stage = [&](const Tile& t, int p, int buf) {
    // a phase lies entirely in one input (NC0 % PSUB == 0, host-checked)
    const bool second = IN1 && p * PSUB >= NC0;
    const float* src = second ? t.src1 : t.src0;
    const int Cs = second ? C1 : C0;
    const int cbase = (second ? p * PSUB - NC0 : p * PSUB) * 8;
    if (IN1 == 2 && second) {
      // coarse patch [row 4][col 18][chunk 8] (lane-linear, out-of-map pixels zero: never weighted)
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, (int)((size_t)h1 * w1 * Cs * 4), 0x00020000);
      const int cy0 = (t.oy0 >> 1) - 1, cx0 = (t.ox0 >> 1) - 1;
      for (int ins = wi; ins < SCR_INS; ins += 4) {
        const int e = ins * 64 + lane, ch = e & 7, pc = e >> 3;
        const int y = cy0 + pc / UP_C, x = cx0 + pc % UP_C;
        const bool ok = (e < UP_R * UP_C * 8) & ((unsigned)y < (unsigned)h1) & ((unsigned)x < (unsigned)w1);
        const unsigned voff = ok ? (unsigned)(((y * w1 + x) * Cs + cbase + ch * 4) * 4) : 0x80000000u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, scr + ins * 256, 16, voff, 0, 0, 0);
      }
      return;
    }
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, (int)((size_t)H * W * Cs * 4), 0x00020000);
    stage_image(rs, smem + buf * BUF_F, t.oy0 - 1, t.ox0 - 1, H, W, Cs, cbase, wi, 4, lpx, lck);
  };
  // IN1 = 2: the staged coarse patch -> the phase image of the tile's 6 x 34 halo (zero outside the map).
  // The halo rows / columns pair up over the coarse patch (oy0 and ox0 are even): halo rows 2 qr, 2 qr + 1
  // (map rows 2 k + 1, 2 k + 2 with k = cy0 + qr) both interpolate coarse rows k, k + 1, with weights
  // (0.75, 0.25) and (0.25, 0.75) -- the values F.interpolate's source coordinates give away from the
  // borders -- and the same for columns.  So a thread takes a 2 x 2 quad of halo pixels for one 16-B
  // channel chunk: 4 coarse reads and 8 lerps for 4 outputs (the per-pixel form needs 16 reads and 12).
  // Quads that touch a map border (clamped source coordinates, or pixels outside the map) take the
  // per-pixel k_up2 expression.  The scale s (2 or 1 in the model) is folded into the row weights.
  auto expand_px = [&](const Tile& t, int r, int c, int ch) {   // k_up2's expression for one pixel
    const int cy0 = (t.oy0 >> 1) - 1, cx0 = (t.ox0 >> 1) - 1;
    const int Y = t.oy0 - 1 + r, X = t.ox0 - 1 + c;
    f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
    if (((unsigned)Y < (unsigned)H) & ((unsigned)X < (unsigned)W)) {
      const float sy = fmaxf(0.5f * ((float)Y + 0.5f) - 0.5f, 0.f);
      const float sx = fmaxf(0.5f * ((float)X + 0.5f) - 0.5f, 0.f);
      const int y0 = min((int)sy, h1 - 1), x0 = min((int)sx, w1 - 1);
      const int y1 = y0 + (y0 < h1 - 1 ? 1 : 0), x1 = x0 + (x0 < w1 - 1 ? 1 : 0);
      const float ly1 = sy - (float)y0, lx1 = sx - (float)x0;
      const float ly0 = 1.f - ly1, lx0 = 1.f - lx1;
      const float* s0 = scr + ((y0 - cy0) * UP_C) * 32 + ch * 4;
      const float* s1 = scr + ((y1 - cy0) * UP_C) * 32 + ch * 4;
      const f32x4 v00 = ld4(s0 + (x0 - cx0) * 32), v01 = ld4(s0 + (x1 - cx0) * 32);
      const f32x4 v10 = ld4(s1 + (x0 - cx0) * 32), v11 = ld4(s1 + (x1 - cx0) * 32);
      v = (ly0 * (lx0 * v00 + lx1 * v01) + ly1 * (lx0 * v10 + lx1 * v11)) * a.in1_scale;
    }
    return v;
  };
  auto expand = [&](const Tile& t, int buf) {
    float* dst = smem + buf * BUF_F;
    const int cy0 = (t.oy0 >> 1) - 1, cx0 = (t.ox0 >> 1) - 1;
    const float sc = a.in1_scale;
    const float w3 = 0.75f * sc, w1 = 0.25f * sc;
    if (WINO_UPQ == 0) {   // per-pixel form (A/B reference)
      for (int f = tid; f < HR * HC * 8; f += 256) {
        const int ch = f & 7, pc = f >> 3, r = pc / HC, c = pc - HC * (pc / HC);
        st4(dst + (r * OM_RP + col_slot(c) * PITCH + ch) * 4, expand_px(t, r, c, ch));
      }
      return;
    }
    for (int f = tid; f < 3 * 17 * 8; f += 256) {
      const int ch = f & 7, q = f >> 3, qr = q / 17, qc = q - 17 * (q / 17);
      const int k = cy0 + qr, m = cx0 + qc;   // coarse rows k, k + 1 and columns m, m + 1
      float* d0 = dst + ((2 * qr) * OM_RP + col_slot(2 * qc) * PITCH + ch) * 4;
      float* d1 = dst + ((2 * qr) * OM_RP + col_slot(2 * qc + 1) * PITCH + ch) * 4;
      if (((unsigned)k < (unsigned)(h1 - 1)) & ((unsigned)m < (unsigned)(w1 - 1))) {
        const float* s0 = scr + ((qr * UP_C + qc) * 8 + ch) * 4;
        const f32x4 v00 = ld4(s0), v01 = ld4(s0 + 32), v10 = ld4(s0 + UP_C * 32), v11 = ld4(s0 + UP_C * 32 + 32);
        // columns: b = 0 (map column 2 m + 1) weights (0.75, 0.25), b = 1 (2 m + 2) (0.25, 0.75)
        const f32x4 t00 = 0.75f * v00 + 0.25f * v01, t01 = 0.25f * v00 + 0.75f * v01;
        const f32x4 t10 = 0.75f * v10 + 0.25f * v11, t11 = 0.25f * v10 + 0.75f * v11;
        st4(d0, w3 * t00 + w1 * t10);
        st4(d1, w3 * t01 + w1 * t11);
        st4(d0 + OM_RP * 4, w1 * t00 + w3 * t10);
        st4(d1 + OM_RP * 4, w1 * t01 + w3 * t11);
      } else {
        st4(d0, expand_px(t, 2 * qr, 2 * qc, ch));
        st4(d1, expand_px(t, 2 * qr, 2 * qc + 1, ch));
        st4(d0 + OM_RP * 4, expand_px(t, 2 * qr + 1, 2 * qc, ch));
        st4(d1 + OM_RP * 4, expand_px(t, 2 * qr + 1, 2 * qc + 1, ch));
      }
    }
  };
  auto up_phase = [&](int p) { return IN1 == 2 && WINO_EXP != 4 && p * PSUB >= NC0; };

  // rows of the 4x4 patch feeding transform row i: (B^T d)_i = d[rA] + sB * d[rB]
  const int rA = (wi == 0) ? 0 : (wi == 2 ? 2 : 1);
  const int rB = (wi == 3) ? 3 : (wi == 2 ? 1 : 2);
  const float sB = (wi == 1) ? 1.f : -1.f;
  const int s0 = col_slot(0) + txl, s1 = col_slot(1) + txl, s2 = col_slot(2) + txl, s3 = col_slot(3) + txl;

  // input transform row i of 8-channel chunk s of the phase in `buf`, for this lane's tile and
  // channels 4h..4h+3: the wave's MFMA A operands for xi = 4i + j.  Split in the LDS reads (issued
  // one chunk ahead where registers allow, so their latency hides under the current chunk's MFMAs)
  // and the add/subtract part.
  auto xread = [&](const float* buf, int s, f32x4* rd) {
    const float* ra = buf + ((2 * tyl + rA) * OM_RP + 2 * s + hf) * 4;
    const float* rb = buf + ((2 * tyl + rB) * OM_RP + 2 * s + hf) * 4;
    rd[0] = ld4(ra + s0 * PITCH * 4); rd[1] = ld4(rb + s0 * PITCH * 4);
    rd[2] = ld4(ra + s1 * PITCH * 4); rd[3] = ld4(rb + s1 * PITCH * 4);
    rd[4] = ld4(ra + s2 * PITCH * 4); rd[5] = ld4(rb + s2 * PITCH * 4);
    rd[6] = ld4(ra + s3 * PITCH * 4); rd[7] = ld4(rb + s3 * PITCH * 4);
  };
  auto xform = [&](const f32x4* rd, f32x4* v) {
    const f32x4 t0 = rd[0] + sB * rd[1];
    const f32x4 t1 = rd[2] + sB * rd[3];
    const f32x4 t2 = rd[4] + sB * rd[5];
    const f32x4 t3 = rd[6] + sB * rd[7];
    v[0] = t0 - t2;
    v[1] = t1 + t2;
    v[2] = t2 - t1;
    v[3] = t1 - t3;
  };

  // XCD-aware persistent schedule: workgroup b is dispatched to XCD b % 8, and XCD x owns the
  // contiguous tile range [x * per, (x + 1) * per) -- tiles that share input (cout slices, halo rows)
  // run at the same time under the same L2.  Static (a.sched == nullptr): the XCD's workgroups stride
  // through it.  Dynamic (a.sched: this stream's 8 counters): the first two tiles are static, the rest
  // are taken from the XCD's counter (relative to its value before the launch, sb), one workgroup-wide
  // atomic fetched a tile ahead -- a workgroup that started late (another stream's kernel held the CU)
  // takes fewer tiles instead of finishing late.  Outputs do not depend on it.
  const int xcd = blockIdx.x & 7, nl = gridDim.x >> 3;   // host: grid is a multiple of 8
  const int per = (ntiles + 7) >> 3;
  const int tend = min((xcd + 1) * per, ntiles);
  // (the fp32-operand variants -- the range re-run -- keep the static schedule: no registers to spare)
  int* const sched = a.sched;
  const bool dyn = F16 && sched != nullptr;
  __shared__ int tslot[2];                                // fetched tile indices, by tile parity
  int T = xcd * per + (blockIdx.x >> 3);
  int Tn = T + nl;                                        // the next tile (static for the first two)
  const int dbase = xcd * per + 2 * nl;                   // dynamic tile d = dbase + counter value
  int par = 0;
#if WINO_TRACE
  const unsigned tr0 = (unsigned)__builtin_amdgcn_s_memtime();
  unsigned tr_wait = 0, tr_epi = 0, tr_x = 0, ntile = 0;
#endif
  if (T < tend) {
  Tile cur = tile_of(T);
  const float* wsl = wbase(cur);
  f32x4 bw[4][2];
  // F16: B operand ring over the (pair, j) blocks, two blocks deep: slot j & 1 holds block j's
  // (u, plane) fragments and is refilled with block j + 2 right after block j's MFMAs
  f16x8 bh[2][2], bl[2][2];
  if constexpr (F16) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        bh[j][u] = ldh8(wsl + ((j * 2 + u) * 2) * 256);
        bl[j][u] = ldh8(wsl + ((j * 2 + u) * 2 + 1) * 256);
      }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int u = 0; u < 2; ++u) bw[j][u] = ld4(wsl + (j * 2 + u) * 256);
  }
  int gp = 0;                     // phases staged so far: buffer of phase gp = gp & 1
  stage(cur, 0, 0);
  lds_dma_barrier();

  for (;;) {
    const bool has_next = Tn < tend;
    const Tile nxt = tile_of(has_next ? Tn : T);
    const float* wnx = wbase(nxt);
    // dynamic: the tile after next, consumed at the next tile's top (written to tslot after phase 0's
    // barrier, when every wave has read the previous value)
    const bool fetch = dyn && has_next;
    int fetched = 0;
    if (fetch && wi == 0 && lane == 0)
      fetched = (int)((unsigned)__hip_atomic_fetch_add(sched + xcd, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) -
                      sb.b[xcd]);
    auto publish = [&](int p) {
      if (p == 0 && fetch && wi == 0 && lane == 0) tslot[par] = fetched;
    };
    auto advance = [&]() {
      T = Tn;
      cur = nxt;
      wsl = wnx;
      Tn = dyn ? dbase + tslot[par] : Tn + nl;
      par ^= 1;
    };

    f32x16 acc[4][2];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int u = 0; u < 2; ++u) acc[j][u] = f32x16{0};

    if constexpr (F16) {
      for (int p = 0; p < NP; ++p, ++gp) {
        const float* buf = smem + (gp & 1) * BUF_F;
        f32x4 rd[8];
        // the phase's first LDS reads go out before the next phase's LDS-DMA is issued, so the DMA
        // issue (~1K cycles per wave) overlaps their latency instead of preceding it
        xread(buf, 0, rd);
        if (WINO_EXP != 1) {
          if (p + 1 < NP) stage(cur, p + 1, (gp + 1) & 1);
          else if (has_next) stage(nxt, 0, (gp + 1) & 1);
        }
        // probe 7 (the fused ResidualBlock's conv1 cost floor): the RELU conv does a third chunk-pair pass per
        // phase (chunks 0, 1 again) = 1.5x its transform / split / MFMA work, the work of a conv1 over the
        // 1-px halo of the next conv's tile, and stores nothing (as probe 5)
        constexpr int SPN = (WINO_EXP == 7 && EPI == STIF_EPI_RELU) ? PSUB / 2 + 1 : PSUB / 2;
#pragma unroll
        for (int sp = 0; sp < SPN; ++sp) {
          // chunk pair (2 sp, 2 sp + 1): lane half h holds channels 4h..4h+3 of both, i.e. the 8
          // K values of a 32x32x16 f16 MFMA; transform both, split all four j, then fetch the next
          // pair's first chunk so its LDS reads hide under this pair's MFMAs
          f32x4 va[4], vb[4];
          xform(rd, va);
          xread(buf, (2 * sp + 1) % PSUB, rd);
          xform(rd, vb);
          const int q = p * (PSUB / 2) + sp % (PSUB / 2);
          const float* wq = wsl + (size_t)q * 16384;
          const float* wq1 = q + 1 < NQ ? wq + 16384 : wnx;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            f16x8 ah, al;
            split_f16x3(va[j], vb[j], ah, al);
            if (j == XREAD_J && 2 * sp + 2 < 2 * SPN) xread(buf, (2 * sp + 2) % PSUB, rd);
#pragma unroll
            for (int u = 0; u < 2; ++u) {
              acc[j][u] = mfma16h(ah, bh[j & 1][u], acc[j][u]);
              acc[j][u] = mfma16h(ah, bl[j & 1][u], acc[j][u]);
              acc[j][u] = mfma16h(al, bh[j & 1][u], acc[j][u]);
            }
            // refill the slot with block j + 2: (pair q, j + 2) or (pair q + 1, j - 2)
            const float* wn = j < 2 ? wq + (j + 2) * 1024 : wq1 + (j - 2) * 1024;
#pragma unroll
            for (int u = 0; u < 2 && WINO_EXP != 2; ++u) {
              bh[j & 1][u] = ldh8(wn + (u * 2) * 256);
              bl[j & 1][u] = ldh8(wn + (u * 2 + 1) * 256);
            }
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        // every load older than the last two blocks' B refills (8) -- the phase's LDS-DMA among
        // them -- has landed
#if WINO_TRACE
        tr_x = (unsigned)__builtin_amdgcn_s_memtime();
#endif
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        __syncthreads();
#if WINO_TRACE
        tr_wait += (unsigned)__builtin_amdgcn_s_memtime() - tr_x;
#endif
        publish(p);
        if (IN1 == 2 && p + 1 < NP && up_phase(p + 1)) {
          expand(cur, (gp + 1) & 1);
          __syncthreads();
        }
      }
    } else
    for (int p = 0; p < NP; ++p, ++gp) {
      if (p + 1 < NP) stage(cur, p + 1, (gp + 1) & 1);
      else if (has_next) stage(nxt, 0, (gp + 1) & 1);
      const float* buf = smem + (gp & 1) * BUF_F;
      f32x4 rd[8];
      xread(buf, 0, rd);
#pragma unroll
      for (int s = 0; s < PSUB; ++s) {
        f32x4 v[4];
        xform(rd, v);
        if (s + 1 < PSUB) xread(buf, s + 1, rd);
        // B operands of the next chunk (the next tile's first chunk after the last one).  bw[j] is
        // reloaded right after its MFMAs, 3/4 of a chunk before its next use; the scheduling
        // barriers keep the compiler from sinking those loads next to their use, which would
        // expose the L2 latency on every j block.
        const int kn = p * PSUB + s + 1;
        const float* wn = kn < NC ? wsl + (size_t)kn * 8192 : wnx;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
#pragma unroll
          for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[j][u] = mfma32(v[j][e], bw[j][u][e], acc[j][u]);
#pragma unroll
          for (int u = 0; u < 2; ++u) bw[j][u] = ld4(wn + (j * 2 + u) * 256);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      // every load older than the last chunk's B-operand prefetches -- the phase's LDS-DMA among
      // them -- has landed; those 8 stay in flight across the barrier
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      __syncthreads();
      publish(p);
      if (IN1 == 2 && p + 1 < NP && up_phase(p + 1)) {
        expand(cur, (gp + 1) & 1);
        __syncthreads();
      }
    }

    // ---- output transform, balanced over all waves.  Wave i holds P_i[b] = sum_j M[i][j] A[j][b]
    // (registers); Y[0] = P_0 + P_1 + P_2, Y[1] = P_1 - P_2 - P_3.  Two rounds (32-cout halves nt):
    // the waves write their P_i[nt] into the buffer of the phase just finished (free after the
    // barrier; the other one is receiving the next tile) transposed to [i][b][tile][co], then every
    // thread combines and stores (pixel, 4-cout) vectors as coalesced 16-B accesses (8 lanes = one
    // pixel's 128 B).  Row swizzle R ^ (bit2(tile) ^ b) keeps both the b32 writes (lane halves 4
    // tiles apart) and the b128 reads (16-lane groups = b 0/1 of one tile) conflict-free.
#if WINO_TRACE
    const unsigned tr_e0 = (unsigned)__builtin_amdgcn_s_memtime();
    ++ntile;
#endif
    float* ex = smem + ((gp - 1) & 1) * BUF_F;
    if (WINO_EXP == 3) {
      f32x16 sm = f32x16{0};
#pragma unroll
      for (int j = 0; j < 4; ++j) sm += acc[j][0] + acc[j][1];
      float tot = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) tot += sm[r];
      a.out[cur.g][(size_t)cur.n * a.out_item + ((size_t)(cur.oy0 * a.Wo + cur.ox0) * a.cout) + tid] = tot;
      __syncthreads();
      if (!has_next) break;
      advance();
      continue;
    }
    f32x16 yv[2][2];   // [local half][b]
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      yv[u][0] = acc[0][u] + acc[1][u] + acc[2][u];
      yv[u][1] = acc[1][u] - acc[2][u] - acc[3][u];
    }
    // Exchange addresses as a per-lane base plus compile-time offsets (no hoisted address VGPRs):
    //   writer (m = mfma_row(r, lane), bit2(m) = hf): row bit 0 is flipped iff hf ^ b, i.e.
    //   +32 floats for even r, -32 for odd r;  reader (m = 16(k >> 1) + txo): bit2(m) = bit2(txo).
    // this thread's outputs: cout quad c4, column ox of the tile, rows k = 0..3
    const int c4 = tid & 7, oxl = (tid >> 3) & 31;
    const int ox = cur.ox0 + oxl;
    const int bb = oxl & 1, txo = oxl >> 1;
    // LSTM: the quad is (i, f, o, g) of hidden channel cout/4; out / out2 / res are 64-ch maps
    constexpr bool LSTM = EPI == STIF_EPI_LSTM;
    const int ostride = LSTM ? 64 : a.cout;
    const size_t slab = (size_t)a.Ho * a.Wo * ostride;
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.out[cur.g] + (size_t)cur.n * a.out_item), (short)0, (int)(slab * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(EPI == STIF_EPI_RES || LSTM ? a.res[cur.g] + (size_t)cur.n * a.res_item : a.in0[cur.g]), (short)0,
        (int)(slab * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t ro2 = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(LSTM ? a.out2[cur.g] + (size_t)cur.n * a.out2_item : a.out[cur.g]), (short)0, (int)(slab * 4),
        0x00020000);
    auto voff = [&](int nt, int k) -> unsigned {
      const int oy = cur.oy0 + k;
      const int co = cur.slice * 64 + nt * 32 + c4 * 4;
      const bool ok = (oy < a.Ho) & (ox < a.Wo) & (co < a.cout);
      return ok ? (unsigned)(((oy * a.Wo + ox) * ostride + (LSTM ? co >> 2 : co)) * 4) : 0x80000000u;
    };
    f32x4 rv[2][4];
    float cc[2][4];
    if (EPI == STIF_EPI_RES) {
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int k = 0; k < 4; ++k)
          rv[nt][k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, voff(nt, k), 0, 0));
    }
    if (LSTM) {
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int k = 0; k < 4; ++k)
          cc[nt][k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rr, voff(nt, k), 0, 0));
    }
    float chk = 0.f;
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      if (nt) __syncthreads();   // round-0 readers are done with the exchange image
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int fl = (hf ^ b) * 32;
        float* wb = ex + ((wi * 2 + b) * 32 + 4 * hf) * 32 + tl;
#pragma unroll
        for (int r = 0; r < 16; ++r)
          wb[((r & 3) + 8 * (r >> 2)) * 32 + ((r & 1) ? -fl : fl)] = yv[nt][b][r];
      }
      __syncthreads();
      const int cob = cur.slice * 64 + nt * 32 + c4 * 4;
      const f32x4 bv = cob < a.cout ? ld4(a.bias[cur.g] + cob) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float* rbase = ex + (bb * 32 + (txo ^ (((txo >> 2) ^ bb) & 1))) * 32 + c4 * 4 + (k >> 1) * 512;
        const f32x4 p1 = ld4(rbase + 1 * 2048), p2 = ld4(rbase + 2 * 2048);
        const f32x4 pe = ld4(rbase + ((k & 1) ? 3 : 0) * 2048);
        f32x4 y = (k & 1) ? (p1 - p2 - pe) : (pe + p1 + p2);
        y = y * (F16 ? F16X3_UNSCALE : 1.f) + bv;   // exact power of two
        if (F16) chk += (cob < a.cout) ? (y[0] + y[1]) + (y[2] + y[3]) : 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (EPI == STIF_EPI_LRELU) y[e] = lrelu01(y[e]);
          if (EPI == STIF_EPI_RELU) y[e] = fmaxf(y[e], 0.f);
          if (EPI == STIF_EPI_OFFMASK && (cob + e) % 3 == 2) y[e] = sigmoidf_(y[e]);
        }
        if (EPI == STIF_EPI_RES) y += rv[nt][k];
        if (LSTM) {
          // ConvLSTMCell (convlstm.py:51-56): c_next = f * c_cur + i * g, h_next = o * tanh(c_next)
          const float cn = sigmoidf_(y[1]) * cc[nt][k] + sigmoidf_(y[0]) * tanhf(y[3]);
          const float hn = sigmoidf_(y[2]) * tanhf(cn);
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, hn), ro, voff(nt, k), 0, 0);
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, cn), ro2, voff(nt, k), 0, 0);
          continue;
        }
        if ((WINO_EXP != 5 && WINO_EXP != 7) || EPI != STIF_EPI_RELU)   // probes 5, 7: the ResidualBlock's conv1 stores nothing
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, y), ro,
                                                 voff(nt, k), 0, 0);
      }
    }
    if (F16) report_range(a.status, not_finite(chk));   // a non-finite output makes the sum non-finite
    __syncthreads();   // exchange buffer free for the next tile's staging
#if WINO_TRACE
    tr_epi += (unsigned)__builtin_amdgcn_s_memtime() - tr_e0;
#endif
    if (!has_next) break;
    advance();
  }
  }
#if WINO_TRACE
  if (g_wtrace && (tid & 63) == 0 && F16 && EPI == STIF_EPI_RELU) {
    typedef unsigned u32x4t __attribute__((ext_vector_type(4)));
    *reinterpret_cast<u32x4t*>(g_wtrace + ((size_t)blockIdx.x * 4 + wi) * 4) =
        u32x4t{(unsigned)__builtin_amdgcn_s_memtime() - tr0, tr_wait, tr_epi, ntile};
  }
#endif
}

// ---------------------------------------------------------------------------------------------
// k_wino_om: the DCN offset/mask conv (DCN_sep.conv_offset_mask, dcn_v2.py:127-133: 64 -> 216,
// STIF_EPI_OFFMASK) in f16x3 with the transformed input held in registers.  k_wino computes one
// 64-cout slice per tile, so for 216 outputs it stages, transforms and splits the same input four
// times.  Here a workgroup stages a 4 x 32 tile's 64 input channels once, every wave turns its
// transform row into the split A operands of all four 16-channel pairs (Ah/Al: 128 VGPRs), and then
// walks the seven 32-cout N-tiles with only the B operands streaming from L2 (a 4-block register
// ring, buffer loads at a uniform block offset): 48 MFMAs and one output-transform exchange per
// N-tile.  The next tile's first staging phase is DMA'd into buffer 0 while the N-tiles run
// (buffer 1 is the exchange image).  LDS-DMA source offsets relative to the tile's halo origin are
// precomputed per lane, so an interior tile's DMA address is one add.
template <int EPI>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_wino_om(stif_conv_args a,
                                                                                        int ntiles) {
  constexpr int SLICE_F = 8 * 8192;             // packed floats per 64-cout slice (8 chunks of 8 channels)
  constexpr int RING = WINO_OM_RING;            // B blocks in flight
  __shared__ __attribute__((aligned(16))) float smem[2 * BUF_F];
  float* const ex = smem + BUF_F;               // exchange image (buffer 1 once the A operands are built)
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wi = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hf = lane >> 5;
  const int tl = lane & 31;
  const int tyl = tl >> 4, txl = tl & 15;
  const int tiles_x = (a.Wo + 31) >> 5;
  const int tiles_y = (a.Ho + WR - 1) / WR;
  const int H = a.H, W = a.W;                   // C0 = 64, in1_mode 0 (host-checked)
  const int ntn = (a.cout + 31) >> 5;           // 32-cout N-tiles
  const int wbytes = ((a.cout + 63) >> 6) * SLICE_F * 4;

  auto tile_of = [&](int T) {
    Tile t;
    t.slice = 0;
    const int x = T % tiles_x;
    int r = T / tiles_x;
    const int y = r % tiles_y;
    r /= tiles_y;
    t.g = r / a.nitems;
    t.n = r - t.g * a.nitems;
    t.oy0 = y * WR;
    t.ox0 = x * 32;
    return t;
  };

  // staging: k_wino's image (stage_image), 32 channels per phase, all four waves issuing
  const int lpx = lane / 9, lck = lane - 9 * (lane / 9);
  auto stage = [&](const Tile& t, int p, int buf) {
    const float* src = a.in0[t.g] + (size_t)t.n * a.in0_item;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, (int)((size_t)H * W * 256), 0x00020000);
    stage_image(rs, smem + buf * BUF_F, t.oy0 - 1, t.ox0 - 1, H, W, 64, p * 32, wi, 4, lpx, lck);
  };


  // input transform row i (k_wino's xread / xform) -> split A operands of chunk pair q
  const int rA = (wi == 0) ? 0 : (wi == 2 ? 2 : 1);
  const int rB = (wi == 3) ? 3 : (wi == 2 ? 1 : 2);
  const float sB = (wi == 1) ? 1.f : -1.f;
  const int s0 = col_slot(0) + txl, s1 = col_slot(1) + txl, s2 = col_slot(2) + txl, s3 = col_slot(3) + txl;
  auto xread = [&](const float* buf, int s, f32x4* rd) {
    const float* ra = buf + ((2 * tyl + rA) * OM_RP + 2 * s + hf) * 4;
    const float* rb = buf + ((2 * tyl + rB) * OM_RP + 2 * s + hf) * 4;
    rd[0] = ld4(ra + s0 * PITCH * 4); rd[1] = ld4(rb + s0 * PITCH * 4);
    rd[2] = ld4(ra + s1 * PITCH * 4); rd[3] = ld4(rb + s1 * PITCH * 4);
    rd[4] = ld4(ra + s2 * PITCH * 4); rd[5] = ld4(rb + s2 * PITCH * 4);
    rd[6] = ld4(ra + s3 * PITCH * 4); rd[7] = ld4(rb + s3 * PITCH * 4);
  };
  auto xform = [&](const f32x4* rd, f32x4* v) {
    const f32x4 t0 = rd[0] + sB * rd[1];
    const f32x4 t1 = rd[2] + sB * rd[3];
    const f32x4 t2 = rd[4] + sB * rd[5];
    const f32x4 t3 = rd[6] + sB * rd[7];
    v[0] = t0 - t2;
    v[1] = t1 + t2;
    v[2] = t2 - t1;
    v[3] = t1 - t3;
  };
  f16x8 Ah[4][4], Al[4][4];
  auto make_a = [&](const float* buf, int sp, int q) {
    f32x4 rd[8], va[4], vb[4];
    xread(buf, 2 * sp, rd);
    xform(rd, va);
    xread(buf, 2 * sp + 1, rd);
    xform(rd, vb);
#pragma unroll
    for (int j = 0; j < 4; ++j) split_f16x3(va[j], vb[j], Ah[q][j], Al[q][j]);
  };

  // B fragments: [slice][pair q][i][j][u][plane][lane][8 halves] (STIF_PACK_WINO_OFFMASK | F16X3);
  // block b = (q, j) of N-tile n at a uniform offset, this wave's row i and lane in the VGPR offset
  const int bvo = (wi * 4096 + lane * 4) * 4;
  auto boff = [&](int n, int b, int plane) {
    return ((n >> 1) * SLICE_F + (b >> 2) * 16384 + (((b & 3) * 2 + (n & 1)) * 2 + plane) * 256) * 4;
  };
  auto wres = [&](int g) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)a.w[g], (short)0, wbytes, 0x00020000);
  };
  f16x8 bh[RING], bl[RING];
  auto ldb = [&](__amdgpu_buffer_rsrc_t r, int n, int b, int slot) {
    bh[slot] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(r, bvo, boff(n, b, 0), 0));
    bl[slot] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(r, bvo, boff(n, b, 1), 0));
  };

  // output transform of N-tile n (k_wino's exchange, one 32-cout round); `last` also waits for the
  // next tile's first staging phase (buffer 0) before the closing barrier
  const int c4 = tid & 7, oxl = (tid >> 3) & 31;
  const int bb = oxl & 1, txo = oxl >> 1;
  auto bias_of = [&](const Tile& t, int n) {   // loaded before the N-tile's B prefetches (vmcnt order)
    const int cob = n * 32 + c4 * 4;
    return cob < a.cout ? ld4(a.bias[t.g] + cob) : f32x4{0.f, 0.f, 0.f, 0.f};
  };
  auto write_p = [&](const f32x16* acc) {
    f32x16 yv[2];
    yv[0] = acc[0] + acc[1] + acc[2];
    yv[1] = acc[1] - acc[2] - acc[3];
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int fl = (hf ^ b) * 32;
      float* wb = ex + ((wi * 2 + b) * 32 + 4 * hf) * 32 + tl;
#pragma unroll
      for (int r = 0; r < 16; ++r) wb[((r & 3) + 8 * (r >> 2)) * 32 + ((r & 1) ? -fl : fl)] = yv[b][r];
    }
  };
  auto read_store = [&](const Tile& t, int n, f32x4 bv) {
    const int ox = t.ox0 + oxl;
    const int cob = n * 32 + c4 * 4;
    const int m3 = cob % 3;
    const bool cok = cob < a.cout;
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.out[t.g] + (size_t)t.n * a.out_item), (short)0, (int)((size_t)a.Ho * a.Wo * a.cout * 4),
        0x00020000);
    float chk = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float* rbase = ex + (bb * 32 + (txo ^ (((txo >> 2) ^ bb) & 1))) * 32 + c4 * 4 + (k >> 1) * 512;
      const f32x4 p1 = ld4(rbase + 1 * 2048), p2 = ld4(rbase + 2 * 2048);
      const f32x4 pe = ld4(rbase + ((k & 1) ? 3 : 0) * 2048);
      f32x4 y = (k & 1) ? (p1 - p2 - pe) : (pe + p1 + p2);
      y = y * F16X3_UNSCALE + bv;
      chk += (y[0] + y[1]) + (y[2] + y[3]);
      // sigmoid(m) on the mask channels (packed position % 3 == 2), branch-free: v_exp + v_rcp
      // (a few ulp, far inside the parity bar)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (EPI == STIF_EPI_OFFMASK) y[e] = (m3 + e) % 3 == 2 ? sigmoid_fast(y[e]) : y[e];
      const int oy = t.oy0 + k;
      const bool ok = (oy < a.Ho) & (ox < a.Wo) & cok & (WINO_EXP != 6);   // probe 6: k_wino_om stores nothing
      const unsigned vo = ok ? (unsigned)(((oy * a.Wo + ox) * a.cout + cob) * 4) : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, y), ro,
                                             vo, 0, 0);
    }
    report_range(a.status, cok & not_finite(chk));   // a non-finite output makes the sum non-finite
  };

  auto mfma_nt = [&](__amdgpu_buffer_rsrc_t wr, __amdgpu_buffer_rsrc_t wrn, int n, f32x16* acc) {
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = f32x16{0};
#pragma unroll
    for (int b = 0; b < 16; ++b) {
      const int q = b >> 2, j = b & 3, s = b % RING;
      acc[j] = mfma16h(Ah[q][j], bh[s], acc[j]);
      acc[j] = mfma16h(Ah[q][j], bl[s], acc[j]);
      acc[j] = mfma16h(Al[q][j], bh[s], acc[j]);
      // refill the slot with the block RING ahead: this N-tile, the next one, or the next tile's first
      if (b + RING < 16) {
        ldb(wr, n, b + RING, s);
      } else {
        const bool nn = n + 1 < ntn;
        ldb(nn ? wr : wrn, nn ? n + 1 : 0, b + RING - 16, s);
      }
#if WINO_OM_SCHED
      __builtin_amdgcn_sched_barrier(0);
#endif
    }
  };

  // XCD-aware persistent schedule (as k_wino): XCD x owns a contiguous range of spatial tiles
  const int xcd = blockIdx.x & 7, nl = gridDim.x >> 3;
  const int per = (ntiles + 7) >> 3;
  const int tend = min((xcd + 1) * per, ntiles);
  int T = xcd * per + (blockIdx.x >> 3);
  if (T >= tend) return;
  Tile cur = tile_of(T);
  __amdgpu_buffer_rsrc_t wr = wres(cur.g);
#pragma unroll
  for (int s = 0; s < RING; ++s) ldb(wr, 0, s, s);
  stage(cur, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (;;) {
    const int Tn = T + nl;
    const bool has_next = Tn < tend;
    const Tile nxt = tile_of(has_next ? Tn : T);
    const __amdgpu_buffer_rsrc_t wrn = wres(nxt.g);
    stage(cur, 1, 1);
    make_a(smem, 0, 0);
    make_a(smem, 1, 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // phase 1 (and the B ring) landed
    __syncthreads();
    make_a(smem + BUF_F, 0, 2);
    make_a(smem + BUF_F, 1, 3);
    __syncthreads();                                     // both staging buffers consumed
    if (has_next) stage(nxt, 0, 0);
#pragma unroll 1
    for (int n = 0; n < ntn; ++n) {
      const f32x4 bv = bias_of(cur, n);   // before the N-tile's B prefetches (vmcnt order)
      f32x16 acc[4];
      mfma_nt(wr, wrn, n, acc);
      write_p(acc);
      __syncthreads();
      read_store(cur, n, bv);
      if (n + 1 == ntn) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // next tile's phase 0 landed
      __syncthreads();
    }
    if (!has_next) break;
    T = Tn;
    cur = nxt;
    wr = wrn;
  }
}

// Host side of the dynamic schedule: the running totals of every counter block, by address.  Per launch the
// increments of XCD x's counter are exact: every dynamic tile is fetched once (D = count - 2 nl valid
// values), and every workgroup that fetches at all (its second static tile exists: F = count - nl, at most
// nl of them) stops after its one failing fetch -- so sb is the counter's value before the launch.
// Launches sharing a block run one after another (one stream), so the totals are exact in order.
std::mutex g_sched_mu;
std::unordered_map<const int*, std::array<unsigned, 8>> g_sched;

void sched_advance(const int* key, int ntiles, int grid, SchedBase& sb) {
  const int nl = grid >> 3, per = (ntiles + 7) >> 3;
  std::lock_guard<std::mutex> lk(g_sched_mu);
  std::array<unsigned, 8>& tot = g_sched[key];   // a new block starts at zero (the caller zeroed it)
  for (int x = 0; x < 8; ++x) {
    sb.b[x] = tot[x];
    const int count = std::max(0, std::min((x + 1) * per, ntiles) - x * per);
    const int dyn_tiles = std::max(0, count - 2 * nl);
    const int fetchers = std::max(0, std::min(nl, count - nl));
    tot[x] += (unsigned)(dyn_tiles + fetchers);
  }
}

// a launch that failed after sched_advance: restore the totals it started from
void sched_undo(const int* key, const SchedBase& sb) {
  std::lock_guard<std::mutex> lk(g_sched_mu);
  std::array<unsigned, 8>& tot = g_sched[key];
  for (int x = 0; x < 8; ++x) tot[x] = sb.b[x];
}

template <int IN1, int EPI>
int launch(const stif_conv_args& a, hipStream_t st) {
  const long long tiles =
      (long long)((a.Wo + 31) / 32) * ((a.Ho + WR - 1) / WR) * ((a.cout + 63) / 64) * a.ngroups * a.nitems;
  if (tiles > 0x7fffffff) return stif_fail(STIF_E_INVALID, "stif_conv3x3_wino: too many tiles");
  if ((long long)a.H * a.W * std::max(a.C0, std::max(a.C1, a.cout)) * 4 >= 0x7fffffffLL)
    return stif_fail(STIF_E_INVALID, "stif_conv3x3_wino: item larger than 2 GB (buffer addressing)");
  if constexpr (WINO_OM && EPI == STIF_EPI_OFFMASK) if ((a.flags & STIF_CONV_F16X3) && a.C0 == 64 && !a.in1_mode) {
    const long long sp = tiles / ((a.cout + 63) / 64);   // spatial tiles: all couts per workgroup
    const int g2 = 8 * (int)std::min<long long>((sp + 7) / 8, (long long)WG_PER_CU * stif_num_cus() / 8);
    hipLaunchKernelGGL((k_wino_om<EPI>), dim3(g2), dim3(256), 0, st, a, (int)sp);
    return stif_check_launch("stif_conv3x3_wino");
  }
  const int grid = 8 * (int)std::min<long long>((tiles + 7) / 8, (long long)WG_PER_CU * stif_num_cus() / 8);
  SchedBase sb{};
  // the dynamic schedule only on request (flag bit and block), and never inside a graph capture: a replayed
  // launch would find the counters past the bases the host recorded for it
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  const bool dyn = a.sched && (a.flags & STIF_CONV_DYNAMIC) && (a.flags & STIF_CONV_F16X3) &&
                   hipStreamIsCapturing(st, &cap) == hipSuccess && cap == hipStreamCaptureStatusNone;
  stif_conv_args ka = a;
  if (!dyn) ka.sched = nullptr;
  if (dyn) sched_advance(a.sched, (int)tiles, grid, sb);
  if (a.flags & STIF_CONV_F16X3)
    hipLaunchKernelGGL((k_wino<IN1, EPI, 1>), dim3(grid), dim3(256), 0, st, ka, (int)tiles, sb);
  else
    hipLaunchKernelGGL((k_wino<IN1, EPI, 0>), dim3(grid), dim3(256), 0, st, ka, (int)tiles, sb);
  const int rc = stif_check_launch("stif_conv3x3_wino");
  if (rc != STIF_OK && dyn) sched_undo(a.sched, sb);   // the kernel never ran: the counters did not move
  return rc;
}

}  // namespace

#if WINO_TRACE
extern "C" int stif_wino_trace_set(unsigned* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_wtrace), &p, sizeof(p)) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int stif_conv3x3_wino(const stif_conv_args* pa, void* stream) {
  if (!pa) return stif_fail(STIF_E_INVALID, "stif_conv3x3_wino: null args");
  const stif_conv_args& a = *pa;
  hipStream_t st = (hipStream_t)stream;
  if (a.ngroups < 1 || a.ngroups > STIF_MAX_GROUPS || a.nitems < 1)
    return stif_fail(STIF_E_INVALID, "stif_conv3x3_wino: bad ngroups/nitems");
  if (a.ks != 3 || a.stride != 1 || a.Ho != a.H || a.Wo != a.W)
    return stif_fail(STIF_E_INVALID, "stif_conv3x3_wino: 3x3 stride-1 'same' convolution only");
  if (a.C0 % 8 || a.C0 <= 0 || (a.in1_mode && (a.C1 % 8 || a.C1 <= 0)))
    return stif_fail(STIF_E_INVALID, "stif_conv3x3_wino: channel counts must be multiples of 8");
  if (a.in1_mode == 2 && (a.H % 2 || a.W % 2))
    return stif_fail(STIF_E_INVALID, "stif_conv3x3_wino: x2 upsampled second input needs even H, W");
  if (a.epi == STIF_EPI_LSTM && (a.cout != 256 || a.in1_mode != 1 || !a.res[0] || !a.out2[0]))
    return stif_fail(STIF_E_INVALID, "stif_conv3x3_wino: LSTM conv must be 128->256 with res = c_cur, out2 = c_next");
  if (a.cout % 64 && a.epi != STIF_EPI_OFFMASK)
    return stif_fail(STIF_E_INVALID, "stif_conv3x3_wino: cout must be a multiple of 64");
  if (a.epi == STIF_EPI_OFFMASK && (a.cout != 216 || a.in1_mode != 0))
    return stif_fail(STIF_E_INVALID, "stif_conv3x3_wino: offset/mask conv must be 64->216");
  if (a.C0 % (8 * PSUB) || (a.in1_mode && a.C1 % (8 * PSUB)))
    return stif_fail(STIF_E_INVALID, "stif_conv3x3_wino: input channel counts must be multiples of 32");
  if (a.epi == STIF_EPI_RES && !a.res[0]) return stif_fail(STIF_E_INVALID, "stif_conv3x3_wino: RES needs res");
#define STIF_WINO_CASE(IN1)                                              \
  switch (a.epi) {                                                       \
    case STIF_EPI_NONE: return launch<IN1, STIF_EPI_NONE>(a, st);        \
    case STIF_EPI_LRELU: return launch<IN1, STIF_EPI_LRELU>(a, st);      \
    case STIF_EPI_RELU: return launch<IN1, STIF_EPI_RELU>(a, st);        \
    case STIF_EPI_RES: return launch<IN1, STIF_EPI_RES>(a, st);          \
    default: break;                                                      \
  }
  if (a.in1_mode == 0 && a.epi == STIF_EPI_OFFMASK) return launch<0, STIF_EPI_OFFMASK>(a, st);
  if (a.in1_mode == 1 && a.epi == STIF_EPI_LSTM) return launch<1, STIF_EPI_LSTM>(a, st);
  if (a.in1_mode == 0) { STIF_WINO_CASE(0) }
  else if (a.in1_mode == 1) { STIF_WINO_CASE(1) }
  else if (a.in1_mode == 2) {   // the cat(., s * up2(.)) convs: NONE / LRELU
    if (a.epi == STIF_EPI_NONE) return launch<2, STIF_EPI_NONE>(a, st);
    if (a.epi == STIF_EPI_LRELU) return launch<2, STIF_EPI_LRELU>(a, st);
  }
#undef STIF_WINO_CASE
  return stif_fail(STIF_E_INVALID, "stif_conv3x3_wino: unsupported in1 mode / epilogue");
}
