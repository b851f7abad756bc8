// k_wino_sp: the f16x3 Winograd F(2x2, 3x3) conv of k_wino (wino.hip) with the work of a tile split between
// two kinds of waves -- warp specialization.
//
// Same operator, packing (STIF_PACK_WINO | STIF_PACK_F16X3), MFMA K order and summation order as k_wino<IN1,
// EPI, 1>, so its outputs are bit-identical; what changes is who does what.  k_wino gives every wave the whole
// chain of its transform row (LDS-DMA wait -> halo reads -> input transform -> operand split -> MFMAs ->
// output-transform exchange) and runs two 4-wave workgroups per CU; its waves are instruction-latency-bound
// (issue 44 %, MFMA-busy 0.20).  Here one 8-wave workgroup per CU runs
//   * 4 T-waves (waves 0-3, transform row i = wave): staging of the 16-channel halo phases (global loads four
//     pairs ahead in registers, then ds_write into one of two image buffers), the input transform of row i,
//     written to LDS in fp32 in the lane order of the MFMA A fragments (a 32-KB slot per 16-channel pair:
//     [row i][j][chunk][lane][16 B], consecutive lanes, conflict-free), and the output side of the exchange
//     (read back, combined with bias / residual, activation, stores);
//   * 4 M-waves (waves 4-7, row i = wave - 4): the A operands from the slot, split to f16 hi/lo beside the
//     MFMAs, B fragments from L2 in k_wino's register ring, 24 MFMAs per pair, and the input side of the
//     output-transform exchange after a tile's last pair.
// One T-wave and one M-wave share each SIMD, so the transform's VALU stream issues beside the other wave's MFMAs.
// The two roles run one pair apart in lock step: step n = M consumes pair n from slot n & 1 while T transforms
// pair n + 1 into slot (n + 1) & 1 and writes pair n + 2 into staging buffer n & 1; one workgroup barrier per step.
//
// Staging image of a 16-channel phase: [halo row 6][column slot 34][16-B chunk 4], even columns in slots 0-16,
// odd ones in 17-33 (k_wino's col_slot), no padding: chunk c of slot S sits at position c ^ ((S >> 2) & 3), so
// the 16 lanes of a ds_read_b128 group (16 consecutive slots, one chunk) hit 16 distinct bank quads.  A staging
// store writes 64 consecutive positions per wave instruction; the swizzle is applied on the source side (lane p
// loads the chunk that belongs at position p).
//
// LDS: 2 staging buffers (13 KB) + 2 A slots (32 KB) + the exchange (2 x 32 KB) = 154 KB: one workgroup per CU,
// two waves per SIMD (<= 256 VGPRs).
#include "abi_util.h"
#include "stif.h"
#include "stif_common.h"
#include "tuning.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace {

constexpr int WR = 4;                      // output rows per tile
constexpr int HC = 34;                     // halo columns
constexpr int RP = HC * 4;                 // 16-B chunks per staged halo row (136 = 0 mod 8)
constexpr int IMG = 6 * RP;                // chunks of a staged 16-channel phase (816)
constexpr int ST_INS = (IMG + 63) / 64;    // 13 wave stores per staged phase (the last partly zero-fill)
constexpr int STG_F = ST_INS * 256;        // floats per staging buffer (13 KB incl. the tail)
constexpr int A_F = 8192;                  // floats per A slot: [i 4][j 4][plane 2][lane 64][4]
constexpr int EX_F = 8192;                 // floats per exchange round (k_wino's [wave][b][32 tiles][32 co])
constexpr int OFF_STG = 0, OFF_A = 2 * STG_F, OFF_EX = OFF_A + 2 * A_F;
constexpr int LDS_F = OFF_EX + 2 * EX_F;
static_assert(LDS_F * 4 <= 160 * 1024 && RP % 8 == 0, "k_wino_sp LDS map");

STIF_DEV int col_slot(int c) { return (c & 1) ? 17 + (c >> 1) : (c >> 1); }
STIF_DEV int slot_col(int s) { return s < 17 ? 2 * s : 2 * (s - 17) + 1; }

// a tile's coordinates and its item's base pointers, all wave-uniform (SGPRs): the kernel-argument pointer
// arrays are read once per tile by scalar loads -- indexed by a VGPR they became vector loads whose use
// waited for vmcnt(0), i.e. for every B-operand / staging load in flight
struct Tile {
  int oy0, ox0, slice, g, n;
  const float* src0;   // T: the item's in0 / in1 maps
  const float* src1;
  float* out;          // M: the item's output, residual, bias and packed weights of its slice
  const float* res;
  const float* bias;
  const float* w;
};
STIF_DEV int sgpr(int v) { return __builtin_amdgcn_readfirstlane(v); }

// a bare workgroup barrier: __syncthreads()'s fence would wait for vmcnt(0), i.e. also for the B-operand and
// staging loads that stay in flight across it.  LDS writes are complete (lgkmcnt) before it.
STIF_DEV void bar_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

#if WINO_SP_TRACE
// timing probe (tools/r5/sp_trace.py): per workgroup 0-7, wave and step, the s_memtime after the step's
// barrier and before the next one; every lane stores to its own address (vector stores)
__device__ unsigned long long* g_sp_trace;
constexpr int TR_STEPS = 96;
// unconditional buffer stores (out-of-range offset past workgroup 7 / step TR_STEPS: dropped), so the
// compiler's vmcnt bookkeeping sees the same count on every path
#define SP_STAMP(slot)                                                                                  \
  do {                                                                                                  \
    const int sl_ = (slot);                                                                             \
    const bool ok_ = blockIdx.x < 8 && sl_ < 2 * TR_STEPS;                                              \
    const unsigned vo_ = ok_ ? (unsigned)(((blockIdx.x * 8 + wv) * 2 * TR_STEPS + sl_) * 64 + lane) * 8u \
                             : 0x80000000u;                                                             \
    const unsigned long long tm_ = __builtin_amdgcn_s_memtime();                                        \
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, tm_), \
                                          trs, vo_, 0, 0);                                              \
  } while (0)
#else
#define SP_STAMP(slot) \
  do {                 \
  } while (0)
#endif

template <int IN1, int EPI>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) void k_wino_sp(stif_conv_args a,
                                                                                        int ntiles) {
  // 64 input channels (IN1 = 0) or 64 | 64 (IN1 = 1): 4 or 8 16-channel pairs per tile (host-checked), so every
  // step of a tile is straight-line code with its role known at compile time
  constexpr int NPR = IN1 ? 8 : 4;
  constexpr bool RES = EPI == STIF_EPI_RES;
  __shared__ __attribute__((aligned(16))) float smem[LDS_F];
#if WINO_SP_TRACE
  const __amdgpu_buffer_rsrc_t trs =
      __builtin_amdgcn_make_buffer_rsrc((void*)g_sp_trace, (short)0, 8 * 8 * 2 * TR_STEPS * 64 * 8, 0x00020000);
#endif
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wi = wv & 3;                      // transform row i
  const bool is_t = wv < 4;
  const int hf = lane >> 5;
  const int tl = lane & 31;
  const int tyl = tl >> 4, txl = tl & 15;

  const int tiles_x = (a.Wo + 31) >> 5;
  const int tiles_y = (a.Ho + WR - 1) / WR;
  const int slices = (a.cout + 63) >> 6;
  const int H = a.H, W = a.W;
  constexpr int NC = 2 * NPR;                 // 8-channel chunks

  auto tile_of = [&](int T) {
    Tile t;
    T = sgpr(T);
    t.slice = sgpr(T % slices);
    int r = T / slices;
    const int x = r % tiles_x;
    r /= tiles_x;
    const int y = r % tiles_y;
    r /= tiles_y;
    t.g = sgpr(r / a.nitems);
    t.n = sgpr(r - t.g * a.nitems);
    t.oy0 = sgpr(y * WR);
    t.ox0 = sgpr(x * 32);
    t.src0 = a.in0[t.g] + (size_t)t.n * a.in0_item;
    t.src1 = IN1 ? a.in1[t.g] + (size_t)t.n * a.in1_item : t.src0;
    t.out = a.out[t.g] + (size_t)t.n * a.out_item;
    t.res = RES ? a.res[t.g] + (size_t)t.n * a.res_item : t.src0;
    t.bias = a.bias[t.g] + t.slice * 64;
    t.w = a.w[t.g] + (size_t)t.slice * NC * 8192;
    return t;
  };

  // XCD-aware persistent schedule (k_wino's): XCD x owns the contiguous tile range [x per, (x + 1) per)
  const int xcd = blockIdx.x & 7, nl = gridDim.x >> 3;   // host: grid is a multiple of 8
  const int per = (ntiles + 7) >> 3;
  const int tend = min((xcd + 1) * per, ntiles);
  const int T0 = xcd * per + (blockIdx.x >> 3);
  if (T0 >= tend) return;
  const int ntw = (tend - T0 + nl - 1) / nl;   // tiles of this workgroup
  const int N = ntw * NPR;                     // pairs (= steps) of this workgroup
  float* const ex = smem + OFF_EX;

  if (is_t) {
    // =========================================================== T-waves: staging, transform, split, and the
    // output side of the exchange
    if (WINO_SP_TPRIO) __builtin_amdgcn_s_setprio(WINO_SP_TPRIO);
    // image piece k of this wave (instruction wi + 4 k < 13): per-lane (halo row, column, source chunk) once
    int dr[4], dc[4], dq[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int p = (wi + 4 * k) * 64 + lane;
      const int r = p / RP, rem = p - RP * (p / RP), s = rem >> 2;
      dr[k] = p < IMG ? r : 1 << 20;   // fails the row range test: zero fill of the tail (and no load at all
                                       // for the pieces of a fourth instruction that does not exist)
      dc[k] = slot_col(s < HC ? s : 0);
      dq[k] = (rem & 3) ^ ((s >> 2) & 3);
    }
    // staging through registers: lane p of load k fetches the 16 B that belong at image position
    // (wi + 4 k) * 64 + p (out-of-image pixels and the tail read as zeros: the conv padding), four pairs ahead
    // of their ds_write into the staging image -- an LDS-DMA into one of two image buffers had one step, and
    // its ~1 us issue-to-landed time set the step
    auto load_pair = [&](const Tile& t, int q, f32x4 (&dst)[4]) {
      const bool second = IN1 && q >= 4;
      const float* src = second ? t.src1 : t.src0;
      const int cbase = 16 * (second ? q - 4 : q);
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, (int)((size_t)H * W * 256), 0x00020000);
      // four loads on every wave (waves 1-3 have three image pieces: their fourth reads out of range, i.e.
      // nothing), so the per-wave vmcnt bookkeeping is the same on every path
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int y = t.oy0 - 1 + dr[k], x = t.ox0 - 1 + dc[k];
        const unsigned off = __umul24((unsigned)(y * W + x), 256u) + (unsigned)(cbase + 4 * dq[k]) * 4u;
        const unsigned voff = (((unsigned)y < (unsigned)H) & ((unsigned)x < (unsigned)W)) ? off : 0x80000000u;
        dst[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, 0, 0));
      }
    };
    auto write_pair = [&](const f32x4 (&v)[4], int buf) {
      float* dst = smem + OFF_STG + buf * STG_F + lane * 4;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (wi + 4 * k < ST_INS) st4(dst + (wi + 4 * k) * 256, v[k]);
    };
    // transform row i of the phase in buffer `buf` (k_wino's xread / xform): rows rA, rB of each 4x4 patch
    const int rA = (wi == 0) ? 0 : (wi == 2 ? 2 : 1);
    const int rB = (wi == 3) ? 3 : (wi == 2 ? 1 : 2);
    const float sB = (wi == 1) ? 1.f : -1.f;
    int ro[8], rdel[4];   // float offsets of (column m, row A|B) for 8-channel chunk 0; chunk 1 differs by rdel[m]
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int S = col_slot(m) + txl;
      const int x = (S >> 2) & 3;
      ro[2 * m] = ((2 * tyl + rA) * RP + 4 * S + (hf ^ x)) * 4;
      ro[2 * m + 1] = ((2 * tyl + rB) * RP + 4 * S + (hf ^ x)) * 4;
      rdel[m] = ((2 + hf) ^ x) * 4 - (hf ^ x) * 4;
    }
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
    auto transform = [&](int stg, int slot) {
      const float* buf = smem + OFF_STG + stg * STG_F;
      f32x4 rd[2][8], va[4], vb[4];
#pragma unroll
      for (int c = 0; c < 2; ++c)   // all 16 reads in flight at once: one LDS latency per step
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          rd[c][2 * m] = ld4(buf + ro[2 * m] + c * rdel[m]);
          rd[c][2 * m + 1] = ld4(buf + ro[2 * m + 1] + c * rdel[m]);
        }
      xform(rd[0], va);
      xform(rd[1], vb);
      float* dst = smem + OFF_A + slot * A_F + (wi * 8) * 256 + lane * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (WINO_SP_MSPLIT) {
          // the transformed values in fp32 ([i][j][chunk a|b][lane][4]); the M wave splits them
          st4(dst + (2 * j) * 256, va[j]);
          st4(dst + (2 * j + 1) * 256, vb[j]);
        } else {
          // the split A fragments ([i][j][plane h|l][lane][8 halves])
          f16x8 ah, al;
          split_f16x3(va[j], vb[j], ah, al);
          st4(dst + (2 * j) * 256, __builtin_bit_cast(f32x4, ah));
          st4(dst + (2 * j + 1) * 256, __builtin_bit_cast(f32x4, al));
        }
      }
    };

    // ---- the exchange's output side (k_wino's reader): thread tid = (cout quad c4, column oxl), rows k
    const int c4 = tid & 7, oxl = (tid >> 3) & 31;
    const int bb = oxl & 1, txo = oxl >> 1;
    bool live = false;   // a real exchange is pending (the first tile's first steps have none)
    auto voff = [&](const Tile& t, int nt, int k, bool on) -> unsigned {
      const int oy = t.oy0 + k, ox = t.ox0 + oxl;
      const int co = t.slice * 64 + nt * 32 + c4 * 4;
      const bool ok = (oy < a.Ho) & (ox < a.Wo) & on;
      return ok ? (unsigned)(((oy * a.Wo + ox) * a.cout + co) * 4) : 0x80000000u;
    };
    const int slab = (int)((size_t)a.Ho * a.Wo * a.cout * 4);
    f32x4 rv[2][4], bv[2];   // the residual and bias of the tile whose exchange comes next
    auto load_out = [&](const Tile& t) {
      bv[0] = ld4(t.bias + c4 * 4);
      bv[1] = ld4(t.bias + 32 + c4 * 4);
      if (RES) {
        const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc((void*)t.res, (short)0, slab, 0x00020000);
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
          for (int k = 0; k < 4; ++k)
            rv[nt][k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, voff(t, nt, k, true), 0, 0));
      }
    };
    // round nt of tile t's exchange: combine the four rows' P, bias (+ residual), activation, store
    auto ex_read = [&](const Tile& t, int nt) {
      const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void*)t.out, (short)0, slab, 0x00020000);
      float chk = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float* rbase =
            ex + nt * EX_F + (bb * 32 + (txo ^ (((txo >> 2) ^ bb) & 1))) * 32 + c4 * 4 + (k >> 1) * 512;
        const f32x4 p1 = ld4(rbase + 1 * 2048), p2 = ld4(rbase + 2 * 2048);
        const f32x4 pe = ld4(rbase + ((k & 1) ? 3 : 0) * 2048);
        f32x4 y = (k & 1) ? (p1 - p2 - pe) : (pe + p1 + p2);
        y = y * F16X3_UNSCALE + bv[nt];   // exact power of two
        chk += live ? (y[0] + y[1]) + (y[2] + y[3]) : 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (EPI == STIF_EPI_LRELU) y[e] = lrelu01(y[e]);
          if (EPI == STIF_EPI_RELU) y[e] = fmaxf(y[e], 0.f);
        }
        if (RES) y += rv[nt][k];
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, y),
                                               ro, voff(t, nt, k, live), 0, 0);
      }
      report_range(a.status, not_finite(chk));
    };

    // tiles: tc = the tile being transformed / exchanged, tl_ = the tile of the pair being loaded (cached)
    int kl = 0;
    Tile tld = tile_of(T0);
    auto tile_at = [&](int k) -> const Tile& {
      if (k != kl) {
        kl = k;
        tld = tile_of(T0 + k * nl);
      }
      return tld;
    };
    // register ring: pair p's staging data in pf[p % 4] from its load (step p - 6) to its write (step p - 2)
    f32x4 pf[4][4], p0[4], p1[4];
    // unconditional (past the last pair: the last pair again), so the compiler's vmcnt accounting stays exact
    auto load_n = [&](int p, f32x4 (&dst)[4]) {
      p = min(p, N - 1);
      load_pair(tile_at(p / NPR), p % NPR, dst);
    };
    load_n(0, p0);
    load_n(1, p1);
#pragma unroll
    for (int p = 2; p < 6; ++p) load_n(p, pf[p & 3]);
    // step -2: pairs 0 and 1 into the staging buffers
    write_pair(p0, 0);
    if (N > 1) write_pair(p1, 1);
    bar_lds();
    // step -1: transform pair 0
    transform(0, 0);
    bar_lds();
    Tile tc = tile_of(T0), tprev = tc;
    int n = 0;
    // step n = k NPR + q: write pair n + 2 (buffer n & 1: pair n's, transformed in step n - 1) from the ring,
    // load pair n + 6 into the freed slot, transform pair n + 1; q = 0 / 1: rounds 0 / 1 of the previous
    // tile's exchange (written by the M waves in its last step); q = NPR - 2: this tile's bias / residual
    auto tstep = [&](auto q_) {
      constexpr int q = decltype(q_)::value;
      constexpr int s = (q + 2) & 3;
      SP_STAMP(2 * n);
      if (n + 2 < N) write_pair(pf[s], n & 1);
      load_n(n + 6, pf[s]);
      if (q == NPR - 2) load_out(tc);
      if (n + 1 < N && WINO_SP_EXP != 2 && WINO_SP_EXP != 4) transform((n + 1) & 1, (n + 1) & 1);
      if (q < 2) ex_read(tprev, q);
      SP_STAMP(2 * n + 1);
      bar_lds();
      ++n;
    };
    for (int k = 0; k < ntw; ++k) {
      live = k > 0;
      tstep(std::integral_constant<int, 0>{});
      tstep(std::integral_constant<int, 1>{});
      tstep(std::integral_constant<int, 2>{});
      tstep(std::integral_constant<int, 3>{});
      if constexpr (NPR == 8) {
        tstep(std::integral_constant<int, 4>{});
        tstep(std::integral_constant<int, 5>{});
        tstep(std::integral_constant<int, 6>{});
        tstep(std::integral_constant<int, 7>{});
      }
      tprev = tc;
      tc = tile_of(k + 1 < ntw ? T0 + (k + 1) * nl : T0);
    }
    // the last tile's exchange (the M waves wrote it before the last barrier)
    live = true;
    ex_read(tprev, 0);
    ex_read(tprev, 1);
    return;
  }

  // ============================================================= M-waves: MFMAs + the exchange's input side
  auto wbase = [&](const Tile& t) { return t.w + wi * 4096 + lane * 4; };
  Tile cur = tile_of(T0);
  const float* wsl = wbase(cur);
  f16x8 bh[2][2], bl[2][2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      bh[j][u] = ldh8(wsl + ((j * 2 + u) * 2) * 256);
      bl[j][u] = ldh8(wsl + ((j * 2 + u) * 2 + 1) * 256);
    }
  bar_lds();   // step -2
  bar_lds();   // step -1
  // P_i of both 32-cout halves into the exchange (k_wino's layout)
  auto ex_write = [&](f32x16 (&acc)[4][2]) {
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      f32x16 yv[2];
      yv[0] = acc[0][nt] + acc[1][nt] + acc[2][nt];
      yv[1] = acc[1][nt] - acc[2][nt] - acc[3][nt];
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int fl = (hf ^ b) * 32;
        float* wb = ex + nt * EX_F + ((wi * 2 + b) * 32 + 4 * hf) * 32 + tl;
#pragma unroll
        for (int r = 0; r < 16; ++r) wb[((r & 3) + 8 * (r >> 2)) * 32 + ((r & 1) ? -fl : fl)] = yv[b][r];
      }
    }
  };
  f32x16 acc[4][2];
  int n = 0;
  Tile nxt = tile_of(ntw > 1 ? T0 + nl : T0);
  const float* wnx = wbase(nxt);
  // one pair: A fragments from the slot, 24 MFMAs, the B ring refilled with the blocks two ahead
  auto mstep = [&](auto q_) {
    constexpr int q = decltype(q_)::value;
    SP_STAMP(2 * n);
    const float* As = smem + OFF_A + (n & 1) * A_F + (wi * 8) * 256 + lane * 4;
    if (q == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int u = 0; u < 2; ++u) acc[j][u] = f32x16{0};
    }
    const float* wq = wsl + (size_t)q * 16384;
    const float* wq1 = q + 1 < NPR ? wq + 16384 : wnx;
    // WINO_SP_MSPLIT: the split of block j + 1 is issued before block j's MFMAs
    f16x8 sh[2], sl[2];
    if (WINO_SP_MSPLIT) split_f16x3(ld4(As), ld4(As + 256), sh[0], sl[0]);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f16x8 ah, al;
      if (WINO_SP_MSPLIT) {
        ah = sh[j & 1];
        al = sl[j & 1];
        if (j < 3)
          split_f16x3(ld4(As + (2 * j + 2) * 256), ld4(As + (2 * j + 3) * 256), sh[(j + 1) & 1], sl[(j + 1) & 1]);
      } else {
        ah = ldh8(As + (2 * j) * 256);
        al = ldh8(As + (2 * j + 1) * 256);
      }
#pragma unroll
      for (int u = 0; u < 2 && WINO_SP_EXP != 3 && WINO_SP_EXP != 4; ++u) {
        acc[j][u] = mfma16h(ah, bh[j & 1][u], acc[j][u]);
        acc[j][u] = mfma16h(ah, bl[j & 1][u], acc[j][u]);
        acc[j][u] = mfma16h(al, bh[j & 1][u], acc[j][u]);
      }
      if (WINO_SP_EXP == 3 || WINO_SP_EXP == 4) acc[j][0][0] += (float)ah[0] + (float)al[1];   // keep the reads
      // refill the slot with block j + 2: (pair q, j + 2) or (next pair, j - 2)
      const float* wn = j < 2 ? wq + (j + 2) * 1024 : wq1 + (j - 2) * 1024;
#pragma unroll
      for (int u = 0; u < 2 && WINO_SP_EXP != 1 && WINO_SP_EXP != 4; ++u) {
        bh[j & 1][u] = ldh8(wn + (u * 2) * 256);
        bl[j & 1][u] = ldh8(wn + (u * 2 + 1) * 256);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (q == NPR - 1) {
      // the exchange area is free: the T waves read the previous tile's rounds in steps q = 0, 1
      ex_write(acc);
      cur = nxt;
      wsl = wnx;
    }
    SP_STAMP(2 * n + 1);
    bar_lds();
    ++n;
  };
  for (int k = 0; k < ntw; ++k) {
    mstep(std::integral_constant<int, 0>{});
    mstep(std::integral_constant<int, 1>{});
    mstep(std::integral_constant<int, 2>{});
    mstep(std::integral_constant<int, 3>{});
    if constexpr (NPR == 8) {
      mstep(std::integral_constant<int, 4>{});
      mstep(std::integral_constant<int, 5>{});
      mstep(std::integral_constant<int, 6>{});
      mstep(std::integral_constant<int, 7>{});
    }
    nxt = tile_of(k + 2 < ntw ? T0 + (k + 2) * nl : T0);
    wnx = wbase(nxt);
  }
}

template <int IN1, int EPI>
int launch_sp(const stif_conv_args& a, hipStream_t st) {
  const long long tiles =
      (long long)((a.Wo + 31) / 32) * ((a.Ho + WR - 1) / WR) * ((a.cout + 63) / 64) * a.ngroups * a.nitems;
  if (tiles > 0x7fffffff) return stif_fail(STIF_E_INVALID, "stif_conv3x3_wino: too many tiles");
  const int grid = 8 * (int)std::min<long long>((tiles + 7) / 8, (long long)stif_num_cus() / 8);
  hipLaunchKernelGGL((k_wino_sp<IN1, EPI>), dim3(grid), dim3(512), 0, st, a, (int)tiles);
  return stif_check_launch("stif_conv3x3_wino (k_wino_sp)");
}

}  // namespace

// Called by stif_conv3x3_wino (wino.hip) after its argument checks: returns -1 when the call is not one
// k_wino_sp covers (then k_wino runs), else the launch status.
int stif_wino_sp_dispatch(const stif_conv_args& a, hipStream_t st) {
  // STIF_WINO_SP=0|1 in the environment overrides the build default (tuning.h WINO_SP): the A/B and the
  // bit-identity test run both kernels in one process
  const char* e = getenv("STIF_WINO_SP");
  const bool enabled = e && *e ? (atoi(e) != 0) : (WINO_SP != 0);
  if (!enabled || !(a.flags & STIF_CONV_F16X3) || a.cout % 64) return -1;
  if (a.in1_mode > 1 || a.C0 != 64 || (a.in1_mode && a.C1 != 64)) return -1;   // 4 or 8 pairs per tile
  if ((long long)a.H * a.W * std::max(a.C0, std::max(a.C1, a.cout)) * 4 >= 0x7fffffffLL) return -1;
#define STIF_SP_CASE(IN1)                                               \
  switch (a.epi) {                                                      \
    case STIF_EPI_NONE: return launch_sp<IN1, STIF_EPI_NONE>(a, st);    \
    case STIF_EPI_LRELU: return launch_sp<IN1, STIF_EPI_LRELU>(a, st);  \
    case STIF_EPI_RELU: return launch_sp<IN1, STIF_EPI_RELU>(a, st);    \
    case STIF_EPI_RES: return launch_sp<IN1, STIF_EPI_RES>(a, st);      \
    default: return -1;                                                 \
  }
  if (a.in1_mode == 0) { STIF_SP_CASE(0) }
  STIF_SP_CASE(1)
#undef STIF_SP_CASE
}

#if WINO_SP_TRACE
extern "C" int stif_wino_sp_trace(void* dev_buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_sp_trace), &dev_buf, sizeof(dev_buf)) == hipSuccess ? 0 : STIF_E_LAUNCH;
}
#endif
