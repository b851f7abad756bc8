// k_wino_sp: the f16x3 Winograd F(2x2, 3x3) conv of k_wino (wino.hip) with the work of a tile split between
// two kinds of waves -- warp specialization.
//
// Same operator, packing (STIF_PACK_WINO | STIF_PACK_F16X3), MFMA K order and summation order as k_wino<IN1,
// EPI, 1>, so its outputs are bit-identical; what changes is who does what.  k_wino gives every wave the whole
// chain of its transform row (LDS-DMA wait -> halo reads -> input transform -> operand split -> MFMAs ->
// output-transform exchange) and runs two 4-wave workgroups per CU; its waves are instruction-latency-bound
// (issue 44 %, MFMA-busy 0.20).  Here one 8-wave workgroup per CU runs
//   * 4 T-waves (waves 0-3, transform row i = wave): LDS-DMA of the 16-channel halo phases, input transform and
//     operand split of row i, written to LDS as the ready MFMA A fragments of that row (a 32-KB slot per
//     16-channel pair: [row i][j][plane][lane][16 B], consecutive lanes, conflict-free);
//   * 4 M-waves (waves 4-7, row i = wave - 4): A fragments from the slot, B fragments from L2 in k_wino's
//     register ring, 24 MFMAs per pair, and the output-transform exchange -- written after a tile's last pair
//     and read back, combined and stored during the next tile's first pair, beside its MFMAs.
// One T-wave and one M-wave share each SIMD, so the transform's VALU stream issues beside the other wave's MFMAs.
// The two roles run one pair apart in lock step: step n = M consumes pair n from slot n & 1 while T transforms
// pair n + 1 into slot (n + 1) & 1 and DMAs pair n + 2 into staging buffer n & 1; one workgroup barrier per step.
//
// Staging image of a 16-channel phase: [halo row 6][column slot 34][16-B chunk 4], even columns in slots 0-16,
// odd ones in 17-33 (k_wino's col_slot), no padding: chunk c of slot S sits at position c ^ ((S >> 2) & 3), so
// the 16 lanes of a ds_read_b128 group (16 consecutive slots, one chunk) hit 16 distinct bank quads.  The LDS-DMA
// writes 64 consecutive positions per instruction; the swizzle is applied on the source side (lane p fetches
// the chunk that belongs at position p).
//
// LDS: 2 staging buffers (13 KB) + 2 A slots (32 KB) + the exchange (2 x 32 KB) = 154 KB: one workgroup per CU,
// two waves per SIMD (<= 256 VGPRs).
#include "abi_util.h"
#include "stif.h"
#include "stif_common.h"
#include "tuning.h"

#include <algorithm>
#include <cstdlib>

namespace {

constexpr int WR = 4;                      // output rows per tile
constexpr int HC = 34;                     // halo columns
constexpr int RP = HC * 4;                 // 16-B chunks per staged halo row (136 = 0 mod 8)
constexpr int IMG = 6 * RP;                // chunks of a staged 16-channel phase (816)
constexpr int DMA_INS = (IMG + 63) / 64;   // 13 LDS-DMA instructions per phase (the last partly zero-fill)
constexpr int STG_F = DMA_INS * 256;       // floats per staging buffer (13 KB incl. the tail)
constexpr int A_F = 8192;                  // floats per A slot: [i 4][j 4][plane 2][lane 64][4]
constexpr int EX_F = 8192;                 // floats per exchange round (k_wino's [wave][b][32 tiles][32 co])
constexpr int OFF_STG = 0, OFF_A = 2 * STG_F, OFF_EX = OFF_A + 2 * A_F;
constexpr int LDS_F = OFF_EX + 2 * EX_F;
static_assert(LDS_F * 4 <= 160 * 1024 && RP % 8 == 0, "k_wino_sp LDS map");

STIF_DEV int col_slot(int c) { return (c & 1) ? 17 + (c >> 1) : (c >> 1); }
STIF_DEV int slot_col(int s) { return s < 17 ? 2 * s : 2 * (s - 17) + 1; }

struct Tile {
  int oy0, ox0, slice, g, n;
};

// a bare workgroup barrier: __syncthreads()'s fence would wait for vmcnt(0), i.e. also for the M-waves'
// B-operand loads that stay in flight across it.  LDS writes are complete (lgkmcnt) before it, LDS-DMA
// (T-waves) by the explicit vmcnt wait.
STIF_DEV void bar_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
STIF_DEV void bar_dma() {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int IN1, int EPI>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) void k_wino_sp(stif_conv_args a,
                                                                                        int ntiles) {
  __shared__ __attribute__((aligned(16))) float smem[LDS_F];
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
  const int H = a.H, W = a.W, C0 = a.C0, C1 = a.C1;
  const int NC = (C0 >> 3) + (IN1 ? (C1 >> 3) : 0);   // 8-channel chunks
  const int NPR = NC >> 1;                             // 16-channel pairs per tile (host: C0, C1 % 16 == 0)

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
    return t;
  };

  // XCD-aware persistent schedule (k_wino's): XCD x owns the contiguous tile range [x per, (x + 1) per)
  const int xcd = blockIdx.x & 7, nl = gridDim.x >> 3;   // host: grid is a multiple of 8
  const int per = (ntiles + 7) >> 3;
  const int tend = min((xcd + 1) * per, ntiles);
  const int T0 = xcd * per + (blockIdx.x >> 3);
  if (T0 >= tend) return;
  const int ntw = (tend - T0 + nl - 1) / nl;   // tiles of this workgroup
  const int N = ntw * NPR;                     // pairs of this workgroup

  if (is_t) {
    // =========================================================== T-waves: staging + transform + split
    // DMA instruction ins = wi + 4 k (k = 0..3, ins < 13): per-lane (halo row, column, source chunk) once
    int dr[4], dc[4], dq[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int p = (wi + 4 * k) * 64 + lane;
      const int r = p / RP, rem = p - RP * (p / RP), s = rem >> 2;
      dr[k] = p < IMG ? r : 1 << 20;   // fails the row range test: zero fill of the tail
      dc[k] = slot_col(s < HC ? s : 0);
      dq[k] = (rem & 3) ^ ((s >> 2) & 3);
    }
    auto stage = [&](const Tile& t, int q, int buf) {
      const bool second = IN1 && 16 * q >= C0;
      const float* src = (second ? a.in1[t.g] + (size_t)t.n * a.in1_item : a.in0[t.g] + (size_t)t.n * a.in0_item);
      const int Cs = second ? C1 : C0;
      const int cbase = second ? 16 * q - C0 : 16 * q;
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, (int)((size_t)H * W * Cs * 4), 0x00020000);
      const unsigned cs4 = (unsigned)Cs * 4u;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int ins = wi + 4 * k;   // wave-uniform
        if (ins < DMA_INS) {
          const int y = t.oy0 - 1 + dr[k], x = t.ox0 - 1 + dc[k];
          const unsigned off = __umul24((unsigned)(y * W + x), cs4) + (unsigned)(cbase + 4 * dq[k]) * 4u;
          const unsigned voff = (((unsigned)y < (unsigned)H) & ((unsigned)x < (unsigned)W)) ? off : 0x80000000u;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, smem + OFF_STG + buf * STG_F + ins * 256, 16, voff, 0, 0, 0);
        }
      }
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
    auto xread = [&](const float* buf, int s, f32x4* rd) {
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        rd[2 * m] = ld4(buf + ro[2 * m] + s * rdel[m]);
        rd[2 * m + 1] = ld4(buf + ro[2 * m + 1] + s * rdel[m]);
      }
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
    auto transform = [&](int stg, int slot) {
      const float* buf = smem + OFF_STG + stg * STG_F;
      f32x4 rd[8], va[4], vb[4];
      xread(buf, 0, rd);
      xform(rd, va);
      xread(buf, 1, rd);
      xform(rd, vb);
      float* dst = smem + OFF_A + slot * A_F + (wi * 8) * 256 + lane * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f16x8 ah, al;
        split_f16x3(va[j], vb[j], ah, al);
        st4(dst + (2 * j) * 256, __builtin_bit_cast(f32x4, ah));
        st4(dst + (2 * j + 1) * 256, __builtin_bit_cast(f32x4, al));
      }
    };
    // the tile of the pair being staged (pair n lies in tile n / NPR of this workgroup's list), cached
    int ks = 0;
    Tile ts = tile_of(T0);
    auto tile_at = [&](int k) -> const Tile& {
      if (k != ks) {
        ks = k;
        ts = tile_of(T0 + k * nl);
      }
      return ts;
    };
    // step -2: pairs 0 and 1 to the staging buffers
    stage(ts, 0, 0);
    if (N > 1) stage(tile_at(1 / NPR), 1 % NPR, 1);
    bar_dma();
    // step -1: transform pair 0
    transform(0, 0);
    bar_dma();
    // step n: stage pair n + 2 (buffer n & 1: pair n's, transformed in step n - 1), transform pair n + 1
    for (int n = 0; n < N; ++n) {
      if (n + 2 < N) stage(tile_at((n + 2) / NPR), (n + 2) % NPR, n & 1);
      if (n + 1 < N) transform((n + 1) & 1, (n + 1) & 1);
      bar_dma();
    }
    return;
  }

  // ============================================================= M-waves: MFMAs + output transform
  const int mt = tid - 256;                    // 0..255 over the 4 M-waves (exchange reader)
  auto wbase = [&](const Tile& t) {
    return a.w[t.g] + (size_t)t.slice * NC * 8192 + wi * 4096 + lane * 4;
  };
  int T = T0;
  Tile cur = tile_of(T);
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

  // ---- exchange (k_wino's): write P_i of both 32-cout halves, read back (pixel, 4-cout) vectors
  float* const ex = smem + OFF_EX;
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
  constexpr bool RES = EPI == STIF_EPI_RES;
  const int c4 = mt & 7, oxl = (mt >> 3) & 31;
  const int bb = oxl & 1, txo = oxl >> 1;
  auto voff = [&](const Tile& t, int nt, int k) -> unsigned {
    const int oy = t.oy0 + k, ox = t.ox0 + oxl;
    const int co = t.slice * 64 + nt * 32 + c4 * 4;
    const bool ok = (oy < a.Ho) & (ox < a.Wo) & (co < a.cout);
    return ok ? (unsigned)(((oy * a.Wo + ox) * a.cout + co) * 4) : 0x80000000u;
  };
  auto out_rsrc = [&](const Tile& t) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)(a.out[t.g] + (size_t)t.n * a.out_item), (short)0,
                                             (int)((size_t)a.Ho * a.Wo * a.cout * 4), 0x00020000);
  };
  auto res_rsrc = [&](const Tile& t) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)(RES ? a.res[t.g] + (size_t)t.n * a.res_item : a.in0[t.g]),
                                             (short)0, (int)((size_t)a.Ho * a.Wo * a.cout * 4), 0x00020000);
  };
  // read round nt of the exchange of tile t, add bias (+ residual), activation, store; returns the range sum
  auto ex_read = [&](const Tile& t, int nt, const f32x4* rv) -> float {
    const __amdgpu_buffer_rsrc_t ro = out_rsrc(t);
    const int cob = t.slice * 64 + nt * 32 + c4 * 4;
    const f32x4 bv = cob < a.cout ? ld4(a.bias[t.g] + cob) : f32x4{0.f, 0.f, 0.f, 0.f};
    float chk = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float* rbase =
          ex + nt * EX_F + (bb * 32 + (txo ^ (((txo >> 2) ^ bb) & 1))) * 32 + c4 * 4 + (k >> 1) * 512;
      const f32x4 p1 = ld4(rbase + 1 * 2048), p2 = ld4(rbase + 2 * 2048);
      const f32x4 pe = ld4(rbase + ((k & 1) ? 3 : 0) * 2048);
      f32x4 y = (k & 1) ? (p1 - p2 - pe) : (pe + p1 + p2);
      y = y * F16X3_UNSCALE + bv;   // exact power of two
      chk += (cob < a.cout) ? (y[0] + y[1]) + (y[2] + y[3]) : 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (EPI == STIF_EPI_LRELU) y[e] = lrelu01(y[e]);
        if (EPI == STIF_EPI_RELU) y[e] = fmaxf(y[e], 0.f);
      }
      if (RES) y += rv[k];
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, y), ro,
                                             voff(t, nt, k), 0, 0);
    }
    return chk;
  };
  auto load_res = [&](const Tile& t, int nt, f32x4* rv) {
    if (RES) {
      const __amdgpu_buffer_rsrc_t rr = res_rsrc(t);
#pragma unroll
      for (int k = 0; k < 4; ++k)
        rv[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, voff(t, nt, k), 0, 0));
    }
  };

  f32x16 acc[4][2];
  Tile prv = cur;          // the tile whose exchange is pending (valid when pend)
  bool pend = false;
  int k_in = 0;            // tile index of pair n within this workgroup's list
  Tile nxt = tile_of(ntw > 1 ? T + nl : T);
  const float* wnx = wbase(nxt);
  for (int n = 0; n < N; ++n) {
    const int q = n - k_in * NPR;
    const float* As = smem + OFF_A + (n & 1) * A_F + (wi * 8) * 256 + lane * 4;
    f32x4 rv[2][4];
    if (q == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int u = 0; u < 2; ++u) acc[j][u] = f32x16{0};
      if (pend) {
        load_res(prv, 0, rv[0]);
        load_res(prv, 1, rv[1]);
      }
    }
    const float* wq = wsl + (size_t)q * 16384;
    const float* wq1 = q + 1 < NPR ? wq + 16384 : wnx;
    float chk = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f16x8 ah = ldh8(As + (2 * j) * 256), al = ldh8(As + (2 * j + 1) * 256);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        acc[j][u] = mfma16h(ah, bh[j & 1][u], acc[j][u]);
        acc[j][u] = mfma16h(ah, bl[j & 1][u], acc[j][u]);
        acc[j][u] = mfma16h(al, bh[j & 1][u], acc[j][u]);
      }
      // refill the slot with block j + 2: (pair q, j + 2) or (next pair, j - 2)
      const float* wn = j < 2 ? wq + (j + 2) * 1024 : wq1 + (j - 2) * 1024;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        bh[j & 1][u] = ldh8(wn + (u * 2) * 256);
        bl[j & 1][u] = ldh8(wn + (u * 2 + 1) * 256);
      }
      __builtin_amdgcn_sched_barrier(0);
      // the previous tile's exchange, beside this tile's first MFMAs (its two rounds after blocks 1 and 2)
      if (q == 0 && pend && (j == 1 || j == 2)) {
        chk += ex_read(prv, j - 1, rv[j - 1]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (q == 0 && pend) {
      report_range(a.status, not_finite(chk));
      pend = false;
    }
    if (q == NPR - 1) {
      // the exchange area is free: the previous tile's rounds were read during this tile's pair 0, at
      // least one barrier ago (NPR >= 2)
      ex_write(acc);
      pend = true;
      prv = cur;
      ++k_in;
      T += nl;
      cur = nxt;
      wsl = wnx;
      nxt = tile_of(k_in + 1 < ntw ? T + nl : T);
      wnx = wbase(nxt);
    }
    bar_lds();
  }
  // the last tile's exchange (published by the last step's barrier)
  {
    f32x4 rv[2][4];
    load_res(prv, 0, rv[0]);
    load_res(prv, 1, rv[1]);
    float chk = ex_read(prv, 0, rv[0]);
    chk += ex_read(prv, 1, rv[1]);
    report_range(a.status, not_finite(chk));
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
  if (a.in1_mode > 1 || a.C0 % 16 || (a.in1_mode && a.C1 % 16)) return -1;
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
