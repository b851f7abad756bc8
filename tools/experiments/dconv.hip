// KERNEL EXPERIMENT (not built into libstif_hip.so; DESIGN.md section 5, "direct f16x3 implicit GEMM"): correct
// (it passed the Winograd test set through a STIF_PACK_DIRECT packing) but 1.1-1.2x slower than k_wino<F16> on the trunk
// shape -- 49 % MFMA-busy at a ~1.7 GHz clock: the 2.25x MFMA work of the direct form is power-bound.
// 3x3 stride-1 convolution on NHWC fp32 maps as a direct implicit GEMM on split-fp16 MFMA operands.
//
// The operator of every 64-cout 3x3 / stride-1 nn.Conv2d of the STIF encoder (feature extraction and
// recon_trunk ResidualBlock_noBN, module_util.py:48-52; the pyramid / PCD / fusion convs,
// Sakuya_arch_test.py:29-67,136-141, incl. the torch.cat inputs), the alternative to the Winograd
// kernel (wino.hip) for the f16x3 operand mode.  Where k_wino spends its issue slots on the input
// transform, the operand split and a cross-wave output transform, this kernel splits each staged
// input value once (x 2^4 -> fp16 h + l, as the split the Winograd kernel does per transform) into an
// LDS image, and its main loop is nothing but LDS reads, L2 weight loads and MFMAs:
//   out[co][px] = sum_{tap, ci} W[co][ci][tap] * x[px + tap][ci]
// per 16-channel block and tap one v_mfma_f32_32x32x16_f16 K step, 3 products (Wh xh + Wh xl + Wl xh)
// on the weights (A, 32 couts, host-packed, split in double) and the staged inputs (B, 32 pixels).
// 2.25x the MFMAs of Winograd F(2x2,3x3), none of its VALU work; the D layout (lane = pixel, 4
// consecutive couts per register group) feeds the epilogue (bias, activation, residual) and 16-B
// stores straight from the accumulators.
//
// Workgroup = 4 waves, tile = 4 output rows x 32 pixels x one 64-cout slice; wave w = cout tile w & 1
// for output rows 2 (w >> 1), 2 (w >> 1) + 1 (two MFMA pixel tiles: each weight fragment feeds two
// MFMAs).  The input halo (6 x 34 pixels x 64 channels) is loaded into registers during the previous
// stage's K loop, split and written to LDS at a pixel pitch of 272 B (16 consecutive pixels hit 16
// distinct bank groups); a cat input (in1_mode 1) is a second 64-channel stage.  Weights stream from
// L2 through a RING-deep register ring, across stage and tile boundaries.  Persistent, XCD-aware.
#include "abi_util.h"
#include "stif.h"
#include "stif_common.h"

#include <algorithm>

namespace {

constexpr int DR = 4;                   // output rows per tile
constexpr int SR = DR + 2, SC = 34;     // staged halo rows / columns
constexpr int PXB = 272;                // LDS bytes per staged pixel: h plane 128 B, l plane 128 B, pad 16 B
constexpr int ST_N = SR * SC * 16;      // float4 elements (64 channels) per stage
constexpr int ST_PER = (ST_N + 255) / 256;
#ifndef DCONV_RING
#define DCONV_RING 6
#endif
constexpr int RING = DCONV_RING;        // weight K steps in flight
static_assert(36 % RING == 0, "the ring slot of a K step must repeat per stage");

struct DTile {
  int oy0, ox0, slice, g, n;
};

// x (fp32 x 4) -> h, l as 2 + 2 packed halves: x 2^4 = h + l (stif_common.h split_f16x3)
STIF_DEV void split4(f32x4 x, unsigned& h0, unsigned& h1, unsigned& l0, unsigned& l1) {
  asm("v_fma_mixlo_f16 %0, %2, %4, 0\n\t"
      "v_fma_mixhi_f16 %0, %3, %4, 0\n\t"
      "v_fma_mixlo_f16 %1, %2, %4, -%0 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %1, %3, %4, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(h0), "=&v"(l0)
      : "v"(x[0]), "v"(x[1]), "s"(F16X3_SCALE_A));
  asm("v_fma_mixlo_f16 %0, %2, %4, 0\n\t"
      "v_fma_mixhi_f16 %0, %3, %4, 0\n\t"
      "v_fma_mixlo_f16 %1, %2, %4, -%0 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %1, %3, %4, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(h1), "=&v"(l1)
      : "v"(x[2]), "v"(x[3]), "s"(F16X3_SCALE_A));
}

template <int IN1, int EPI>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_dconv(stif_conv_args a,
                                                                                      int ntiles) {
  constexpr int NSG = IN1 ? 2 : 1;      // 64-channel stages (in0, then in1)
  constexpr int KS = NSG * 36;          // K steps per tile: stage x 4 channel blocks x 9 taps
  __shared__ __attribute__((aligned(16))) unsigned char smem[SR * SC * PXB];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ctl = wv & 1, rg = wv >> 1;             // cout tile within the slice, row pair
  const int hf = lane >> 5, l32 = lane & 31;
  const int tiles_x = (a.Wo + 31) >> 5;
  const int tiles_y = (a.Ho + DR - 1) / DR;
  const int slices = a.cout >> 6;
  const int H = a.H, W = a.W;
  const int CT = slices * 2;                        // cout tiles of the packed weight
  const int wbytes = KS * CT * 2048;

  auto tile_of = [&](int T) {
    DTile t;
    t.slice = T % slices;
    int r = T / slices;
    const int x = r % tiles_x;
    r /= tiles_x;
    const int y = r % tiles_y;
    r /= tiles_y;
    t.g = r / a.nitems;
    t.n = r - t.g * a.nitems;
    t.oy0 = y * DR;
    t.ox0 = x * 32;
    return t;
  };

  // ---- input stage: 6 x 34 pixels x 64 channels, element e = pixel * 16 + float4 index
  f32x4 sv[ST_PER];
  auto load_stage = [&](const DTile& t, int sg) {
    const bool second = IN1 && sg == 1;
    const float* src = second ? a.in1[t.g] + (size_t)t.n * a.in1_item : a.in0[t.g] + (size_t)t.n * a.in0_item;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, (int)((size_t)H * W * 256), 0x00020000);
#pragma unroll
    for (int i = 0; i < ST_PER; ++i) {
      const int e = tid + 256 * i;
      const int px = e >> 4, c4 = e & 15;
      const int row = px / SC, col = px - row * SC;
      const int y = t.oy0 - 1 + row, x = t.ox0 - 1 + col;
      const bool ok = (e < ST_N) & ((unsigned)y < (unsigned)H) & ((unsigned)x < (unsigned)W);
      const unsigned vo = ok ? (unsigned)(((y * W + x) * 64 + c4 * 4) * 4) : 0x80000000u;
      sv[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, 0, 0));
    }
  };
  auto write_stage = [&]() {
#pragma unroll
    for (int i = 0; i < ST_PER; ++i) {
      const int e = tid + 256 * i;
      if (ST_N % 256 != 0 && e >= ST_N) break;
      unsigned h0, h1, l0, l1;
      split4(sv[i], h0, h1, l0, l1);
      unsigned char* p = smem + (e >> 4) * PXB + (e & 15) * 8;
      *reinterpret_cast<__attribute__((ext_vector_type(2))) unsigned*>(p) = {h0, h1};
      *reinterpret_cast<__attribute__((ext_vector_type(2))) unsigned*>(p + 128) = {l0, l1};
    }
  };

  // ---- weights: [k step][cout tile][plane][lane][8 halves]; ring slot = k step % RING
  const int wvo = lane * 16;
  auto wres = [&](int g) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)a.w[g], (short)0, wbytes, 0x00020000);
  };
  f16x8 wh[RING], wl[RING];
  auto ldw = [&](__amdgpu_buffer_rsrc_t r, int ks, int ct, int slot) {
    const int o = (ks * CT + ct) * 2048;
    wh[slot] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(r, wvo, o, 0));
    wl[slot] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(r, wvo, o + 1024, 0));
  };

  // ---- B fragments: pixel tile pt (output row 2 rg + pt), tap (ky, kx), channel block cb
  const int rbase = (2 * rg * SC + l32) * PXB + hf * 16;
  auto ldx = [&](int pt, int tap, int cb, f16x8& xh, f16x8& xl) {
    const int ky = tap / 3, kx = tap - 3 * (tap / 3);
    const unsigned char* p = smem + rbase + ((pt + ky) * SC + kx) * PXB + cb * 32;
    xh = *reinterpret_cast<const f16x8*>(p);
    xl = *reinterpret_cast<const f16x8*>(p + 128);
  };

  const int xcd = blockIdx.x & 7, nl = gridDim.x >> 3;   // host: grid is a multiple of 8
  const int per = (ntiles + 7) >> 3;
  const int tend = min((xcd + 1) * per, ntiles);
  int T = xcd * per + (blockIdx.x >> 3);
  if (T >= tend) return;
  DTile cur = tile_of(T);
  __amdgpu_buffer_rsrc_t wr = wres(cur.g);
  int ct = 2 * cur.slice + ctl;
#pragma unroll
  for (int s = 0; s < RING; ++s) ldw(wr, s, ct, s);
  load_stage(cur, 0);

  for (;;) {
    const int Tn = T + nl;
    const bool has_next = Tn < tend;
    const DTile nxt = tile_of(has_next ? Tn : T);
    const __amdgpu_buffer_rsrc_t wrn = wres(nxt.g);
    const int ctn = 2 * nxt.slice + ctl;
    f32x16 acc[2];
    acc[0] = f32x16{0};
    acc[1] = f32x16{0};
#pragma unroll
    for (int sg = 0; sg < NSG; ++sg) {
      __syncthreads();                 // every wave is done reading the previous stage
      write_stage();
      __syncthreads();
      // the next stage's input lands during this stage's K loop
      if (sg + 1 < NSG) load_stage(cur, sg + 1);
      else if (has_next) load_stage(nxt, 0);
      // K loop of the stage: the B fragments of step k + 1 are read before the MFMAs of step k, and
      // every weight refill is pinned behind its step's MFMAs by a scheduling barrier (left alone, the
      // compiler sinks the ring loads next to their use and the L2 latency shows on every step)
      f16x8 xb[2][4];
      ldx(0, 0, 0, xb[0][0], xb[0][1]);
      ldx(1, 0, 0, xb[0][2], xb[0][3]);
#pragma unroll
      for (int kk = 0; kk < 36; ++kk) {
        const int ks = sg * 36 + kk;               // uniform
        const int s = ks % RING;                   // RING divides 36: the slot pattern repeats per tile
        const int c = kk & 1;
        if (kk + 1 < 36) {
          ldx(0, (kk + 1) % 9, (kk + 1) / 9, xb[c ^ 1][0], xb[c ^ 1][1]);
          ldx(1, (kk + 1) % 9, (kk + 1) / 9, xb[c ^ 1][2], xb[c ^ 1][3]);
        }
        acc[0] = mfma16h(wh[s], xb[c][0], acc[0]);
        acc[1] = mfma16h(wh[s], xb[c][2], acc[1]);
        acc[0] = mfma16h(wh[s], xb[c][1], acc[0]);
        acc[1] = mfma16h(wh[s], xb[c][3], acc[1]);
        acc[0] = mfma16h(wl[s], xb[c][0], acc[0]);
        acc[1] = mfma16h(wl[s], xb[c][2], acc[1]);
        // refill: K step ks + RING of this tile, or of the next tile
        const int kn = ks + RING;
        if (kn < KS) ldw(wr, kn, ct, s);
        else ldw(wrn, kn - KS, ctn, s);
        __builtin_amdgcn_sched_barrier(0);
      }
    }

    // ---- epilogue: lane = pixel, register group q = couts 8q + 4hf .. + 3 of the cout tile
    const int ox = cur.ox0 + l32;
    const int cbase = cur.slice * 64 + ctl * 32 + 4 * hf;
    const size_t slab = (size_t)a.Ho * a.Wo * a.cout;
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.out[cur.g] + (size_t)cur.n * a.out_item), (short)0, (int)(slab * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(EPI == STIF_EPI_RES ? a.res[cur.g] + (size_t)cur.n * a.res_item : a.out[cur.g]), (short)0,
        (int)(slab * 4), 0x00020000);
    float chk = 0.f;
#pragma unroll
    for (int pt = 0; pt < 2; ++pt) {
      const int oy = cur.oy0 + 2 * rg + pt;
      const bool ok = (oy < a.Ho) & (ox < a.Wo);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int co = cbase + 8 * q;
        const unsigned vo = ok ? (unsigned)(((oy * a.Wo + ox) * a.cout + co) * 4) : 0x80000000u;
        f32x4 y = f32x4{acc[pt][4 * q], acc[pt][4 * q + 1], acc[pt][4 * q + 2], acc[pt][4 * q + 3]} * F16X3_UNSCALE +
                  ld4(a.bias[cur.g] + co);
        chk += (y[0] + y[1]) + (y[2] + y[3]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (EPI == STIF_EPI_LRELU) y[e] = lrelu01(y[e]);
          if (EPI == STIF_EPI_RELU) y[e] = fmaxf(y[e], 0.f);
        }
        if (EPI == STIF_EPI_RES) y += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, vo, 0, 0));
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, y),
                                               ro, vo, 0, 0);
      }
    }
    report_range(a.status, not_finite(chk));   // a non-finite output makes the sum non-finite
    if (!has_next) break;
    T = Tn;
    cur = nxt;
    wr = wrn;
    ct = ctn;
  }
}

int num_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

template <int IN1, int EPI>
int launch(const stif_conv_args& a, hipStream_t st) {
  const long long tiles = (long long)((a.Wo + 31) / 32) * ((a.Ho + DR - 1) / DR) * (a.cout / 64) * a.ngroups * a.nitems;
  if (tiles > 0x7fffffff) return stif_fail(STIF_E_INVALID, "stif_conv3x3_f16x3: too many tiles");
  const int grid = 8 * (int)std::min<long long>((tiles + 7) / 8, 2LL * num_cus() / 8);
  hipLaunchKernelGGL((k_dconv<IN1, EPI>), dim3(grid), dim3(256), 0, st, a, (int)tiles);
  return stif_check_launch("stif_conv3x3_f16x3");
}

}  // namespace

extern "C" int stif_conv3x3_f16x3(const stif_conv_args* pa, void* stream) {
  if (!pa) return stif_fail(STIF_E_INVALID, "stif_conv3x3_f16x3: null args");
  const stif_conv_args& a = *pa;
  hipStream_t st = (hipStream_t)stream;
  if (a.ngroups < 1 || a.ngroups > STIF_MAX_GROUPS || a.nitems < 1)
    return stif_fail(STIF_E_INVALID, "stif_conv3x3_f16x3: bad ngroups/nitems");
  if (a.ks != 3 || a.stride != 1 || a.Ho != a.H || a.Wo != a.W)
    return stif_fail(STIF_E_INVALID, "stif_conv3x3_f16x3: 3x3 stride-1 'same' convolution only");
  if (a.C0 != 64 || (a.in1_mode == 1 && a.C1 != 64) || (a.in1_mode != 0 && a.in1_mode != 1))
    return stif_fail(STIF_E_INVALID, "stif_conv3x3_f16x3: 64 input channels (+ 64 with in1_mode 1)");
  if (a.cout % 64 || a.cout <= 0) return stif_fail(STIF_E_INVALID, "stif_conv3x3_f16x3: cout must be a multiple of 64");
  if (!(a.flags & STIF_CONV_F16X3)) return stif_fail(STIF_E_INVALID, "stif_conv3x3_f16x3: weights must be STIF_PACK_DIRECT | STIF_PACK_F16X3");
  if ((long long)a.H * a.W * std::max(64, a.cout) * 4 >= 0x7fffffffLL)
    return stif_fail(STIF_E_INVALID, "stif_conv3x3_f16x3: item larger than 2 GB (buffer addressing)");
  if (a.epi == STIF_EPI_RES && !a.res[0]) return stif_fail(STIF_E_INVALID, "stif_conv3x3_f16x3: RES needs res");
#define STIF_DCONV_CASE(IN1)                                             \
  switch (a.epi) {                                                       \
    case STIF_EPI_NONE: return launch<IN1, STIF_EPI_NONE>(a, st);        \
    case STIF_EPI_LRELU: return launch<IN1, STIF_EPI_LRELU>(a, st);      \
    case STIF_EPI_RELU: return launch<IN1, STIF_EPI_RELU>(a, st);        \
    case STIF_EPI_RES: return launch<IN1, STIF_EPI_RES>(a, st);          \
    default: break;                                                      \
  }
  if (a.in1_mode == 0) { STIF_DCONV_CASE(0) }
  else { STIF_DCONV_CASE(1) }
#undef STIF_DCONV_CASE
  return stif_fail(STIF_E_INVALID, "stif_conv3x3_f16x3: unsupported epilogue");
}
