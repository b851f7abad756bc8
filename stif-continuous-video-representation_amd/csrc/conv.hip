// Implicit-GEMM convolution on NHWC fp32 maps with fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// Replaces every nn.Conv2d of the STIF encoder (Sakuya_arch_test.py:282-293, PCD_Align
// :29-67, Easy_PCD :136-141, ConvLSTMCell convlstm.py:36-40, BiDeformableConvLSTM :254)
// and fuses what the reference runs as separate ATen ops around them:
//   * torch.cat of the two inputs       -> read from two pointers (in0 | in1)
//   * F.interpolate(x2, bilinear) (*2)  -> computed while staging in1 into LDS
//   * bias + LeakyReLU / ReLU / residual add / sigmoid(mask) / ConvLSTM gates -> epilogue
//
// GEMM view: M = output pixels, N = output channels, K = cin * ks * ks.
// Workgroup = 4 waves; tile = (4*MT) output rows x 32 columns x (32*NT) couts.
// Wave w owns MT rows (one 32-pixel MFMA M-tile each) x NT N-tiles.
// K is walked in chunks of 8 input channels: the chunk's halo tile and weight
// slice are staged in LDS, then every tap issues 4 MFMAs per (M,N) tile: lane
// half h supplies channels 4h..4h+3 of the chunk through one ds_read_b128 for A
// (input) and one for B (weights) -- the K order inside a chunk is a permutation
// shared by both operands, so no shuffles are needed.
#include "stif_common.h"
#include "stif.h"
#include "abi_util.h"

#include <algorithm>

namespace {

// F16 (the 3x3 64 -> 64 convs with weights packed STIF_PACK_PLAIN | STIF_PACK_F16X3, as the DCN
// core): split-fp16 MFMA with two taps per 32x32x16 MFMA, lane half h supplying tap 2p + h for the
// chunk's 8 channels (tap 9 = zero weights).
template <int KS, int S, int MT, int NT, int NW, int IN1, int EPI, int F16 = 0>
__global__ __launch_bounds__(NW * 64) void k_conv(stif_conv_args a) {
  constexpr int TH = NW * MT;              // output rows per workgroup
  constexpr int HR = (TH - 1) * S + KS;    // halo rows
  constexpr int HC = 31 * S + KS;          // halo cols
  constexpr int T2 = KS * KS;
  constexpr int NJ = NT * 32;              // couts per workgroup
  constexpr int PAD = KS / 2;
  constexpr int NTH = NW * 64;
  // input halo image [row][h][col][4 floats] (h = channel half of the 8-channel chunk): lane-linear,
  // so the LDS-DMA fills it directly and a wave's A-operand read is 32 consecutive 16-B slots
  constexpr int IN_EL = HR * 2 * HC;
  constexpr int IN_INST = (IN_EL + 63) / 64;
  constexpr int IN_F = IN_INST * 256;
  constexpr int W_EL = F16 ? 5 * NT * 2 * 64 : T2 * NT * 64;   // weight fragments per chunk: [tap][nt][lane][4]
  static_assert(!F16 || (KS == 3 && IN1 == 0 && EPI != STIF_EPI_LSTM), "F16: 3x3 single-input convs");
  constexpr int W_F = W_EL * 4;
  constexpr int BUF_F = IN_F + W_F;
  constexpr int SM_F = (2 * BUF_F > NW * 1024) ? 2 * BUF_F : NW * 1024;
  constexpr int EPT = (IN_EL + NTH - 1) / NTH;   // register-staged (upsampled) elements per thread
  __shared__ __attribute__((aligned(16))) float smem[SM_F];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = tid >> 6;
  const int l32 = lane & 31;
  const int hf = lane >> 5;
  const int tiles_x = (a.Wo + 31) >> 5;
  // XCD-aware tile order: workgroups b = x mod 8 run on XCD x, so XCD x takes a contiguous range of
  // spatial tiles and vertically adjacent tiles (sharing halo rows and the 128-B pixel lines that
  // successive 8-channel chunks re-touch) run under one L2 (stride-2 convs: 228 -> 196 us per C1
  // dispatch; round-robin tiles put vertical neighbours on different XCDs)
  const int nbx = gridDim.x;
  const int bx = (nbx & 7) ? (int)blockIdx.x : (int)(blockIdx.x & 7) * (nbx >> 3) + (int)(blockIdx.x >> 3);
  const int tx = bx % tiles_x;
  const int ty = bx / tiles_x;
  const int slice = blockIdx.y;
  const int g = blockIdx.z / a.nitems;
  const int n = blockIdx.z - g * a.nitems;

  const int H = a.H, W = a.W, C0 = a.C0, C1 = a.C1;
  const float* in0 = a.in0[g] + (size_t)n * a.in0_item;
  const float* in1 = IN1 ? a.in1[g] + (size_t)n * a.in1_item : nullptr;
  const int H1 = (IN1 == 2) ? (H >> 1) : H, W1 = (IN1 == 2) ? (W >> 1) : W;
  const __amdgpu_buffer_rsrc_t r0 =
      __builtin_amdgcn_make_buffer_rsrc((void*)in0, (short)0, (int)((size_t)H * W * C0 * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t r1 = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(IN1 == 1 ? in1 : in0), (short)0, (int)((size_t)H * W * (IN1 == 1 ? C1 : C0) * 4), 0x00020000);
  const int oy0 = ty * TH, ox0 = tx * 32;
  const int iy0 = oy0 * S - PAD, ix0 = ox0 * S - PAD;
  const int NC0 = C0 >> 3;
  const int NC = NC0 + (IN1 ? (C1 >> 3) : 0);
  const float* wsl = a.w[g] + (size_t)slice * NC * W_F;   // packed [slice][chunk][tap][nt][lane][4]

  // ---- staging: LDS-DMA for plain inputs and weights; registers for the x2-upsampled input
  auto stage_dma = [&](int c, int buf) {
    float* si = smem + buf * BUF_F;
    float* sw = si + IN_F;
    if (!(IN1 == 2 && c >= NC0)) {
      const bool second = c >= NC0;
      const int cc = second ? c - NC0 : c;
      const int Cs = second ? C1 : C0;
      for (int i = wv; i < IN_INST; i += NW) {
        const int e = i * 64 + lane;
        const int col = e % HC, rh = e / HC, h = rh & 1, row = rh >> 1;
        const int y = iy0 + row, x = ix0 + col;
        const bool ok = e < IN_EL && y >= 0 && y < H && x >= 0 && x < W;
        const unsigned voff = ok ? (unsigned)((((size_t)y * W + x) * Cs + cc * 8 + h * 4) * 4) : 0x80000000u;
        if (second)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(r1, si + i * 256, 16, voff, 0, 0, 0);
        else
          __builtin_amdgcn_raw_ptr_buffer_load_lds(r0, si + i * 256, 16, voff, 0, 0, 0);
      }
    }
    const float* wc = wsl + (size_t)c * W_F;
    for (int i = wv; i < W_EL / 64; i += NW)
      __builtin_amdgcn_global_load_lds(wc + (i * 64 + lane) * 4, sw + i * 256, 16, 0, 0);
  };
  f32x4 ur[EPT][4];
  float uw[EPT][4];
  auto up_issue = [&](int c) {   // F.interpolate(x2, bilinear, align_corners=False) corner loads
    const int co = (c - NC0) * 8;
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      const int e = tid + k * NTH;
      const int col = e % HC, rh = e / HC, h = rh & 1, row = rh >> 1;
      const int y = iy0 + row, x = ix0 + col;
      const bool ok = e < IN_EL && y >= 0 && y < H && x >= 0 && x < W;
      const float sy = fmaxf(0.5f * ((float)y + 0.5f) - 0.5f, 0.f);
      const float sx = fmaxf(0.5f * ((float)x + 0.5f) - 0.5f, 0.f);
      const int y0 = min((int)sy, H1 - 1), x0 = min((int)sx, W1 - 1);
      const int y1 = y0 + (y0 < H1 - 1 ? 1 : 0), x1 = x0 + (x0 < W1 - 1 ? 1 : 0);
      const float ly1 = sy - (float)y0, lx1 = sx - (float)x0;
      uw[k][0] = ok ? 1.f - ly1 : 0.f;
      uw[k][1] = ok ? ly1 : 0.f;
      uw[k][2] = 1.f - lx1;
      uw[k][3] = lx1;
      const int c4 = co + h * 4;
      const int yy0 = ok ? y0 : 0, yy1 = ok ? y1 : 0, xx0 = ok ? x0 : 0, xx1 = ok ? x1 : 0;
      ur[k][0] = ld4(in1 + ((size_t)yy0 * W1 + xx0) * C1 + c4);
      ur[k][1] = ld4(in1 + ((size_t)yy0 * W1 + xx1) * C1 + c4);
      ur[k][2] = ld4(in1 + ((size_t)yy1 * W1 + xx0) * C1 + c4);
      ur[k][3] = ld4(in1 + ((size_t)yy1 * W1 + xx1) * C1 + c4);
    }
  };
  auto up_commit = [&](int buf) {
    float* si = smem + buf * BUF_F;
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      const int e = tid + k * NTH;
      if (e < IN_EL) {
        const f32x4 v = (uw[k][0] * (uw[k][2] * ur[k][0] + uw[k][3] * ur[k][1]) +
                         uw[k][1] * (uw[k][2] * ur[k][2] + uw[k][3] * ur[k][3])) * a.in1_scale;
        st4(si + e * 4, v);
      }
    }
  };

  f32x16 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x16{0};

  stage_dma(0, 0);
  if (IN1 == 2 && NC0 == 0) { up_issue(0); up_commit(0); }
  lds_dma_barrier();
  for (int c = 0; c < NC; ++c) {
    const int nb = (c + 1) & 1;
    const bool more = c + 1 < NC;
    const bool up_next = IN1 == 2 && more && c + 1 >= NC0;
    if (more) {
      stage_dma(c + 1, nb);
      if (up_next) up_issue(c + 1);
    }
    const float* si = smem + (c & 1) * BUF_F;
    const float* sw = si + IN_F;
    if constexpr (F16) {
#pragma unroll
      for (int pp = 0; pp < 5; ++pp) {
        const int tap = min(2 * pp + hf, 8);   // tap 9: any finite operand, its weights are zero
        const int ky = tap / 3, kx = tap - 3 * ky;
        f16x8 ah[MT], al[MT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const int oy = wv * MT + mt;
          const float* pa = si + (((oy * S + ky) * 2) * HC + l32 * S + kx) * 4;
          split_f16x3(ld4(pa), ld4(pa + HC * 4), ah[mt], al[mt]);
        }
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const float* wp = sw + (pp * NT + nt) * 512 + lane * 4;   // [pair][nt][plane][lane][8 halves]
          const f16x8 bh = ldh8(wp), bl = ldh8(wp + 256);
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            acc[mt][nt] = mfma16h(ah[mt], bh, acc[mt][nt]);
            acc[mt][nt] = mfma16h(ah[mt], bl, acc[mt][nt]);
            acc[mt][nt] = mfma16h(al[mt], bh, acc[mt][nt]);
          }
        }
      }
    } else
#pragma unroll
    for (int tap = 0; tap < T2; ++tap) {
      const int ky = tap / KS, kx = tap % KS;
      f32x4 av[MT], bv[NT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int oy = wv * MT + mt;
        av[mt] = ld4(si + (((oy * S + ky) * 2 + hf) * HC + l32 * S + kx) * 4);
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) bv[nt] = ld4(sw + ((tap * NT + nt) * 64 + lane) * 4);
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma32(av[mt][q], bv[nt][q], acc[mt][nt]);
    }
    if (up_next) up_commit(nb);
    lds_dma_barrier();
  }

  // ---- epilogue (smem is free after the final barrier): one 4-KB block per wave
  float* blk = smem + wv * 1024;
  const float* bias = a.bias[g] + slice * NJ;
  const int rpx = lane >> 3, c4 = lane & 7;   // read-back mapping: px = 8i + rpx, channels 4*c4..
  if constexpr (EPI == STIF_EPI_LSTM) {
    static_assert(NT == 4, "LSTM epilogue needs the i,f,o,g tiles of one hidden channel in one lane");
    float* hout = a.out[g] + (size_t)n * a.out_item;
    float* cout_ = a.out2[g] + (size_t)n * a.out2_item;
    const float* ccur = a.res[g] + (size_t)n * a.res_item;
    const int hc0 = slice * 32;           // hidden channels of this slice (STIF_PACK_LSTM)
    const float bi = bias[l32], bff = bias[32 + l32], bo = bias[64 + l32], bg = bias[96 + l32];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int y = oy0 + wv * MT + mt;
      const int yc = min(y, a.Ho - 1);
      f32x16 hv, cv;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int x = min(ox0 + mfma_row(r, lane), a.Wo - 1);
        const float cc = ccur[((size_t)yc * a.Wo + x) * 64 + hc0 + l32];
        const float i_ = sigmoidf_(acc[mt][0][r] + bi);
        const float f_ = sigmoidf_(acc[mt][1][r] + bff);
        const float o_ = sigmoidf_(acc[mt][2][r] + bo);
        const float g_ = tanhf(acc[mt][3][r] + bg);
        const float cn = f_ * cc + i_ * g_;
        cv[r] = cn;
        hv[r] = o_ * tanhf(cn);
      }
#pragma unroll
      for (int which = 0; which < 2; ++which) {
        tile_to_lds(blk, which ? cv : hv, lane);
        float* dst = which ? cout_ : hout;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int px = i * 8 + rpx, x = ox0 + px;
          const f32x4 v = lds_row4(blk, px, c4);
          if (y < a.Ho && x < a.Wo) st4(dst + ((size_t)y * a.Wo + x) * 64 + hc0 + c4 * 4, v);
        }
      }
    }
  } else {
    float* out = a.out[g] + (size_t)n * a.out_item;
    const float* res = (EPI == STIF_EPI_RES) ? a.res[g] + (size_t)n * a.res_item : nullptr;
    const int cs = a.cout;   // pixel stride of the output
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int cob = slice * NJ + nt * 32;   // first cout of this tile
      if (cob >= a.cout) break;
      const float bv = bias[nt * 32 + l32];
      const int co = cob + l32;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int y = oy0 + wv * MT + mt;
        f32x16 v;
        bool bad = false;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float t = acc[mt][nt][r] * (F16 ? F16X3_UNSCALE : 1.f) + bv;
          if (F16) bad |= not_finite(t);
          if (EPI == STIF_EPI_LRELU) t = lrelu01(t);
          if (EPI == STIF_EPI_RELU) t = fmaxf(t, 0.f);
          if (EPI == STIF_EPI_OFFMASK) {
            if (co < 216 && (co % 3) == 2) t = sigmoidf_(t);
          }
          v[r] = t;
        }
        if (F16) report_range(a.status, bad && co < a.cout);
        tile_to_lds(blk, v, lane);
        f32x4 rv[4];
        if (EPI == STIF_EPI_RES) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int x = min(ox0 + i * 8 + rpx, a.Wo - 1);
            rv[i] = ld4(res + ((size_t)min(y, a.Ho - 1) * a.Wo + x) * cs + cob + c4 * 4);
          }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int px = i * 8 + rpx, x = ox0 + px;
          f32x4 o = lds_row4(blk, px, c4);
          if (EPI == STIF_EPI_RES) o = rv[i] + o;
          if (y < a.Ho && x < a.Wo && cob + c4 * 4 < a.cout)
            st4(out + ((size_t)y * a.Wo + x) * cs + cob + c4 * 4, o);
        }
      }
    }
  }
}

// ---------------------------------------------------------------- 1x1 convs on split-fp16 MFMA
// k_conv1x1<NC, IN1>: the 1x1 convs of the STIF graph on split-fp16 MFMA, EPI_NONE -- the (64 | 64) ->
// 64 cat convs (Easy_PCD / PCD fusion, ConvBLSTM conv_1x1; Sakuya_arch_test.py:141,254; NC = 8,
// IN1) and the decoder's LR projection 200 -> 256 (NC = 13, the last 16-channel chunk half used).
// HBM-bound (e.g. 768 B and 16 KFLOP per pixel for the cat convs), so the kernel is built for
// memory-level parallelism: the 64-cout slice's weights (NC 16-channel chunks x 2 N-tiles x 2 planes)
// are LDS-DMA'd once per workgroup, and each wave walks 32-pixel M-tiles, issuing all of a tile's
// 16-B activation loads per lane (its pixel's 8 consecutive channels 16 c + 8 h.. of chunk c for lane
// half h) before its first MFMA; outputs leave as b32 stores, a half-wave writing one pixel's 32
// couts (128 B).  Tiles never straddle items (an item's last tile is partial: its lanes past H * W
// load the last pixel and store nothing).  Pixel p of item n: in0 + n * in0_item + p * C0 (in1 alike).
template <int NC, int IN1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(IN1 ? 4 : 2))) void k_conv1x1(stif_conv_args a,
                                                                                                int tiles_per_item) {
  __shared__ __attribute__((aligned(16))) float sw[NC * 1024];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, hf = lane >> 5, l32 = lane & 31;
  const int slice = blockIdx.y, g = blockIdx.z;
  const float* wsl = a.w[g] + (size_t)slice * NC * 1024;
  // (through a plain pointer: the builtin on the dependent-size __shared__ array itself makes this
  // clang drop the kernel's host launch stub)
  float* const swp = sw;
  for (int i = wv; i < NC * 4; i += 4)
    __builtin_amdgcn_global_load_lds(wsl + (i * 64 + lane) * 4, swp + i * 256, 16, 0, 0);
  lds_dma_barrier();
  const int ntiles = tiles_per_item * a.nitems;
  const int HW = a.H * a.W, C0 = IN1 ? 64 : a.C0, C1 = 64;   // host: (64 | 64) or one C0-channel input
  constexpr int NC0 = IN1 ? NC / 2 : NC;   // chunks read from in0
  const float b0 = a.bias[g][slice * 64 + l32], b1 = a.bias[g][slice * 64 + 32 + l32];
  bool bad = false;
  for (int mt = blockIdx.x * 4 + wv; mt < ntiles; mt += gridDim.x * 4) {
    const int n = mt / tiles_per_item, p0 = (mt - n * tiles_per_item) * 32;
    const size_t px = (size_t)min(p0 + l32, HW - 1);
    const float* x0 = a.in0[g] + (size_t)n * a.in0_item + px * C0;
    const float* x1 = IN1 ? a.in1[g] + (size_t)n * a.in1_item + px * C1 : x0;
    f32x4 xv[NC][2];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int ch = 16 * (c < NC0 ? c : c - NC0);
      const int cs = c < NC0 ? C0 : C1;
      // a half-used last chunk (C % 16 == 8): lane half 1 re-reads half 0's channels (zero weights)
      const float* xp = (c < NC0 ? x0 : x1) + ch + (ch + 8 < cs ? 8 * hf : 0);
      xv[c][0] = ld4(xp);
      xv[c][1] = ld4(xp + 4);
    }
    f32x16 acc0 = f32x16{0}, acc1 = f32x16{0};
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      f16x8 ah, al;
      split_f16x3(xv[c][0], xv[c][1], ah, al);
      const float* wp = sw + c * 1024 + lane * 4;   // [chunk][nt][plane][lane][8 halves]
      const f16x8 bh0 = ldh8(wp), bl0 = ldh8(wp + 256), bh1 = ldh8(wp + 512), bl1 = ldh8(wp + 768);
      acc0 = mfma16h(ah, bh0, acc0);
      acc1 = mfma16h(ah, bh1, acc1);
      acc0 = mfma16h(ah, bl0, acc0);
      acc1 = mfma16h(ah, bl1, acc1);
      acc0 = mfma16h(al, bh0, acc0);
      acc1 = mfma16h(al, bh1, acc1);
    }
    float* o = a.out[g] + (size_t)n * a.out_item + (size_t)p0 * a.cout + slice * 64 + l32;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float v0 = acc0[r] * F16X3_UNSCALE + b0, v1 = acc1[r] * F16X3_UNSCALE + b1;
      bad |= not_finite(v0 + v1);
      const int pr = mfma_row(r, lane);
      if (p0 + pr < HW) {
        o[(size_t)pr * a.cout] = v0;
        o[(size_t)pr * a.cout + 32] = v1;
      }
    }
  }
  report_range(a.status, bad);
}

template <int NC, int IN1>
int launch_conv1x1(const stif_conv_args& a, hipStream_t st, int wg_per_cu) {
  const int tpi = (a.H * a.W + 31) / 32;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  const long long wgs = ((long long)tpi * a.nitems + 3) / 4;
  // wg_per_cu workgroups per CU over all (slice, group) grid planes, each walking several M-tiles
  const int per = a.ngroups * (a.cout / 64);
  const int gx = (int)std::max<long long>(1, std::min<long long>(wgs, ((long long)wg_per_cu * cus + per - 1) / per));
  hipLaunchKernelGGL((k_conv1x1<NC, IN1>), dim3(gx, a.cout / 64, a.ngroups), dim3(256), 0, st, a, tpi);
  return stif_check_launch("stif_conv2d_nhwc");
}

template <int KS, int S, int MT, int NT, int NW, int IN1, int EPI, int F16 = 0>
int launch(const stif_conv_args& a, hipStream_t st) {
  constexpr int TH = NW * MT;
  const int tiles = ((a.Wo + 31) / 32) * ((a.Ho + TH - 1) / TH);
  const int slices = ((a.cout + 31) / 32 + NT - 1) / NT;
  dim3 grid(tiles, slices, a.ngroups * a.nitems);
  hipLaunchKernelGGL((k_conv<KS, S, MT, NT, NW, IN1, EPI, F16>), grid, dim3(NW * 64), 0, st, a);
  return stif_check_launch("stif_conv2d_nhwc");
}

// ---------------------------------------------------------------- conv_first (3 -> 64)
__global__ __launch_bounds__(256) void k_conv_first(const float* __restrict__ x, const float* __restrict__ w,
                                                    const float* __restrict__ b, float* __restrict__ out,
                                                    int n, int h, int wd) {
  __shared__ float s_w[27 * 64];   // [cin*9+tap][cout]
  __shared__ float s_b[64];
  for (int e = threadIdx.x; e < 27 * 64; e += 256) {
    const int co = e & 63, k = e >> 6;
    s_w[e] = w[co * 27 + k];
  }
  if (threadIdx.x < 64) s_b[threadIdx.x] = b[threadIdx.x];
  __syncthreads();
  // thread = (pixel, 16-cout quarter)
  const long long total = (long long)n * h * wd * 4;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const int qd = (int)(e & 3);
    const long long pix = e >> 2;
    const int xx = (int)(pix % wd);
    const int yy = (int)((pix / wd) % h);
    const int img = (int)(pix / ((long long)wd * h));
    float acc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = 0.f;
#pragma unroll 1
    for (int ci = 0; ci < 3; ++ci) {
      const float* xp = x + ((size_t)img * 3 + ci) * h * wd;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int y = yy + t / 3 - 1, xq = xx + t % 3 - 1;
        const float v = (y >= 0 && y < h && xq >= 0 && xq < wd) ? xp[(size_t)y * wd + xq] : 0.f;
        const float* wr = s_w + (ci * 9 + t) * 64 + qd * 16;
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[j] = fmaf(v, wr[j], acc[j]);
      }
    }
    float* op = out + pix * 64 + qd * 16;
#pragma unroll
    for (int j = 0; j < 16; j += 4) {
      f32x4 v;
      v[0] = lrelu01(acc[j] + s_b[qd * 16 + j]);
      v[1] = lrelu01(acc[j + 1] + s_b[qd * 16 + j + 1]);
      v[2] = lrelu01(acc[j + 2] + s_b[qd * 16 + j + 2]);
      v[3] = lrelu01(acc[j + 3] + s_b[qd * 16 + j + 3]);
      st4(op + j, v);
    }
  }
}

}  // namespace

extern "C" int stif_conv2d_nhwc(const stif_conv_args* pa, void* stream) {
  if (!pa) return stif_fail(STIF_E_INVALID, "stif_conv2d_nhwc: null args");
  const stif_conv_args& a = *pa;
  hipStream_t st = (hipStream_t)stream;
  if (a.ngroups < 1 || a.ngroups > STIF_MAX_GROUPS || a.nitems < 1)
    return stif_fail(STIF_E_INVALID, "stif_conv2d_nhwc: bad ngroups/nitems");
  if ((long long)a.H * a.W * std::max(a.C0, std::max(a.C1, a.cout)) * 4 >= 0x7fffffffLL)
    return stif_fail(STIF_E_INVALID, "stif_conv2d_nhwc: item larger than 2 GB (buffer addressing)");
  const bool f16 = a.flags & STIF_CONV_F16X3;
  const bool f16_cat = a.in1_mode == 1 && a.C0 == 64 && a.C1 == 64;   // (64 | 64) -> 64k
  const bool f16_proj = a.in1_mode == 0 && a.C0 == 200;                 // the decoder's LR projection
  const bool f16_1x1 = a.ks == 1 && a.stride == 1 && (f16_cat || f16_proj) && a.cout % 64 == 0 && a.epi == STIF_EPI_NONE;
  if (f16 && !(a.ks == 3 && a.stride == 2 && a.cout == 64 && a.C0 == 64 && a.in1_mode == 0) && !f16_1x1)
    return stif_fail(STIF_E_INVALID, "stif_conv2d_nhwc: STIF_CONV_F16X3 takes the 3x3 stride-2 64 -> 64 convs and "
                                     "the 1x1 (64 | 64) -> 64k and 200 -> 64k convs only");
  if (a.C0 % 8 || a.C0 <= 0 || (a.in1_mode && (a.C1 % 8 || a.C1 <= 0)))
    return stif_fail(STIF_E_INVALID, "stif_conv2d_nhwc: channel counts must be multiples of 8");
  const int pad = a.ks / 2;
  if ((a.ks != 1 && a.ks != 3) || (a.stride != 1 && a.stride != 2) ||
      a.Ho != (a.H + 2 * pad - a.ks) / a.stride + 1 || a.Wo != (a.W + 2 * pad - a.ks) / a.stride + 1)
    return stif_fail(STIF_E_INVALID, "stif_conv2d_nhwc: bad ks/stride/output size");
  if (a.in1_mode == 2 && (a.H % 2 || a.W % 2))
    return stif_fail(STIF_E_INVALID, "stif_conv2d_nhwc: x2 upsample input needs even H, W");
  if ((a.epi == STIF_EPI_RES || a.epi == STIF_EPI_LSTM) && !a.res[0])
    return stif_fail(STIF_E_INVALID, "stif_conv2d_nhwc: epilogue needs res");

  // dispatch on the shapes the STIF graph uses
  if (a.ks == 3 && a.stride == 1 && a.epi == STIF_EPI_LSTM) {
    if (a.cout != 256 || a.in1_mode != 1) return stif_fail(STIF_E_INVALID, "LSTM conv must be 128->256");
    return launch<3, 1, 1, 4, 8, 1, STIF_EPI_LSTM>(a, st);
  }
  if (a.ks == 3 && a.stride == 1 && a.epi == STIF_EPI_OFFMASK) {
    if (a.in1_mode != 0 || a.cout > 224) return stif_fail(STIF_E_INVALID, "offset conv must be 64->216");
    return launch<3, 1, 1, 7, 8, 0, STIF_EPI_OFFMASK>(a, st);
  }
  if (a.ks == 3 && a.stride == 2) {
    if (a.in1_mode != 0) return stif_fail(STIF_E_INVALID, "strided conv takes one input");
    switch (a.epi) {
      case STIF_EPI_LRELU:
        return f16 ? launch<3, 2, 1, 2, 4, 0, STIF_EPI_LRELU, 1>(a, st) : launch<3, 2, 1, 2, 4, 0, STIF_EPI_LRELU>(a, st);
      case STIF_EPI_NONE:
        return f16 ? launch<3, 2, 1, 2, 4, 0, STIF_EPI_NONE, 1>(a, st) : launch<3, 2, 1, 2, 4, 0, STIF_EPI_NONE>(a, st);
      default: break;
    }
    return stif_fail(STIF_E_INVALID, "strided conv: unsupported epilogue");
  }
  if (a.ks == 1) {
    if (f16) return f16_cat ? launch_conv1x1<8, 1>(a, st, 4) : launch_conv1x1<13, 0>(a, st, 3);
    if (a.epi != STIF_EPI_NONE) return stif_fail(STIF_E_INVALID, "1x1 conv: unsupported epilogue");
    if (a.in1_mode == 0) return launch<1, 1, 2, 2, 4, 0, STIF_EPI_NONE>(a, st);
    if (a.in1_mode == 1) return launch<1, 1, 2, 2, 4, 1, STIF_EPI_NONE>(a, st);
    return stif_fail(STIF_E_INVALID, "1x1 conv: unsupported in1 mode");
  }
  // 3x3 stride 1
#define STIF_CONV_CASE(IN1)                                                   \
  switch (a.epi) {                                                            \
    case STIF_EPI_NONE: return launch<3, 1, 2, 2, 4, IN1, STIF_EPI_NONE>(a, st); \
    case STIF_EPI_LRELU: return launch<3, 1, 2, 2, 4, IN1, STIF_EPI_LRELU>(a, st); \
    case STIF_EPI_RELU: return launch<3, 1, 2, 2, 4, IN1, STIF_EPI_RELU>(a, st); \
    case STIF_EPI_RES: return launch<3, 1, 2, 2, 4, IN1, STIF_EPI_RES>(a, st);   \
    default: break;                                                           \
  }
  if (a.in1_mode == 0) { STIF_CONV_CASE(0) }
  else if (a.in1_mode == 1) { STIF_CONV_CASE(1) }
  else if (a.in1_mode == 2) { STIF_CONV_CASE(2) }
#undef STIF_CONV_CASE
  return stif_fail(STIF_E_INVALID, "stif_conv2d_nhwc: unsupported combination");
}

extern "C" int stif_conv_first(const float* x, const float* w, const float* b, float* out, int n, int h,
                               int wd, void* stream) {
  if (!x || !w || !b || !out || n <= 0 || h <= 0 || wd <= 0)
    return stif_fail(STIF_E_INVALID, "stif_conv_first: bad arguments");
  const long long total = (long long)n * h * wd * 4;
  long long blocks = (total + 255) / 256;
  if (blocks > 65535) blocks = 65535;
  hipLaunchKernelGGL(k_conv_first, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, x, w, b, out, n,
                     h, wd);
  return stif_check_launch("stif_conv_first");
}
