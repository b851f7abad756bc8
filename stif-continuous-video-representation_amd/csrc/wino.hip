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
//     i crosses waves (one LDS exchange per 32-cout half).
// Input halo tiles (6 rows x 34 columns x 32 channels per phase) are LDS-DMA'd, double-buffered,
// even and odd columns in separate runs so a lane's 4 patch columns are conflict-free reads.
#include "abi_util.h"
#include "stif.h"
#include "stif_common.h"

namespace {

constexpr int WR = 4;      // output rows per workgroup
constexpr int HR = 6;      // halo rows
constexpr int HC = 34;     // halo columns
constexpr int PSUB = 4;    // 8-channel chunks per staging phase
constexpr int IN_EL = HR * PSUB * 2 * HC;      // 16-B elements per phase buffer
constexpr int IN_INST = (IN_EL + 63) / 64;     // LDS-DMA instructions per phase
constexpr int BUF_F = IN_INST * 256;           // floats per phase buffer
constexpr int EPI_F = 2 * 4 * 2 * 32 * 32;     // epilogue exchange: [nt][i][b][tile][32 co]
constexpr int SM_F = (2 * BUF_F > EPI_F) ? 2 * BUF_F : EPI_F;

// slot of halo column c in its (row, chunk, half) run: even columns first, then odd
STIF_DEV int col_slot(int c) { return (c & 1) ? 17 + (c >> 1) : (c >> 1); }

template <int IN1, int EPI>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_wino(stif_conv_args a) {
  __shared__ __attribute__((aligned(16))) float smem[SM_F];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wi = __builtin_amdgcn_readfirstlane(tid >> 6);   // transform row i of this wave
  const int hf = lane >> 5;
  const int tl = lane & 31;                                  // Winograd tile of this lane
  const int tyl = tl >> 4, txl = tl & 15;

  const int tiles_x = (a.Wo + 31) >> 5;
  const int tx = blockIdx.x % tiles_x;
  const int ty = blockIdx.x / tiles_x;
  const int slice = blockIdx.y;
  const int g = blockIdx.z / a.nitems;
  const int n = blockIdx.z - g * a.nitems;
  const int H = a.H, W = a.W, C0 = a.C0, C1 = a.C1;
  const float* in0 = a.in0[g] + (size_t)n * a.in0_item;
  const float* in1 = IN1 ? a.in1[g] + (size_t)n * a.in1_item : in0;
  const __amdgpu_buffer_rsrc_t r0 =
      __builtin_amdgcn_make_buffer_rsrc((void*)in0, (short)0, (int)((size_t)H * W * C0 * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t r1 = __builtin_amdgcn_make_buffer_rsrc(
      (void*)in1, (short)0, (int)((size_t)H * W * (IN1 ? C1 : C0) * 4), 0x00020000);
  const int oy0 = ty * WR, ox0 = tx * 32;
  const int iy0 = oy0 - 1, ix0 = ox0 - 1;
  const int NC0 = C0 >> 3;
  const int NC = NC0 + (IN1 ? (C1 >> 3) : 0);
  const int NP = (NC + PSUB - 1) / PSUB;
  // packed U: [slice][chunk][i][j][nt][lane][4]
  const float* wsl = a.w[g] + (size_t)slice * NC * 8192 + wi * 2048 + lane * 4;

  auto stage = [&](int p, int buf) {
    float* dst = smem + buf * BUF_F;
    for (int q = wi; q < IN_INST; q += 4) {
      const int e = q * 64 + lane;
      const int slot = e % HC;
      const int rest = e / HC;
      const int h = rest & 1, sub = (rest >> 1) % PSUB, row = (rest >> 1) / PSUB;
      const int col = slot < 17 ? 2 * slot : 2 * (slot - 17) + 1;
      const int k = p * PSUB + sub;
      const int y = iy0 + row, x = ix0 + col;
      const bool ok = e < IN_EL && k < NC && y >= 0 && y < H && x >= 0 && x < W;
      const bool second = IN1 && k >= NC0;
      const int Cs = second ? C1 : C0;
      const int cc = second ? k - NC0 : k;
      const unsigned voff = ok ? (unsigned)((((size_t)y * W + x) * Cs + cc * 8 + h * 4) * 4) : 0x80000000u;
      if (second)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r1, dst + q * 256, 16, voff, 0, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r0, dst + q * 256, 16, voff, 0, 0, 0);
    }
  };

  // rows of the 4x4 patch feeding transform row i: (B^T d)_i = d[rA] + sB * d[rB]
  const int rA = (wi == 0) ? 0 : (wi == 2 ? 2 : 1);
  const int rB = (wi == 3) ? 3 : (wi == 2 ? 1 : 2);
  const float sB = (wi == 1) ? 1.f : -1.f;
  const int s0 = col_slot(0) + txl, s1 = col_slot(1) + txl, s2 = col_slot(2) + txl, s3 = col_slot(3) + txl;

  f32x16 acc[4][2];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j][0] = acc[j][1] = f32x16{0};

  f32x4 bw[4][2];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) bw[j][nt] = ld4(wsl + (j * 2 + nt) * 256);

  stage(0, 0);
  lds_dma_barrier();
  for (int p = 0; p < NP; ++p) {
    if (p + 1 < NP) stage(p + 1, (p + 1) & 1);
    const float* buf = smem + (p & 1) * BUF_F;
    const int nsub = min(PSUB, NC - p * PSUB);
    for (int s = 0; s < nsub; ++s) {
      const int k = p * PSUB + s;
      // ---- input transform row i for this lane's tile and 4 channels
      const float* ra = buf + (((2 * tyl + rA) * PSUB + s) * 2 + hf) * HC * 4;
      const float* rb = buf + (((2 * tyl + rB) * PSUB + s) * 2 + hf) * HC * 4;
      const f32x4 t0 = ld4(ra + s0 * 4) + sB * ld4(rb + s0 * 4);
      const f32x4 t1 = ld4(ra + s1 * 4) + sB * ld4(rb + s1 * 4);
      const f32x4 t2 = ld4(ra + s2 * 4) + sB * ld4(rb + s2 * 4);
      const f32x4 t3 = ld4(ra + s3 * 4) + sB * ld4(rb + s3 * 4);
      f32x4 v[4];
      v[0] = t0 - t2;
      v[1] = t1 + t2;
      v[2] = t2 - t1;
      v[3] = t1 - t3;
      const bool more = k + 1 < NC;
      const float* wn = wsl + (size_t)(k + 1) * 8192;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[j][nt] = mfma32(v[j][e], bw[j][nt][e], acc[j][nt]);
        }
        // B operands of the next chunk, issued once this j's are consumed
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
          if (more) bw[j][nt] = ld4(wn + (j * 2 + nt) * 256);
      }
    }
    lds_dma_barrier();
  }

  // ---- output transform: P_i[b] = sum_j M[i][j] A[j][b] in registers, Y = sum_i A^T[a][i] P_i
  float* ex = smem;
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    f32x16 p0 = acc[0][nt] + acc[1][nt] + acc[2][nt];
    f32x16 p1 = acc[1][nt] - acc[2][nt] - acc[3][nt];
    float* d0 = ex + ((nt * 4 + wi) * 2 + 0) * 1024;
    float* d1 = ex + ((nt * 4 + wi) * 2 + 1) * 1024;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int t = mfma_row(r, lane);
      d0[t * 32 + tl] = p0[r];
      d1[t * 32 + tl] = p1[r];
    }
  }
  __syncthreads();
  const int c4 = tid & 7, t = tid >> 3;       // (tile, 4 couts) per thread and 32-cout half
  const int oyt = oy0 + 2 * (t >> 4), oxt = ox0 + 2 * (t & 15);
  const float* bias = a.bias[g] + slice * 64;
  float* out = a.out[g] + (size_t)n * a.out_item;
  const float* res = (EPI == STIF_EPI_RES) ? a.res[g] + (size_t)n * a.res_item : nullptr;
  const int cs = a.cout;
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int co = slice * 64 + nt * 32 + c4 * 4;
    if (co >= a.cout) break;
    f32x4 P[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int b = 0; b < 2; ++b) P[i][b] = ld4(ex + ((nt * 4 + i) * 2 + b) * 1024 + t * 32 + c4 * 4);
    const f32x4 bv = ld4(bias + nt * 32 + c4 * 4);
#pragma unroll
    for (int ar = 0; ar < 2; ++ar)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        f32x4 y = ar == 0 ? P[0][b] + P[1][b] + P[2][b] : P[1][b] - P[2][b] - P[3][b];
        y += bv;
        const int oy = oyt + ar, ox = oxt + b;
        if (oy < a.Ho && ox < a.Wo) {
          const size_t o = ((size_t)oy * a.Wo + ox) * cs + co;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (EPI == STIF_EPI_LRELU) y[e] = lrelu01(y[e]);
            if (EPI == STIF_EPI_RELU) y[e] = fmaxf(y[e], 0.f);
          }
          if (EPI == STIF_EPI_RES) y += ld4(res + o);
          st4(out + o, y);
        }
      }
  }
}

template <int IN1, int EPI>
int launch(const stif_conv_args& a, hipStream_t st) {
  const int tiles = ((a.Wo + 31) / 32) * ((a.Ho + WR - 1) / WR);
  const int slices = (a.cout + 63) / 64;
  dim3 grid(tiles, slices, a.ngroups * a.nitems);
  hipLaunchKernelGGL((k_wino<IN1, EPI>), grid, dim3(256), 0, st, a);
  return stif_check_launch("stif_conv3x3_wino");
}

}  // namespace

extern "C" int stif_conv3x3_wino(const stif_conv_args* pa, void* stream) {
  if (!pa) return stif_fail(STIF_E_INVALID, "stif_conv3x3_wino: null args");
  const stif_conv_args& a = *pa;
  hipStream_t st = (hipStream_t)stream;
  if (a.ngroups < 1 || a.ngroups > STIF_MAX_GROUPS || a.nitems < 1)
    return stif_fail(STIF_E_INVALID, "stif_conv3x3_wino: bad ngroups/nitems");
  if (a.ks != 3 || a.stride != 1 || a.Ho != a.H || a.Wo != a.W)
    return stif_fail(STIF_E_INVALID, "stif_conv3x3_wino: 3x3 stride-1 'same' convolution only");
  if (a.C0 % 8 || a.C0 <= 0 || (a.in1_mode == 1 && (a.C1 % 8 || a.C1 <= 0)))
    return stif_fail(STIF_E_INVALID, "stif_conv3x3_wino: channel counts must be multiples of 8");
  if (a.cout % 64) return stif_fail(STIF_E_INVALID, "stif_conv3x3_wino: cout must be a multiple of 64");
  if (a.epi == STIF_EPI_RES && !a.res[0]) return stif_fail(STIF_E_INVALID, "stif_conv3x3_wino: RES needs res");
#define STIF_WINO_CASE(IN1)                                              \
  switch (a.epi) {                                                       \
    case STIF_EPI_NONE: return launch<IN1, STIF_EPI_NONE>(a, st);        \
    case STIF_EPI_LRELU: return launch<IN1, STIF_EPI_LRELU>(a, st);      \
    case STIF_EPI_RELU: return launch<IN1, STIF_EPI_RELU>(a, st);        \
    case STIF_EPI_RES: return launch<IN1, STIF_EPI_RES>(a, st);          \
    default: break;                                                      \
  }
  if (a.in1_mode == 0) { STIF_WINO_CASE(0) }
  else if (a.in1_mode == 1) { STIF_WINO_CASE(1) }
#undef STIF_WINO_CASE
  return stif_fail(STIF_E_INVALID, "stif_conv3x3_wino: unsupported in1 mode / epilogue");
}
