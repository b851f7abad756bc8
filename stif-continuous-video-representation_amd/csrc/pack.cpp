// Host-side (CPU) weight packing for the gfx950 kernels.  Pure C++, no GPU needed;
// runs once per load_state_dict (reference weight layouts: nn.Conv2d [cout][cin][k][k],
// nn.Linear [out][in], as in the 442-key LunaTokis state dict).
#include <string.h>

#include <vector>

#include "dec_layout.h"
#include "stif.h"

extern int stif_fail(int code, const char* msg);

namespace {

int round32(int x) { return (x + 31) & ~31; }
int round64(int x) { return (x + 63) & ~63; }

// Winograd F(2x2, 3x3) weight transform U = G g G^T (wino.hip), in double
void wino_u(const float* g, double u[4][4]) {
  static const double G[4][3] = {{1, 0, 0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0, 0, 1}};
  double t[4][3];
  for (int a = 0; a < 4; ++a)
    for (int q = 0; q < 3; ++q) t[a][q] = G[a][0] * g[q] + G[a][1] * g[3 + q] + G[a][2] * g[6 + q];
  for (int a = 0; a < 4; ++a)
    for (int b = 0; b < 4; ++b) u[a][b] = t[a][0] * G[b][0] + t[a][1] * G[b][1] + t[a][2] * G[b][2];
}

// 32-wide N-tiles per workgroup slice of stif_conv2d_nhwc for a packing mode (conv.hip dispatch)
int slice_tiles(int mode) { return mode == STIF_PACK_OFFMASK ? 7 : (mode == STIF_PACK_LSTM ? 4 : 2); }
int cout_padded(int cout, int mode) {
  const int nj = 32 * slice_tiles(mode);
  return (cout + nj - 1) / nj * nj;
}

// source row of packed output channel j
int src_row(int j, int cout, int mode) {
  if (j >= cout) return -1;
  if (mode == STIF_PACK_OFFMASK) {
    // packed [group][tap][dy, dx, mask]  <-  reference channels: offset = cat(o1, o2) = ch 0..143 with
    // (group g, tap k) at g*18 + 2k (+1 for w); mask = ch 144 + g*9 + k (dcn_v2.py:134-138,
    // dcn_v2_im2col_cuda.cu:160-167)
    const int g = j / 27, k = (j % 27) / 3, e = j % 3;
    if (e == 0) return g * 18 + 2 * k;
    if (e == 1) return g * 18 + 2 * k + 1;
    return 144 + g * 9 + k;
  }
  if (mode == STIF_PACK_WINO_LSTM) {
    // packed 4h + gate <- reference row gate*64 + h (gates i, f, o, g; convlstm.py:49)
    return (j & 3) * 64 + (j >> 2);
  }
  if (mode == STIF_PACK_LSTM) {
    // packed slice s (128 outputs) = gates i, f, o, g of hidden channels 32s..32s+31 (convlstm.py:49)
    const int s = j / 128, gate = (j % 128) / 32, jj = j % 32;
    return gate * 64 + s * 32 + jj;
  }
  return j;
}

// F(q, h): feature held by MFMA accumulator register q of lane half h (see dec_layout.h)
inline int feat_of(int q, int h) { return (q & 3) + 8 * (q >> 2) + 4 * h; }

// pack W[rows x cols] (row-major, leading dim ld, sub-block starting at (r0, c0), n_out x k_in)
void pack_tiles(float* dst, const float* W, int ld, int r0, int c0, int n_out, int k_in) {
  const int OT = (n_out + 31) / 32, KT = (k_in + 31) / 32;
  for (int ot = 0; ot < OT; ++ot)
    for (int kt = 0; kt < KT; ++kt)
      for (int v = 0; v < 4; ++v)
        for (int lane = 0; lane < 64; ++lane)
          for (int e = 0; e < 4; ++e) {
            const int q = 4 * v + e;
            const int row = ot * 32 + (lane & 31);
            const int col = kt * 32 + feat_of(q, lane >> 5);
            const float val = (row < n_out && col < k_in) ? W[(size_t)(r0 + row) * ld + c0 + col] : 0.f;
            dst[((((size_t)ot * KT + kt) * 4 + v) * 64 + lane) * 4 + e] = val;
          }
}

void copy_vec(float* dst, const float* src, int n, int npad) {
  for (int i = 0; i < npad; ++i) dst[i] = i < n ? src[i] : 0.f;
}

void column(float* dst, const float* W, int ld, int rows, int col) {
  for (int i = 0; i < rows; ++i) dst[i] = W[(size_t)i * ld + col];
}

// SineLayer: sin(omega_0 * (W x + b)) with omega_0 = 30 (SIREN.py:44-51): the packed copies of every
// sine layer's weights and bias carry the factor (computed in double, rounded once), so the kernels
// evaluate sin(W' x + b') without the multiply.  `rev`: the factor is omega_0 / (2 pi), i.e. the
// pre-activations come out in revolutions, the unit of the hardware sine (v_sin_f32), and the kernel's
// range reduction is x - rint(x) (the f16x3 decoder: stif_sin_rev)
constexpr double OMEGA0 = 30.0;
constexpr double TWO_PI = 6.283185307179586476925286766559;
std::vector<float> omega(const float* src, size_t n, bool rev) {
  const double s = rev ? OMEGA0 / TWO_PI : OMEGA0;
  std::vector<float> d(n);
  for (size_t i = 0; i < n; ++i) d[i] = (float)(s * (double)src[i]);
  return d;
}

}  // namespace

extern "C" size_t stif_conv_weight_floats(int cout, int cin, int ks, int mode) {
  // DCNSEP | F16X3 (the fused DCN_sep's offset/mask conv): 36 steps x 8 groups x 2 planes x 1 KB
  if (mode == (STIF_PACK_DCNSEP | STIF_PACK_F16X3)) return (size_t)36 * 7 * 2 * 256;
  if (mode == (STIF_PACK_DCNPAIR | STIF_PACK_F16X3)) return (size_t)4 * 9 * 2 * 2 * 256;
  // PLAIN | F16X3 (the DCN core, 64 -> 64 3x3): 5 tap pairs x 2 nt x 2 planes x 1 KB per 8-channel group
  if (mode == (STIF_PACK_PLAIN | STIF_PACK_F16X3) && ks == 3) return (size_t)(cin / 8) * 5 * 2 * 2 * 256;
  // PLAIN | F16X3 1x1 (k_conv1x1): 2 nt x 2 planes x 1 KB per (64-cout slice, 16-channel chunk)
  if (mode == (STIF_PACK_PLAIN | STIF_PACK_F16X3) && ks == 1) return (size_t)(cout + 63) / 64 * ((cin + 15) / 16) * 1024;
  mode &= ~STIF_PACK_F16X3;   // Winograd: same bytes, two fp16 planes per fp32 value
  if (mode == STIF_PACK_WINO || mode == STIF_PACK_WINO_OFFMASK || mode == STIF_PACK_WINO_LSTM)
    return (size_t)round64(cout) * cin * 16;
  return (size_t)cout_padded(cout, mode) * cin * ks * ks;
}

extern "C" size_t stif_conv_bias_floats(int cout, int mode) {
  if (mode == (STIF_PACK_DCNSEP | STIF_PACK_F16X3)) return 256;
  if (mode == (STIF_PACK_DCNPAIR | STIF_PACK_F16X3)) return 64;
  mode &= ~STIF_PACK_F16X3;
  return (mode == STIF_PACK_WINO || mode == STIF_PACK_WINO_OFFMASK || mode == STIF_PACK_WINO_LSTM)
             ? (size_t)round64(cout)
             : (size_t)cout_padded(cout, mode);
}

namespace {
// [slice][chunk][i][j][nt][lane][4]: U[4i+j] of cout slice*64 + nt*32 + (lane & 31), input channel
// chunk*8 + 4*(lane >> 5) + e -- the B fragments wave i of stif_conv3x3_wino loads per 8-channel chunk
// perm: output-row permutation of the direct packing (STIF_PACK_PLAIN or STIF_PACK_OFFMASK)
int pack_wino(const float* w, const float* b, int cout, int cin, int perm, float* w_dst, float* b_dst) {
  const int cp = round64(cout), NS = cp / 64, NC = cin / 8;
  for (int s = 0; s < NS; ++s)
    for (int nt = 0; nt < 2; ++nt)
      for (int l = 0; l < 64; ++l) {
        const int co = s * 64 + nt * 32 + (l & 31);
        const int sr = src_row(co, cout, perm);
        for (int c = 0; c < NC; ++c)
          for (int e = 0; e < 4; ++e) {
            const int ci = c * 8 + 4 * (l >> 5) + e;
            double u[4][4] = {{0}};
            if (sr >= 0) wino_u(w + ((size_t)sr * cin + ci) * 9, u);
            for (int i = 0; i < 4; ++i)
              for (int j = 0; j < 4; ++j)
                w_dst[((((((size_t)s * NC + c) * 4 + i) * 4 + j) * 2 + nt) * 64 + l) * 4 + e] = (float)u[i][j];
          }
      }
  if (b_dst)
    for (int j = 0; j < cp; ++j) {
      const int sr = src_row(j, cout, perm);
      b_dst[j] = (sr >= 0 && b) ? b[sr] : 0.f;
    }
  return STIF_OK;
}

// x * 2^10 split into fp16 h = rne(x 2^10), l = rne(x 2^10 - h) (double arithmetic)
void split_f16x3_host(double x, _Float16* h, _Float16* l) {
  const double v = x * 1024.0;
  *h = (_Float16)v;
  *l = (_Float16)(v - (double)*h);
}

// split range of a packed weight: |x 2^10| must round to a finite fp16 (|x| < 64 less half an fp16 ulp)
constexpr double F16X3_WMAX = 65504.0 / 1024.0;
bool f16x3_ok(double x) { return x >= -F16X3_WMAX && x <= F16X3_WMAX; }
int range_fail(const char* what) {
  return stif_fail(STIF_E_RANGE, what);
}

// PLAIN | F16X3, the fused DCN core (k_dcn<F16>): [group][tap pair p][nt][plane][lane][8 halves];
// element e of lane l holds tap 2p + (l >> 5) (tap 9 = zero padding), input channel 8 group + e,
// cout nt * 32 + (l & 31)
int pack_dcn_f16x3(const float* w, const float* b, int cout, int cin, float* w_dst, float* b_dst) {
  for (size_t i = 0; i < (size_t)cout * cin * 9; ++i)
    if (!f16x3_ok(w[i])) return range_fail("stif_pack_conv_weight: a weight is outside the f16x3 range (|w| < 64); pack it without STIF_PACK_F16X3");
  _Float16* dst = reinterpret_cast<_Float16*>(w_dst);
  for (int g = 0; g < cin / 8; ++g)
    for (int p = 0; p < 5; ++p)
      for (int nt = 0; nt < 2; ++nt)
        for (int l = 0; l < 64; ++l)
          for (int e = 0; e < 8; ++e) {
            const int tap = 2 * p + (l >> 5), ci = 8 * g + e, co = nt * 32 + (l & 31);
            const double x = tap < 9 ? (double)w[((size_t)co * cin + ci) * 9 + tap] : 0.0;
            const size_t o = ((((size_t)g * 5 + p) * 2 + nt) * 2) * 512 + l * 8 + e;
            split_f16x3_host(x, dst + o, dst + o + 512);
          }
  if (b_dst)
    for (int j = 0; j < cout; ++j) b_dst[j] = b ? b[j] : 0.f;
  return STIF_OK;
}

// STIF_PACK_F16X3: [slice][pair q][i][j][nt][plane][lane][8 halves]; element e of lane l holds input
// channel 16 q + 8 (e >> 2) + 4 (l >> 5) + (e & 3) -- lane half h supplies channels 4h..4h+3 of both
// 8-channel chunks of the pair, exactly the A operand k_wino<F16> builds -- as U * 2^10 split into
// h = rne16(U 2^10), l = rne16(U 2^10 - h) (double arithmetic, so l is the correctly rounded residual)
int pack_wino_f16x3(const float* w, const float* b, int cout, int cin, int perm, float* w_dst, float* b_dst) {
  if (cin % 16) return stif_fail(STIF_E_INVALID, "f16x3 winograd pack needs cin % 16 == 0");
  const int cp = round64(cout), NS = cp / 64, NQ = cin / 16;
  // |U| <= 9/4 max|g| (G g G^T, rows of G sum to <= 1.5 in magnitude): checked on U itself
  for (size_t i = 0; i < (size_t)cout * cin; ++i) {
    double u[4][4];
    wino_u(w + i * 9, u);
    for (int a = 0; a < 16; ++a)
      if (!f16x3_ok(u[a / 4][a % 4]))
        return range_fail("stif_pack_conv_weight: a Winograd weight G g G^T is outside the f16x3 range (|U| < 64); pack it without STIF_PACK_F16X3");
  }
  _Float16* dst = reinterpret_cast<_Float16*>(w_dst);
  for (int s = 0; s < NS; ++s)
    for (int nt = 0; nt < 2; ++nt)
      for (int l = 0; l < 64; ++l) {
        const int co = s * 64 + nt * 32 + (l & 31);
        const int sr = src_row(co, cout, perm);
        for (int q = 0; q < NQ; ++q)
          for (int e = 0; e < 8; ++e) {
            const int ci = 16 * q + 8 * (e >> 2) + 4 * (l >> 5) + (e & 3);
            double u[4][4] = {{0}};
            if (sr >= 0) wino_u(w + ((size_t)sr * cin + ci) * 9, u);
            for (int i = 0; i < 4; ++i)
              for (int j = 0; j < 4; ++j) {
                const double x = u[i][j] * 1024.0;
                const _Float16 h = (_Float16)x;
                const _Float16 lo = (_Float16)(x - (double)h);
                const size_t o = ((((((size_t)s * NQ + q) * 4 + i) * 4 + j) * 2 + nt) * 2) * 512 + l * 8 + e;
                dst[o] = h;
                dst[o + 512] = lo;
              }
          }
      }
  if (b_dst)
    for (int j = 0; j < cp; ++j) {
      const int sr = src_row(j, cout, perm);
      b_dst[j] = (sr >= 0 && b) ? b[sr] : 0.f;
    }
  return STIF_OK;
}
// PLAIN | F16X3, 1x1 (k_conv1x1): [slice][chunk c16][nt][plane][lane][8 halves]; element e of lane l
// holds input channel 16 c16 + 8 (l >> 5) + e of cout slice * 64 + nt * 32 + (l & 31) -- lane half h
// supplies its pixel's 8 consecutive channels 16 c16 + 8 h .. as the A operand -- as W * 2^10 split;
// a half-used last chunk (cin % 16 == 8) has zero weights in its upper half
int pack_1x1_f16x3(const float* w, const float* b, int cout, int cin, float* w_dst, float* b_dst) {
  if (cout % 64) return stif_fail(STIF_E_INVALID, "PLAIN | F16X3 1x1 packing needs cout % 64 == 0");
  for (size_t i = 0; i < (size_t)cout * cin; ++i)
    if (!f16x3_ok(w[i])) return range_fail("stif_pack_conv_weight: a weight is outside the f16x3 range (|w| < 64); pack it without STIF_PACK_F16X3");
  const int NS = cout / 64, NC = (cin + 15) / 16;
  _Float16* dst = reinterpret_cast<_Float16*>(w_dst);
  for (int s = 0; s < NS; ++s)
    for (int c = 0; c < NC; ++c)
      for (int nt = 0; nt < 2; ++nt)
        for (int l = 0; l < 64; ++l)
          for (int e = 0; e < 8; ++e) {
            const int co = s * 64 + nt * 32 + (l & 31), ci = 16 * c + 8 * (l >> 5) + e;
            const size_t o = (((((size_t)s * NC + c) * 2 + nt) * 2) * 64 + l) * 8 + e;
            split_f16x3_host(ci < cin ? (double)w[(size_t)co * cin + ci] : 0.0, dst + o, dst + o + 512);
          }
  if (b_dst)
    for (int j = 0; j < cout; ++j) b_dst[j] = b ? b[j] : 0.f;
  return STIF_OK;
}
// DCNSEP | F16X3: conv_offset_mask (216 x 64 x 3 x 3) as the A operands of k_dcn_sep's phase 1,
// [k = 9 c + tap][M-tile m 7][plane][lane][8 halves].  Row i of M-tile m lands in accumulator register
// r = (i & 3) + 4 (i >> 3) of lane half h = (i >> 2) & 1; lane half h owns the deformable groups
// h, h + 2, h + 4, h + 6 (the groups it samples in phase 2) and its slot s = 16 m + r holds value
// v = 27 a + 3 tap + comp of group 2 a + h (slots 108..111 zero): the reference channel of (group g,
// tap k) is offset dy g*18 + 2k, dx g*18 + 2k + 1, mask 144 + g*9 + k (dcn_v2.py:134-138,
// dcn_v2_im2col_cuda.cu:160-167).  216 rows in 7 M-tiles (224).
int dcnsep_src_row(int m, int i) {
  const int hh = (i >> 2) & 1, r = (i & 3) + 4 * (i >> 3), v = 16 * m + r;
  if (v >= 108) return -1;
  const int g = 2 * (v / 27) + hh, tap = (v % 27) / 3, comp = v % 3;
  return comp == 0 ? g * 18 + 2 * tap : (comp == 1 ? g * 18 + 2 * tap + 1 : 144 + g * 9 + tap);
}
int pack_dcnsep_f16x3(const float* w, const float* b, int cout, int cin, int ks, float* w_dst, float* b_dst) {
  if (cout != 216 || cin != 64 || ks != 3)
    return stif_fail(STIF_E_INVALID, "STIF_PACK_DCNSEP packing needs the 64 -> 216 3x3 conv_offset_mask weight");
  for (size_t i = 0; i < (size_t)cout * cin * 9; ++i)
    if (!f16x3_ok(w[i])) return range_fail("stif_pack_conv_weight: a weight is outside the f16x3 range (|w| < 64); pack it without STIF_PACK_F16X3");
  _Float16* dst = reinterpret_cast<_Float16*>(w_dst);
  for (int k = 0; k < 36; ++k)
    for (int m = 0; m < 7; ++m)
      for (int l = 0; l < 64; ++l) {
        const int src = dcnsep_src_row(m, l & 31), c = k / 9, t = k % 9;
        for (int e = 0; e < 8; ++e) {
          const int ci = 16 * c + 8 * (l >> 5) + e;
          const double x = src >= 0 ? (double)w[((size_t)src * cin + ci) * 9 + t] : 0.0;
          const size_t o = (((size_t)k * 7 + m) * 2) * 512 + l * 8 + e;
          split_f16x3_host(x, dst + o, dst + o + 512);
        }
      }
  if (b_dst)
    for (int m = 0; m < 8; ++m)
      for (int i = 0; i < 32; ++i) {
        const int src = m < 7 ? dcnsep_src_row(m, i) : -1;
        b_dst[m * 32 + i] = (src >= 0 && b) ? b[src] : 0.f;
      }
  return STIF_OK;
}
// DCNPAIR | F16X3: the DCN weight (64 x 64 x 3 x 3) for k_dcn_sep's phase 2, which contracts two
// deformable groups per K step: [group pair a 4][tap 9][nt 2][plane][lane][8 halves], element e of lane l
// holding input channel 8 (2 a + (l >> 5)) + e at `tap`, cout nt * 32 + (l & 31)
int pack_dcnpair_f16x3(const float* w, const float* b, int cout, int cin, int ks, float* w_dst, float* b_dst) {
  if (cout != 64 || cin != 64 || ks != 3)
    return stif_fail(STIF_E_INVALID, "STIF_PACK_DCNPAIR packing needs a 64 -> 64 3x3 weight");
  for (size_t i = 0; i < (size_t)cout * cin * 9; ++i)
    if (!f16x3_ok(w[i])) return range_fail("stif_pack_conv_weight: a weight is outside the f16x3 range (|w| < 64); pack it without STIF_PACK_F16X3");
  _Float16* dst = reinterpret_cast<_Float16*>(w_dst);
  for (int a = 0; a < 4; ++a)
    for (int t = 0; t < 9; ++t)
      for (int nt = 0; nt < 2; ++nt)
        for (int l = 0; l < 64; ++l)
          for (int e = 0; e < 8; ++e) {
            const int ci = 8 * (2 * a + (l >> 5)) + e, co = nt * 32 + (l & 31);
            const size_t o = ((((size_t)a * 9 + t) * 2 + nt) * 2) * 512 + l * 8 + e;
            split_f16x3_host((double)w[((size_t)co * cin + ci) * 9 + t], dst + o, dst + o + 512);
          }
  if (b_dst)
    for (int j = 0; j < cout; ++j) b_dst[j] = b ? b[j] : 0.f;
  return STIF_OK;
}
}  // namespace

extern "C" int stif_pack_conv_weight(const float* w, const float* b, int cout, int cin, int ks, int mode,
                                     float* w_dst, float* b_dst) {
  if (!w || !w_dst || cout <= 0 || cin <= 0 || cin % 8 || (ks != 1 && ks != 3))
    return stif_fail(STIF_E_INVALID, "stif_pack_conv_weight: bad arguments");
  const bool f16x3 = (mode & STIF_PACK_F16X3) != 0;
  mode &= ~STIF_PACK_F16X3;
  if (mode == STIF_PACK_DCNSEP) {
    if (!f16x3) return stif_fail(STIF_E_INVALID, "STIF_PACK_DCNSEP exists for split-fp16 operands only (| STIF_PACK_F16X3)");
    return pack_dcnsep_f16x3(w, b, cout, cin, ks, w_dst, b_dst);
  }
  if (mode == STIF_PACK_DCNPAIR) {
    if (!f16x3) return stif_fail(STIF_E_INVALID, "STIF_PACK_DCNPAIR exists for split-fp16 operands only (| STIF_PACK_F16X3)");
    return pack_dcnpair_f16x3(w, b, cout, cin, ks, w_dst, b_dst);
  }
  if ((mode == STIF_PACK_OFFMASK || mode == STIF_PACK_WINO_OFFMASK) && cout != 216)
    return stif_fail(STIF_E_INVALID, "offmask pack needs cout=216");
  if ((mode == STIF_PACK_LSTM || mode == STIF_PACK_WINO_LSTM) && cout != 256)
    return stif_fail(STIF_E_INVALID, "lstm pack needs cout=256");
  if (mode == STIF_PACK_WINO || mode == STIF_PACK_WINO_OFFMASK || mode == STIF_PACK_WINO_LSTM) {
    if (ks != 3) return stif_fail(STIF_E_INVALID, "winograd pack needs a 3x3 kernel");
    const int perm = mode == STIF_PACK_WINO ? STIF_PACK_PLAIN : (mode == STIF_PACK_WINO_OFFMASK ? STIF_PACK_OFFMASK : mode);
    return f16x3 ? pack_wino_f16x3(w, b, cout, cin, perm, w_dst, b_dst) : pack_wino(w, b, cout, cin, perm, w_dst, b_dst);
  }
  if (f16x3 && mode == STIF_PACK_PLAIN && ks == 1) return pack_1x1_f16x3(w, b, cout, cin, w_dst, b_dst);
  if (f16x3 && mode == STIF_PACK_PLAIN) {
    if (ks != 3 || cout != 64 || cin != 64)
      return stif_fail(STIF_E_INVALID, "PLAIN | F16X3 (DCN core) packing needs a 64 -> 64 3x3 weight");
    return pack_dcn_f16x3(w, b, cout, cin, w_dst, b_dst);
  }
  if (f16x3) return stif_fail(STIF_E_INVALID, "STIF_PACK_F16X3 applies to the Winograd and DCN packings only");
  // layout [slice][chunk][tap][nt][lane][4]: the B fragments of one (slice, chunk) are one
  // contiguous block, copied to LDS by LDS-DMA; lane l of N-tile nt holds cout
  // slice*NJ + nt*32 + (l & 31), input channels chunk*8 + 4*(l >> 5) + e.
  const int NT = slice_tiles(mode), NJ = 32 * NT, cp = cout_padded(cout, mode), T2 = ks * ks, NC = cin / 8;
  const int NS = cp / NJ;
  for (int s = 0; s < NS; ++s)
    for (int c = 0; c < NC; ++c)
      for (int t = 0; t < T2; ++t)
        for (int nt = 0; nt < NT; ++nt)
          for (int l = 0; l < 64; ++l) {
            const int j = s * NJ + nt * 32 + (l & 31);
            const int sr = src_row(j, cout, mode);
            for (int e = 0; e < 4; ++e) {
              const int ci = c * 8 + 4 * (l >> 5) + e;
              w_dst[(((((size_t)s * NC + c) * T2 + t) * NT + nt) * 64 + l) * 4 + e] =
                  sr < 0 ? 0.f : w[((size_t)sr * cin + ci) * T2 + t];
            }
          }
  if (b_dst)
    for (int j = 0; j < cp; ++j) {
      const int sr = src_row(j, cout, mode);
      b_dst[j] = (sr < 0 || !b) ? 0.f : b[sr];
    }
  return STIF_OK;
}

extern "C" size_t stif_dec_proj_floats(void) { return stif_conv_weight_floats(256, stif_dec::SRC_C, 1, STIF_PACK_PLAIN); }

extern "C" int stif_pack_dec_proj_ex(const float* feat_w0, const float* feat_b0, const float* flow_w0,
                                     const float* enc_w0, int lr_image, float* w_dst, float* b_dst);

extern "C" int stif_pack_dec_proj(const float* feat_w0, const float* feat_b0, const float* flow_w0,
                                  const float* enc_w0, float* w_dst, float* b_dst) {
  return stif_pack_dec_proj_ex(feat_w0, feat_b0, flow_w0, enc_w0, 1, w_dst, b_dst);
}

// lr_image = 0 (decoding_test): P2..P4 leave the image columns out -- the flow / encode stages then
// sample the x4-upsampled frames themselves (stif_dec_image); P1 always folds the nearest LR image.
extern "C" int stif_pack_dec_proj_ex(const float* feat_w0, const float* feat_b0, const float* flow_w0,
                                     const float* enc_w0, int lr_image, float* w_dst, float* b_dst) {
  // P1 = feat_imnet.net.0 on [q_feat(192) | q_inp(6)] + bias        (Sakuya_arch_test.py:399)
  // P2 = flow_imnet.net.0 on [q_feat0(192) | q_inp(6)]             (:418, input cols 64..261)
  // P3 = encode_imnet.net.0 on [q_feat3(192) | q_img1(6)]          (:455, cols 128..319, 512..517)
  // P4 = encode_imnet.net.0 on [q_feat4(192) | q_img2(6)]          (cols 320..511, 518..523)
  if (!feat_w0 || !feat_b0 || !flow_w0 || !enc_w0 || !w_dst || !b_dst)
    return stif_fail(STIF_E_INVALID, "stif_pack_dec_proj: null");
  const int C = stif_dec::SRC_C;
  std::vector<float> W((size_t)256 * C, 0.f), B(256, 0.f);
  // first layers are sine layers: omega_0-scaled (see stif_pack_dec_mlp)
  const bool rev = (lr_image & STIF_DEC_REVOLUTIONS) != 0;
  const std::vector<float> fw = omega(feat_w0, 64 * 201, rev), fb = omega(feat_b0, 64, rev),
                           lw = omega(flow_w0, 64 * 263, rev), ew = omega(enc_w0, 64 * 525, rev);
  feat_w0 = fw.data();
  feat_b0 = fb.data();
  flow_w0 = lw.data();
  enc_w0 = ew.data();
  for (int o = 0; o < 64; ++o) {
    for (int c = 0; c < 198; ++c) {
      W[(size_t)o * C + c] = feat_w0[(size_t)o * 201 + c];
      if (c < 192 || (lr_image & 1)) W[(size_t)(64 + o) * C + c] = flow_w0[(size_t)o * 263 + 64 + c];
    }
    for (int c = 0; c < 192; ++c) {
      W[(size_t)(128 + o) * C + c] = enc_w0[(size_t)o * 525 + 128 + c];
      W[(size_t)(192 + o) * C + c] = enc_w0[(size_t)o * 525 + 320 + c];
    }
    for (int c = 0; c < 6 && (lr_image & 1); ++c) {
      W[(size_t)(128 + o) * C + 192 + c] = enc_w0[(size_t)o * 525 + 512 + c];
      W[(size_t)(192 + o) * C + 192 + c] = enc_w0[(size_t)o * 525 + 518 + c];
    }
    B[o] = feat_b0[o];
  }
  return stif_pack_conv_weight(W.data(), B.data(), 256, C, 1, STIF_PACK_PLAIN | (lr_image & STIF_PACK_F16X3), w_dst,
                               b_dst);
}

extern "C" size_t stif_dec_mlp_floats(void) { return stif_dec::MLP_FLOATS; }



namespace {
bool tile_f16x3_ok(const float* t) {
  for (int i = 0; i < stif_dec::T; ++i)
    if (!f16x3_ok(t[i])) return false;
  return true;
}

// fp32 tile [v][lane][4] -> split-fp16 tile [m][plane][lane][8 halves] in place (x 2^10): element
// (m, e) of a lane = fp32 element (v = 2m + (e >> 2), e & 3), i.e. feature F(8m + e, lane >> 5)
void tile_to_f16x3(float* t) {
  std::vector<float> src(t, t + stif_dec::T);
  _Float16* dst = reinterpret_cast<_Float16*>(t);
  for (int m = 0; m < 2; ++m)
    for (int l = 0; l < 64; ++l)
      for (int e = 0; e < 8; ++e) {
        const double x = src[((2 * m + (e >> 2)) * 64 + l) * 4 + (e & 3)];
        const size_t o = ((size_t)(2 * m) * 64 + l) * 8 + e;
        split_f16x3_host(x, dst + o, dst + o + 512);
      }
}
// fp32 tile [v][lane][4] -> the 16x16x32 split-fp16 tile of k_dec2q (dec_layout.h Q_*) at dst: element
// (s, e) of lane l = W[16 s + (l & 15)][16 (e >> 2) + 4 (l >> 4) + (e & 3)], read from the fp32 tile where
// row r, column c sits at lane r + 32 ((c >> 2) & 1), register (c & 3) + 4 (c >> 3)
void tile_to_q16(const float* src, float* t) {
  _Float16* dst = reinterpret_cast<_Float16*>(t);
  for (int s = 0; s < 2; ++s)
    for (int l = 0; l < 64; ++l)
      for (int e = 0; e < 8; ++e) {
        const int row = 16 * s + (l & 15), col = 16 * (e >> 2) + 4 * (l >> 4) + (e & 3);
        const int r = (col & 3) + 4 * (col >> 3);
        const double x = src[((r >> 2) * 64 + row + 32 * ((col >> 2) & 1)) * 4 + (r & 3)];
        const size_t o = ((size_t)(2 * s) * 64 + l) * 8 + e;
        split_f16x3_host(x, dst + o, dst + o + 512);
      }
}
}  // namespace

extern "C" int stif_pack_dec_mlp(const float* const* f, const float* const* l, const float* const* e, float* d) {
  return stif_pack_dec_mlp_ex(f, l, e, d, 0);
}

extern "C" int stif_pack_dec_mlp_ex(const float* const* f, const float* const* l, const float* const* e, float* d,
                                    int flags) {
  using namespace stif_dec;
  if (!f || !l || !e || !d) return stif_fail(STIF_E_INVALID, "stif_pack_dec_mlp: null");
  for (int i = 0; i < 8; ++i)
    if (!f[i] || !l[i]) return stif_fail(STIF_E_INVALID, "stif_pack_dec_mlp: null layer");
  for (int i = 0; i < 10; ++i)
    if (!e[i]) return stif_fail(STIF_E_INVALID, "stif_pack_dec_mlp: null layer");
  memset(d, 0, sizeof(float) * MLP_FLOATS);
  // omega_0-scaled copies of the sine layers (all but the last, linear, layer of each MLP)
  std::vector<float> fs[6], ls[6], es[8];
  const size_t fn[6] = {64 * 201, 64, 64 * 64, 64, 256 * 64, 256};
  const size_t ln[6] = {64 * 263, 64, 64 * 64, 64, 256 * 64, 256};
  const size_t en[8] = {64 * 525, 64, 64 * 64, 64, 256 * 64, 256, 256 * 256, 256};
  const float* F[8];
  const float* Lw[8];
  const float* E[10];
  for (int i = 0; i < 6; ++i) {
    fs[i] = omega(f[i], fn[i], flags & STIF_CONV_F16X3);
    ls[i] = omega(l[i], ln[i], flags & STIF_CONV_F16X3);
    F[i] = fs[i].data();
    Lw[i] = ls[i].data();
  }
  for (int i = 0; i < 8; ++i) {
    es[i] = omega(e[i], en[i], flags & STIF_CONV_F16X3);
    E[i] = es[i].data();
  }
  F[6] = f[6]; F[7] = f[7];
  Lw[6] = l[6]; Lw[7] = l[7];
  E[8] = e[8]; E[9] = e[9];
  f = F;
  l = Lw;
  e = E;
  // feat_imnet: f = {w0[64x201], b0, w1[64x64], b1, w2[256x64], b2, w3[64x256], b3}
  column(d + F_WRY, f[0], 201, 64, 198);
  column(d + F_WRX, f[0], 201, 64, 199);
  column(d + F_WT, f[0], 201, 64, 200);
  pack_tiles(d + F_W1, f[2], 64, 0, 0, 64, 64);
  copy_vec(d + F_B1, f[3], 64, 64);
  pack_tiles(d + F_W2, f[4], 64, 0, 0, 256, 64);
  copy_vec(d + F_B2, f[5], 256, 256);
  pack_tiles(d + F_W3, f[6], 256, 0, 0, 64, 256);
  copy_vec(d + F_B3, f[7], 64, 64);
  // flow_imnet: l = {w0[64x263], b0, w1[64x64], b1, w2[256x64], b2, w3[4x256], b3}
  pack_tiles(d + L_W0, l[0], 263, 0, 0, 64, 64);
  column(d + L_WT, l[0], 263, 64, 262);
  copy_vec(d + L_B0, l[1], 64, 64);
  pack_tiles(d + L_W1, l[2], 64, 0, 0, 64, 64);
  copy_vec(d + L_B1, l[3], 64, 64);
  pack_tiles(d + L_W2, l[4], 64, 0, 0, 256, 64);
  copy_vec(d + L_B2, l[5], 256, 256);
  pack_tiles(d + L_W3, l[6], 256, 0, 0, 4, 256);
  copy_vec(d + L_B3, l[7], 4, 32);
  // encode_imnet: e = {w0[64x525], b0, w1[64x64], b1, w2[256x64], b2, w3[256x256], b3, w4[3x256], b4}
  pack_tiles(d + E_W0, e[0], 525, 0, 0, 64, 128);
  column(d + E_WT, e[0], 525, 64, 524);
  copy_vec(d + E_B0, e[1], 64, 64);
  pack_tiles(d + E_W1, e[2], 64, 0, 0, 64, 64);
  copy_vec(d + E_B1, e[3], 64, 64);
  pack_tiles(d + E_W2, e[4], 64, 0, 0, 256, 64);
  copy_vec(d + E_B2, e[5], 256, 256);
  pack_tiles(d + E_W3, e[6], 256, 0, 0, 256, 256);
  copy_vec(d + E_B3, e[7], 256, 256);
  pack_tiles(d + E_W4, e[8], 256, 0, 0, 3, 256);
  copy_vec(d + E_B4, e[9], 3, 32);
  // image columns for the high-resolution-image decoder (decoding_test)
  pack_tiles(d + I_L, l[0], 263, 0, 256, 64, 6);
  pack_tiles(d + I_E1, e[0], 525, 0, 512, 64, 6);
  pack_tiles(d + I_E2, e[0], 525, 0, 518, 64, 6);
  // plain last layers for the VALU dot products
  memcpy(d + L_W3V, l[6], sizeof(float) * 4 * 256);
  memcpy(d + E_W4V, e[8], sizeof(float) * 3 * 256);
  memcpy(d + E_W4V_B3, d + E_B3, sizeof(float) * 256);   // layer-3 biases beside W4 (one LDS-DMA tile)
  if (flags & STIF_CONV_F16X3) {
    // every MFMA weight tile split; the fp32 image tiles (img_mma) scaled to the accumulators' 2^14
    const int regions[][2] = {{F_W1, 4}, {F_W2, 16}, {F_W3, 16}, {L_W0, 4}, {L_W1, 4}, {L_W2, 16}, {L_W3, 8},
                              {E_W0, 8}, {E_W1, 4}, {E_W2, 16}, {E_W3, 64}, {E_W4, 8}};
    // sine-layer tiles carry omega_0 = 30: their reference weights must stay below 64 / 30
    for (const auto& r : regions)
      for (int k = 0; k < r[1]; ++k)
        if (!tile_f16x3_ok(d + r[0] + k * T))
          return range_fail("stif_pack_dec_mlp_ex: a SIREN weight (times omega_0 for sine layers) is outside the f16x3 range (|w| < 64); pack with flags = 0");
    // k_dec2q's copies of encode_imnet's tiles, from the fp32 tiles before they are split in place
    const int qregions[][3] = {{E_W0, Q_W0, 8}, {E_W1, Q_W1, 4}, {E_W2, Q_W2, 16}, {E_W3, Q_W3, 64}};
    for (const auto& r : qregions)
      for (int k = 0; k < r[2]; ++k) tile_to_q16(d + r[0] + k * T, d + r[1] + k * T);
    for (const auto& r : regions)
      for (int k = 0; k < r[1]; ++k) tile_to_f16x3(d + r[0] + k * T);
    for (int i = I_L; i < I_END; ++i) d[i] *= 16384.f;
  }
  return STIF_OK;
}
