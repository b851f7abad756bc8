// Shared device helpers for the STIF gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define STIF_DEV __device__ __forceinline__

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// v_mfma_f32_32x32x2_f32: D[32x32] += A[32x2] * B[2x32].
// lane l supplies A[i = l&31][k = l>>5] and B[k = l>>5][j = l&31];
// D/C: 16 regs, col = l&31, row = (r&3) + 8*(r>>2) + 4*(l>>5).
STIF_DEV f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// v_mfma_f32_32x32x16_f16: D[32x32] += A[32x16] * B[16x32]; lane l supplies 8 K values of row
// (A) / column (B) l & 31, selected by (l >> 5, element) -- the same selection for A and B, so any
// consistent (lane half, element) -> input-channel assignment is a valid K order.  D as mfma32.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
STIF_DEV f32x16 mfma16h(f16x8 a, f16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
STIF_DEV f16x8 ldh8(const float* p) { return __builtin_bit_cast(f16x8, *reinterpret_cast<const f32x4*>(p)); }

// fp32 products on fp16 MFMA by operand splitting (Markidis et al. 2018; Ootomo & Yokota 2022):
// x * 2^s = h + l with h = fp16(x * 2^s) (RNE) and l = fp16(x * 2^s - h) (the residual is exact in
// fp32, then rounded to 11 bits), so x is carried to ~22 significant bits; a * b is accumulated as
// ah*bh + ah*bl + al*bh in one fp32 accumulator (al*bl < 2^-22 |ab| dropped).  Scales: activations
// (A) 2^4, weights (B, host packing) 2^10 -- the residual l stays a normal fp16 for |x| >= 2^-3
// (A) / 2^-9 (B); below that its absolute error is < 2^-29 (A), 2^-35 (B).  Range: |A| < 4096
// (Winograd-transformed inputs: |activation| < 1024), |B| < 64.  Result unscaled by 2^-14.
#define F16X3_SCALE_A 16.0f
#define F16X3_UNSCALE 0x1p-14f
STIF_DEV void split_f16x3(f32x4 x0, f32x4 x1, f16x8& h, f16x8& l) {
  // per pair (x, y): h = fp16(x * 2^4), fp16(y * 2^4); l = fp16(fma(x, 2^4, -h.lo)), ... -- all four
  // as v_fma_mix{lo,hi}_f16 (fp32 multiply-add, fp16 operand read directly, fp16 result).  x * 2^4 - h
  // is exact in fp32, so l equals fp16(x * 2^4 - float(h)) bit for bit, at 4 VALU ops per pair
  // instead of ~7 (the compiler's lowering of the plain expression scales, converts h back to fp32
  // and subtracts separately)
#if STIF_SPLIT_C
  // plain-expression form (diagnostic): the compiler sees the VALU ops, so its hazard recognizer covers them
  const f32x4 s0 = x0 * F16X3_SCALE_A, s1 = x1 * F16X3_SCALE_A;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float v = e < 4 ? s0[e] : s1[e - 4];
    const _Float16 hh = (_Float16)v;
    h[e] = hh;
    l[e] = (_Float16)(v - (float)hh);
  }
  return;
#endif
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  u32x4 hv, lv;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float x = e < 2 ? x0[2 * e] : x1[2 * e - 4];
    const float y = e < 2 ? x0[2 * e + 1] : x1[2 * e - 3];
    unsigned hp, lp;
    asm(
#if STIF_SPLIT_NOP_PRE
        "s_nop 7\n\ts_nop 7\n\t"
#endif
        "v_fma_mixlo_f16 %0, %2, %4, 0\n\t"
        "v_fma_mixhi_f16 %0, %3, %4, 0\n\t"
        "v_fma_mixlo_f16 %1, %2, %4, -%0 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %1, %3, %4, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
#if STIF_SPLIT_NOP
        "\n\ts_nop 4"
#endif
        : "=&v"(hp), "=&v"(lp)
        : "v"(x), "v"(y), "s"(F16X3_SCALE_A));
    hv[e] = hp;
    lv[e] = lp;
  }
  h = __builtin_bit_cast(f16x8, hv);
  l = __builtin_bit_cast(f16x8, lv);
}

// f16x3 operand-range report.  An operand outside the split range (|A * 2^4| > 65504) becomes an fp16
// infinity, and every product it enters turns into inf or NaN (h = inf, l = -inf: inf - inf), so the
// outputs it feeds are not finite.  The kernels test their pre-activation outputs with this and set
// the caller's optional status word (a plain vector store; concurrent writers all store 1).
STIF_DEV bool not_finite(float x) { return !(__builtin_fabsf(x) <= 3.40282347e38f); }
STIF_DEV void report_range(int* status, bool bad) {
  if (status != nullptr && bad) *status = 1;
}

STIF_DEV int mfma_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

STIF_DEV f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
STIF_DEV void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }

STIF_DEV float lrelu01(float x) { return x >= 0.f ? x : x * 0.1f; }
STIF_DEV float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }
// 1 / (1 + 2^(-x log2 e)) with v_exp_f32 and v_rcp_f32 (each ~1 ulp): ~3e-7 relative
STIF_DEV float sigmoid_fast(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -1.44269504088896341f));
}

enum { STIF_ACT_NONE = 0, STIF_ACT_LRELU = 1, STIF_ACT_RELU = 2, STIF_ACT_RES = 3,
       STIF_ACT_OFFMASK = 4, STIF_ACT_LSTM = 5 };

// sin(2 pi x) for pre-activations in revolutions (the f16x3 decoder: omega_0 / (2 pi) is folded into
// the packed sine-layer weights, stif_pack_dec_mlp_ex): x - rint(x) is exact, so the one rounding of
// the reduction is the fp32 accumulation of x itself, as for a pre-activation in radians; then the
// hardware v_sin_f32 on [-1/2, 1/2] revolutions (~4e-7 absolute, tools/experiments/sin_acc.hip).
// 2 VALU + one transcendental (8 issue cycles): the SIREN decoder is VALU-issue-bound and evaluates one
// sine per hidden unit.  Used instead of ocml sinf, whose Payne-Hanek path costs ~200 VGPRs in the MLP
// kernels.
STIF_DEV float stif_sin_rev(float x) { return __builtin_amdgcn_sinf(x - __builtin_rintf(x)); }

// sin(x) for the fp32-operand decoder (F16 = 0, the fp32 re-run the range guard promises): quadrant
// reduction by pi/2 (q = rint(x 2/pi), 3-part Cody-Waite constant, exact products for |q| < 2^12,
// i.e. |x| < 6400) and minimax-free Taylor polynomials on [-pi/4, pi/4] through r^9 (sin) / r^8 (cos):
// ~1e-7 absolute, the accuracy of the reference's torch.sin within a few ulp; ~20 VALU, no
// transcendental.  The f16x3 decoder uses the faster stif_sin_rev above.
__host__ __device__ __forceinline__ float stif_sin_poly(float x) {
  const float qm = fmaf(x, 0.636619772367581343076f, 12582912.0f);   // round(x * 2/pi) by the magic add
  const float q = qm - 12582912.0f;
  float r = fmaf(q, -1.5703125f, x);                                   // pi/2 = P1 + P2 + P3, P1 8 bits
  r = fmaf(q, -4.837512969970703125e-4f, r);
  r = fmaf(q, -7.54978995489188216e-8f, r);
  const float s = r * r;
  const float ps = fmaf(fmaf(fmaf(fmaf(s, 2.75573192e-6f, -1.98412698e-4f), s, 8.33333333e-3f), s, -1.66666667e-1f) * s, r, r);
  const float pc = fmaf(fmaf(fmaf(fmaf(s, 2.48015873e-5f, -1.38888889e-3f), s, 4.16666667e-2f), s, -0.5f), s, 1.0f);
  const int qi = (int)q;
  const float v = (qi & 1) ? pc : ps;
  return (qi & 2) ? -v : v;
}
// The hardware sine reduces its argument itself, exactly: v_sin_f32 of x and of x - rint(x) have the same
// maximum error against sin(2 pi x) -- 1.1-1.3e-7 in every band from |x| <= 0.5 to |x| <= 1e7 revolutions, 6-34 %
// of results one ulp apart (tools/r5/vsin_reduce.hip, profiles/r05_sin_raw.log) -- so the f16x3 decoder skips the
// two-instruction reduction (DEC_SIN_RAW = 1).
#ifndef DEC_SIN_RAW
#define DEC_SIN_RAW 1
#endif
template <int F16>
STIF_DEV float siren_sin(float x) {
  if constexpr (F16 && DEC_SIN_RAW) return __builtin_amdgcn_sinf(x);
  else if constexpr (F16) return stif_sin_rev(x);
  else return stif_sin_poly(x);
}

// XCD-aware block order for grids of independent pixel blocks: workgroups are dealt round-robin over
// the 8 XCDs (blocks b and b + 8 share one; each XCD has its own L2), so block b takes logical block
// start(b % 8) + b / 8 -- every XCD walks a contiguous range of blocks, and maps read by neighbouring
// blocks (halos, bilinear gathers) stay in one L2 instead of being fetched by several.  A bijection of
// [0, nb) for any nb; speed only, never correctness.
STIF_DEV int xcd_block(int b, int nb) {
  const int x = b & 7, q = nb >> 3, r = nb & 7;
  return x * q + min(x, r) + (b >> 3);
}

// Epilogue helper: write one 32 px x 32 cout accumulator tile (lane = cout, regs = px) into the
// wave's private 4-KB LDS block as [px][co] with the 16-B slot XOR-swizzled by px & 3 (bank-conflict
// free for both the b32 writes and the b128 row reads), so the global stores become coalesced
// 16-B accesses (8 pixels x 128 B per wave instruction).
STIF_DEV void tile_to_lds(float* blk, const f32x16& v, int lane) {
  const int l32 = lane & 31, hf = lane >> 5;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int px = (r & 3) + 8 * (r >> 2) + 4 * hf;
    blk[px * 32 + (((l32 >> 2) ^ (px & 3)) << 2) + (l32 & 3)] = v[r];
  }
}
STIF_DEV f32x4 lds_row4(const float* blk, int px, int c4) { return ld4(blk + px * 32 + ((c4 ^ (px & 3)) << 2)); }

// Barrier for LDS filled by LDS-DMA (buffer_load/global_load ... lds): the DMA completes
// asynchronously on each wave's vmcnt and gfx950's back-off barrier does not drain it, so every
// wave waits for its own transfers before the workgroup barrier that publishes them.
STIF_DEV void lds_dma_barrier() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}
