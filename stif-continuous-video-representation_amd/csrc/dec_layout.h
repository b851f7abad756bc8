// Packed layout of the implicit-decoder MLP weights (shared by pack.cpp and decoder.hip).
//
// The decoder runs every SIREN layer as D^T = W . X^T on v_mfma_f32_32x32x2_f32 with
// the HR pixel on the lane (j = lane & 31) and features in registers: a 32-feature
// tile lives in 16 accumulator registers, register r of lane half h holding feature
// F(r, h) = (r & 3) + 8 * (r >> 2) + 4 * h.  That register tile is directly the B
// operand of the next layer if the next layer's weights are read in the same K
// order, so one weight tile (32 out x 32 in) is stored as
//   [v = 0..3][lane = 0..63][e = 0..3]  ->  W[32*ot + (lane & 31)][32*kt + F(4v + e, lane >> 5)]
// (1024 floats; each wave-instruction of a float4 load reads 1 KiB contiguously).
#pragma once

namespace stif_dec {

constexpr int T = 1024;  // floats per packed 32x32 weight tile

// feat_imnet (201 -> 64 -> 64 -> 256 -> 64); layer 0's 198 LR inputs live in the projection P1
constexpr int F_WRY = 0, F_WRX = 64, F_WT = 128;
constexpr int F_W1 = 192, F_B1 = F_W1 + 4 * T;
constexpr int F_W2 = F_B1 + 64, F_B2 = F_W2 + 16 * T;
constexpr int F_W3 = F_B2 + 256, F_B3 = F_W3 + 16 * T;
constexpr int F_END = F_B3 + 64;
// flow_imnet (263 -> 64 -> 64 -> 256 -> 4); layer 0: HRfeat part packed, feat/inp part in P2
constexpr int L_W0 = F_END, L_WT = L_W0 + 4 * T, L_B0 = L_WT + 64;
constexpr int L_W1 = L_B0 + 64, L_B1 = L_W1 + 4 * T;
constexpr int L_W2 = L_B1 + 64, L_B2 = L_W2 + 16 * T;
constexpr int L_W3 = L_B2 + 256, L_B3 = L_W3 + 8 * T;
constexpr int L_END = L_B3 + 32;
// encode_imnet (525 -> 64 -> 64 -> 256 -> 256 -> 3); layer 0: q_feat1|q_feat2 packed, rest in P3/P4
constexpr int E_W0 = L_END, E_WT = E_W0 + 8 * T, E_B0 = E_WT + 64;
constexpr int E_W1 = E_B0 + 64, E_B1 = E_W1 + 4 * T;
constexpr int E_W2 = E_B1 + 64, E_B2 = E_W2 + 16 * T;
constexpr int E_W3 = E_B2 + 256, E_B3 = E_W3 + 64 * T;
constexpr int E_W4 = E_B3 + 256, E_B4 = E_W4 + 8 * T;
constexpr int E_END = E_B4 + 32;

// image columns of the first layers as packed 32x32 tiles (K = the 6 image channels, zero padded;
// only used when the flow / encode stages sample a high-resolution image, decoding_test --
// otherwise the LR image lives in P2..P4): 4 MFMAs per output tile with the channels as B operand
constexpr int I_L = E_END;             // flow_imnet.net.0 columns 256..261 (q_inp), 2 tiles
constexpr int I_E1 = I_L + 2 * T;      // encode_imnet.net.0 columns 512..517 (q_img1)
constexpr int I_E2 = I_E1 + 2 * T;     // encode_imnet.net.0 columns 518..523 (q_img2)
constexpr int I_END = I_E2 + 2 * T;

// the two narrow last layers (flow 256 -> 4, rgb 256 -> 3) as plain row-major [out][256] rows: they
// run as per-lane VALU dot products over the lane's 128 features + one cross-half add, instead of
// 128 MFMAs per 32 pixels of which 28/32 (29/32) would multiply zero-padded rows
constexpr int L_W3V = I_END;             // [4][256]
constexpr int E_W4V = L_W3V + 4 * 256;   // [3][256], padded to a whole 4-KB tile (LDS-DMA granule)
constexpr int E_W4V_B3 = E_W4V + 768;    // the pad holds a copy of E_B3 (k_dec2 reads it from LDS)
constexpr int V_END = E_W4V + 1024;

// encode_imnet's MFMA tiles again for the 16-pixel stage 2 (k_dec2q, f16x3 packing only; zero otherwise): the
// same [ot][kt] tile order, each 32x32 tile as two 16-row sub-tiles s of v_mfma_f32_16x16x32_f16 A operands
// [s][plane h|l][lane][8 halves], lane l holding row 16 s + (l & 15) and input feature
// 16 (e >> 2) + 4 (l >> 4) + (e & 3) -- the order in which a 16x16 accumulator pair holds a 32-feature tile
constexpr int Q_W0 = V_END, Q_W1 = Q_W0 + 8 * T, Q_W2 = Q_W1 + 4 * T, Q_W3 = Q_W2 + 16 * T;
constexpr int Q_END = Q_W3 + 64 * T;

constexpr int MLP_FLOATS = Q_END;
constexpr int IMG_C = 8;      // high-resolution image channels: rgb0 rgb1 + 2 zero (16-B aligned pixels)
constexpr int PROJ_C = 256;   // LR projection channels: P1 | P2 | P3 | P4
constexpr int SRC_C = 200;    // LR source channels: feat t0|t1|t2 (192) + rgb0 rgb1 (6) + 2 zero

}  // namespace stif_dec
