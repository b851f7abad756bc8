/*
 * stif.h -- C ABI of libstif_hip.so, the MI355X (gfx950) engine for the STIF
 * LunaTokis forward (reference: codes/models/modules/Sakuya_arch_test.py).
 *
 * Conventions (every entry point):
 *   - plain device pointers (fp32), sizes as ints; no framework types;
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream);
 *   - outputs and workspaces are caller-allocated; nothing allocates per call;
 *   - stateless and reentrant; returns 0 on success or a STIF_E_* code, with a
 *     message retrievable through stif_last_error() (thread-local);
 *   - feature maps are NHWC ([item][y][x][channel]) unless a name says NCHW.
 *
 * The drop-in for the reference's native operator is stif_dcn_v2_forward; it
 * replaces `_ext.dcn_v2_forward` (DCNv2/src/vision.cpp:4, declared
 * DCNv2/src/dcn_v2.h:9-23, CUDA body DCNv2/src/cuda/dcn_v2_cuda.cu:42-172).
 * The remaining entry points are the fused stages the engine's LunaTokis host
 * (stif_amd.model) drives; INTEGRATION.md shows the reference-side bindings.
 */
#ifndef STIF_H
#define STIF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  STIF_OK = 0,
  STIF_E_INVALID = 1,   /* bad argument / unsupported shape */
  STIF_E_LAUNCH = 2,    /* kernel launch failed */
  STIF_E_WORKSPACE = 3, /* workspace too small */
  STIF_E_RANGE = 4      /* STIF_PACK_F16X3 packing: a weight exceeds the split-fp16 range (pack in fp32) */
};

/* activation / epilogue selector of stif_conv2d_nhwc and stif_dcn_nhwc */
enum {
  STIF_EPI_NONE = 0,
  STIF_EPI_LRELU = 1,   /* LeakyReLU(0.1)  (Sakuya_arch_test.py:69) */
  STIF_EPI_RELU = 2,    /* ReLU            (module_util.py:51) */
  STIF_EPI_RES = 3,     /* out = res + conv (ResidualBlock_noBN, module_util.py:48-52) */
  STIF_EPI_OFFMASK = 4, /* sigmoid on the mask channels of a DCN offset/mask conv (dcn_v2.py:134-138) */
  STIF_EPI_LSTM = 5     /* ConvLSTMCell gates (convlstm.py:47-56): out=h_next, out2=c_next, res=c_cur */
};

#define STIF_MAX_GROUPS 8

/* Direct/implicit-GEMM convolution on NHWC fp32 maps (replaces nn.Conv2d in the
 * hot path).  The input is the channel concatenation [in0 | in1] (so torch.cat
 * never materialises); in1 may be read through a fused bilinear x2 upsample
 * (F.interpolate(scale_factor=2, mode='bilinear', align_corners=False) times
 * in1_scale, Sakuya_arch_test.py:86-87).  A launch covers `ngroups` weight sets
 * x `nitems` items per set (item i of set g uses in0[g] + i*in0_item, ...).
 * Weights are packed by stif_pack_conv_weight. */
typedef struct {
  const float* in0[STIF_MAX_GROUPS];
  const float* in1[STIF_MAX_GROUPS];
  const float* w[STIF_MAX_GROUPS];     /* packed, see stif_pack_conv_weight */
  const float* bias[STIF_MAX_GROUPS];  /* [cout_pad], packed order */
  float* out[STIF_MAX_GROUPS];
  const float* res[STIF_MAX_GROUPS];   /* STIF_EPI_RES: residual; STIF_EPI_LSTM: c_cur */
  float* out2[STIF_MAX_GROUPS];        /* STIF_EPI_LSTM: c_next */
  long long in0_item, in1_item, out_item, res_item, out2_item;  /* element strides between items */
  int ngroups, nitems;
  int H, W, C0;            /* in0: H x W x C0, C0 % 8 == 0 */
  int C1, in1_mode;        /* in1_mode: 0 none, 1 same resolution, 2 half resolution + x2 bilinear */
  float in1_scale;
  int Ho, Wo;              /* output resolution */
  int cout;                /* logical output channels (64, 216, 256) */
  int ks, stride;          /* 1 or 3; 1 or 2 (padding = ks/2) */
  int epi;                 /* STIF_EPI_* */
  int flags;               /* STIF_CONV_F16X3: weights packed with STIF_PACK_F16X3 (stif_conv3x3_wino only) */
  int* status;             /* optional device word (NULL = none): with STIF_CONV_F16X3, set to 1 when an output
                              element is not finite before its activation -- the signature of an activation
                              outside the split-fp16 operand range (see STIF_CONV_F16X3) */
  int* sched;              /* device block of 8 ints, zero when first used, read only with flags & STIF_CONV_DYNAMIC
                              (stif_conv3x3_wino, STIF_CONV_F16X3 launches; ignored otherwise, and ignored while the
                              stream is capturing a graph): per-XCD tile counters of the persistent kernel's dynamic
                              schedule.  The library keeps each block's running totals on the host, so the launches
                              that use one block must run in issue order (one stream) and the block must not be
                              freed and re-allocated while the library is loaded.  Outputs are identical either way.
                              Zero-initialise the whole struct: fields added at its end keep their old meaning
                              only when zero. */
} stif_conv_args;

/* stif_conv_args.flags: fp32 products on the fp16 MFMA pipe by 3-term operand splitting (x = h + l,
 * a*b = ah*bh + ah*bl + al*bh, fp32 accumulation; ~22 significant bits per operand, see
 * stif_common.h).  Valid range: |activations| < 1024 (Winograd: |transformed inputs| < 4096),
 * |packed weights| < 64.  Both limits are enforced: the packers return STIF_E_RANGE for a weight
 * outside it, and an activation outside it turns the outputs it feeds into NaN/inf, which the
 * kernels report through the `status` word (the host then re-runs the call in fp32). */
#define STIF_CONV_F16X3 1
/* stif_conv_args.flags: take the persistent Winograd conv's tiles from the per-XCD counters in `sched`
 * (dynamic schedule) instead of the static stride; without this bit `sched` is never read. */
#define STIF_CONV_DYNAMIC 2

int stif_conv2d_nhwc(const stif_conv_args* args, void* stream);

/* The same operator for 3x3 / stride 1 / 'same' shapes by Winograd F(2x2,3x3) on fp32 MFMA
 * (2.25x fewer multiply-adds; all arithmetic fp32): weights packed with STIF_PACK_WINO
 * (epi NONE / LRELU / RELU / RES), STIF_PACK_WINO_OFFMASK (epi OFFMASK, cout 216) or
 * STIF_PACK_WINO_LSTM (epi LSTM, 128 -> 256: out = h_next, out2 = c_next, res = c_cur, 64-ch maps);
 * in1_mode 0 or 1; C0 and C1 multiples of 32. */
int stif_conv3x3_wino(const stif_conv_args* args, void* stream);

/* out = scale * F.interpolate(in, scale_factor=2, mode='bilinear', align_corners=False) on NHWC
 * maps (PCD_Align's coarse-to-fine step, Sakuya_arch_test.py:86-87); in [n][h1][w1][c],
 * out [n][2h1][2w1][c], items `in_item` / `out_item` floats apart, c % 4 == 0. */
int stif_upsample2x_nhwc(const float* in, float* out, int n, int h1, int w1, int c, float scale,
                         long long in_item, long long out_item, void* stream);

/* conv_first (3 -> 64, 3x3) + LeakyReLU, reading NCHW RGB frames [n,3,h,w]
 * (Sakuya_arch_test.py:318) and writing NHWC [n,h,w,64]. w: [64,3,3,3] as in the state dict. */
int stif_conv_first(const float* x_nchw, const float* w, const float* b, float* out,
                    int n, int h, int w_, void* stream);

/* Fused modulated deformable conv (DCN_sep core, 64 -> 64, 3x3, 8 groups):
 * bilinear sampling (dmcn_im2col_bilinear semantics) straight into LDS and an
 * fp32-MFMA contraction; no columns buffer.  offmask is the NHWC output of the
 * offset/mask conv packed with STIF_PACK_OFFMASK (216 channels per pixel,
 * [group][tap][dy, dx, sigmoid(mask)]). */
typedef struct {
  const float* in[STIF_MAX_GROUPS];
  const float* offmask[STIF_MAX_GROUPS];
  const float* w[STIF_MAX_GROUPS];     /* packed like a 64->64 3x3 conv */
  const float* bias[STIF_MAX_GROUPS];
  float* out[STIF_MAX_GROUPS];
  long long in_item, om_item, out_item;
  int ngroups, nitems, H, W;
  int epi;                              /* STIF_EPI_NONE or STIF_EPI_LRELU */
  int flags;                            /* STIF_CONV_F16X3: w packed STIF_PACK_PLAIN | STIF_PACK_F16X3 */
  int* status;                          /* optional device word, as stif_conv_args.status */
} stif_dcn_args;

int stif_dcn_nhwc(const stif_dcn_args* args, void* stream);

/* Fused DCN_sep (dcn_v2.py:127-140) in one launch: conv_offset_mask (64 -> 216, 3x3) + chunk / cat /
 * sigmoid + the modulated deformable conv (64 -> 64, 3x3, 8 groups) -- the offset/mask map never leaves
 * the registers (split-fp16 MFMA only, flags = STIF_CONV_F16X3).  fea: the offset branch's feature
 * (NHWC 64 ch); in: the deformable conv's input (NHWC 64 ch); w_om / b_om: conv_offset_mask packed
 * with STIF_PACK_DCNSEP | STIF_PACK_F16X3; w / bias: the DCN weight packed STIF_PACK_DCNPAIR |
 * STIF_PACK_F16X3.  Replaces the pair conv (STIF_EPI_OFFMASK) -> stif_dcn_nhwc. */
typedef struct {
  const float* fea[STIF_MAX_GROUPS];
  const float* in[STIF_MAX_GROUPS];
  const float* w_om[STIF_MAX_GROUPS];
  const float* b_om[STIF_MAX_GROUPS];
  const float* w[STIF_MAX_GROUPS];
  const float* bias[STIF_MAX_GROUPS];
  float* out[STIF_MAX_GROUPS];
  long long fea_item, in_item, out_item;
  int ngroups, nitems, H, W;
  int epi;                              /* STIF_EPI_NONE or STIF_EPI_LRELU */
  int flags;                            /* STIF_CONV_F16X3 (required) */
  int* status;                          /* optional device word, as stif_conv_args.status */
} stif_dcn_sep_args;

int stif_dcn_sep_nhwc(const stif_dcn_sep_args* args, void* stream);

/* Drop-in for `_ext.dcn_v2_forward` (dcn_v2.h:9-23): NCHW fp32 input [b,c,h,w],
 * weight [co,c,kh,kw], bias [co], offset [b, dg*2*kh*kw, ho, wo],
 * mask [b, dg*kh*kw, ho, wo]; output [b, co, ho, wo] (caller-allocated).
 * Any kernel/stride/pad/dilation/group combination of the reference is
 * accepted.  The STIF shape (c = co = 64, 3x3, stride 1, pad 1, dilation 1, 8 groups: every
 * DCN_sep of LunaTokis) runs the fused im2col-free kernel of stif_dcn_nhwc (fp32 MFMA) between
 * NCHW<->NHWC transposes, with the weights packed on the device -- workspace 344 floats per
 * pixel (the reference's im2col path: 576); every other shape runs im2col + GEMM one sample at a
 * time (workspace c*kh*kw*ho*wo floats, the reference's per-sample `columns`).
 * workspace: at least stif_dcn_v2_workspace_size bytes, 16-B aligned. */
size_t stif_dcn_v2_workspace_size(int batch, int channels, int height, int width, int channels_out,
                                  int kernel_h, int kernel_w, int stride_h, int stride_w, int pad_h,
                                  int pad_w, int dilation_h, int dilation_w, int deformable_group);
int stif_dcn_v2_forward(const float* input, const float* weight, const float* bias,
                        const float* offset, const float* mask, float* output,
                        int batch, int channels, int height, int width, int channels_out,
                        int kernel_h, int kernel_w, int stride_h, int stride_w, int pad_h, int pad_w,
                        int dilation_h, int dilation_w, int deformable_group,
                        void* workspace, size_t workspace_bytes, void* stream);

/* Drop-in for `_ext.dcn_v2_backward` (dcn_v2.h:39-52, vision.cpp:5; CUDA body dcn_v2_cuda.cu:204-335):
 * the same NCHW tensors as stif_dcn_v2_forward plus grad_output [b, co, ho, wo]; writes grad_input
 * [b,c,h,w], grad_offset [b, dg*2*kh*kw, ho, wo], grad_mask [b, dg*kh*kw, ho, wo], grad_weight
 * [co,c,kh,kw] and grad_bias [co] (caller-allocated; all overwritten).  Per sample, as the reference:
 * columns gradient = W^T grad_output (fp32 MFMA GEMM), the coordinate / mask gradients
 * (modulated_deformable_col2im_coord semantics, one thread per group x tap x pixel), the input
 * gradient scattered to the bilinear corners with fp32 atomics (modulated_deformable_col2im), the
 * forward columns and grad_weight += grad_output columns^T, grad_bias += sum grad_output.
 * workspace: at least stif_dcn_v2_backward_workspace_size bytes (c*kh*kw*ho*wo floats), 16-B aligned. */
size_t stif_dcn_v2_backward_workspace_size(int batch, int channels, int height, int width, int channels_out,
                                           int kernel_h, int kernel_w, int stride_h, int stride_w, int pad_h,
                                           int pad_w, int dilation_h, int dilation_w, int deformable_group);
int stif_dcn_v2_backward(const float* input, const float* weight, const float* bias, const float* offset,
                         const float* mask, const float* grad_output, float* grad_input, float* grad_offset,
                         float* grad_mask, float* grad_weight, float* grad_bias, int batch, int channels, int height,
                         int width, int channels_out, int kernel_h, int kernel_w, int stride_h, int stride_w,
                         int pad_h, int pad_w, int dilation_h, int dilation_w, int deformable_group, void* workspace,
                         size_t workspace_bytes, void* stream);

/* ---- implicit decoder (LunaTokis.decoding, Sakuya_arch_test.py:364-459) ---- */

/* Assemble the decoder's LR source map [n,h,w,200] = [feat t0 | t1 | t2 | inp rgb0 rgb1 | 0 0]
 * from the three NHWC latent maps and the NCHW input pair x [n,2,3,h,w]. */
int stif_dec_pack_lr(const float* f0, const float* f1, const float* f2, const float* x_nchw,
                     float* out, int n, int h, int w, void* stream);

/* Per-axis sampling tables of the HR query grid (host-computed, fp32, see
 * stif_amd.coords): for every HR row (then column): nearest LR index, rel
 * coordinate, bilinear LR indices i0/i1, weights w0/w1 (0 if out of range), and
 * the warpgrid linspace base. Layout: struct of arrays, one float/int per entry. */
typedef struct {
  const int* near_y; const float* rel_y; const int* by0; const int* by1; const float* wy0; const float* wy1;
  const float* lin_y;
  const int* near_x; const float* rel_x; const int* bx0; const int* bx1; const float* wx0; const float* wx1;
  const float* lin_x;
  /* optional (NULL = identity): HR pixel whose HRfeat the flow stage reads for a query -- the
   * local ensemble's shifted queries (decoding_localensemble, Sakuya_arch_test.py:1022-1025) */
  const int* hr_y; const int* hr_x;
} stif_dec_tables;

/* Optional high-resolution image for the flow / encode stages (decoding_test samples
 * HRinp = F.upsample(inp, x4, bilinear), Sakuya_arch_test.py:513-514, instead of the LR frames;
 * pack the projection with stif_pack_dec_proj_ex(..., lr_image = 0) then).  img: [n][ih][iw][8]
 * (rgb0 rgb1 0 0, stif_upsample_image); by0..wx1: bilinear rows / columns / weights of the
 * image at every HR query row / column (as in stif_dec_tables). */
typedef struct {
  const float* img;
  int ih, iw;
  const int* by0; const int* by1; const float* wy0; const float* wy1;
  const int* bx0; const int* bx1; const float* wx0; const float* wx1;
} stif_dec_image;

/* Stage 1 (per HR pixel): feat_imnet -> HRfeat [n,HH,WW,64]; flow_imnet -> flow [n,HH,WW,4].
 * proj: [n,h,w,256] LR projections (P1 | P2 | P3 | P4) from stif_conv2d_nhwc (1x1, packed by
 * stif_pack_dec_proj).  mlp: packed by stif_pack_dec_mlp.  t: [n] query time per item. */
int stif_dec_stage1(const float* proj, const float* mlp, const stif_dec_tables* tab, const stif_dec_image* img,
                    const float* t, float* hrfeat, float* flow, int n, int h, int w, int HH, int WW, void* stream);

/* Stage 2 (per HR pixel): warp grids from flow, bilinear HRfeat / projections, encode_imnet
 * -> RGB, written NCHW [n,3,HH,WW] (LunaTokis output layout, unclamped). */
int stif_dec_stage2(const float* proj, const float* mlp, const float* hrfeat, const float* flow,
                    const stif_dec_tables* tab, const stif_dec_image* img, const float* t, float* out_nchw,
                    int n, int h, int w, int HH, int WW, void* stream);
/* The same stages with flags = STIF_CONV_F16X3: every SIREN layer on split-fp16 MFMA (mlp packed by
 * stif_pack_dec_mlp_ex with the same flag); flags = 0 is stif_dec_stage1 / stif_dec_stage2.
 * status: optional device word (NULL = none), set to 1 by stage 2 in f16x3 mode when an RGB output or
 * the stage-1 flow it reads is not finite (an HRfeat / hidden activation outside the split range
 * propagates to the RGB; a flow_imnet one to the flow, which the warpgrid clamp would otherwise turn
 * into a finite grid). */
int stif_dec_stage1_ex(const float* proj, const float* mlp, const stif_dec_tables* tab, const stif_dec_image* img,
                       const float* t, float* hrfeat, float* flow, int n, int h, int w, int HH, int WW, int flags,
                       int* status, void* stream);
int stif_dec_stage2_ex(const float* proj, const float* mlp, const float* hrfeat, const float* flow,
                       const stif_dec_tables* tab, const stif_dec_image* img, const float* t, float* out, int n, int h,
                       int w, int HH, int WW, int flags, int* status, void* stream);

/* out = sum_k pred_k * wgt_k (per HR pixel weights [HH*WW], shared by the n items): the
 * local ensemble's area blend (Sakuya_arch_test.py:1076-1084). pred_k / out: [n][3][HH][WW]. */
int stif_dec_blend4(const float* const* pred, const float* const* wgt, float* out, int n, int HH, int WW,
                    void* stream);

/* HRinp for decoding_test: F.upsample(x, scale_factor=s, mode='bilinear') (align_corners=False)
 * of the NCHW pair x [n][2][3][h][w] as NHWC [n][s*h][s*w][8] (rgb0 rgb1 0 0). */
int stif_upsample_image(const float* x_nchw, float* out, int n, int h, int w, int s, void* stream);

/* ---- video harness I/O (custom_video_test.py:88-103) ---- */

/* data.util.imresize_np(frame, scale, antialiasing) of nf cv2-style uint8 BGR HWC frames [nf][H][W][3]
 * (separable cubic, symmetric padding; data/util.py:302-371), written as the model input: RGB NCHW
 * float / 255 [nf][3][oH][oW].  wH [oH][PH], iH [oH] (first symmetric-padded row), sH (top padding)
 * and the W equivalents come from calculate_weights_indices (stif_amd.video.resize_tables). */
int stif_resize_frames(const unsigned char* bgr, float* out_rgb_nchw, int nf, int H, int W, int oH, int oW,
                       const float* wH, const int* iH, int PH, int sH, const float* wW, const int* iW, int PW, int sW,
                       void* stream);
/* (clamp(x, 0, 1) * 255).astype(uint8) of NCHW RGB frames [n][3][H][W] -> HWC uint8 [n][H][W][3]. */
int stif_frames_to_u8(const float* nchw, unsigned char* hwc, int n, int H, int W, void* stream);

/* ---- host-side weight packing (pure CPU, callable without a GPU) ---- */
enum { STIF_PACK_PLAIN = 0, STIF_PACK_OFFMASK = 1, STIF_PACK_LSTM = 2, STIF_PACK_WINO = 3, STIF_PACK_WINO_OFFMASK = 4,
       STIF_PACK_WINO_LSTM = 5, STIF_PACK_DCNSEP = 6, STIF_PACK_DCNPAIR = 7 };
/* OR'ed into a STIF_PACK_WINO* mode: the f16x3 split packing for stif_conv3x3_wino with
 * flags = STIF_CONV_F16X3 (same size in bytes) */
#define STIF_PACK_F16X3 16

/* Size in floats of a packed conv weight / bias for a packing mode. */
size_t stif_conv_weight_floats(int cout, int cin, int ks, int mode);
size_t stif_conv_bias_floats(int cout, int mode);
/* w_oihw: [cout][cin][ks][ks] (nn.Conv2d layout).  dst layout:
 * [slice][cin/8][ks*ks][nt][lane 64][4] -- the MFMA B fragments of one (slice, 8-channel chunk),
 * contiguous so the kernel copies them to LDS with LDS-DMA; a slice is 32*NT output channels
 * (NT = 7 for OFFMASK, 4 for LSTM, 2 otherwise), cout padded to a whole slice with zeros, and
 * output rows permuted per `mode` (OFFMASK: [group][tap][dy, dx, mask]; LSTM: gates i,f,o,g
 * of 32 hidden channels per slice).
 * STIF_PACK_WINO (3x3 only, for stif_conv3x3_wino): the Winograd-domain weights U = G g G^T
 * (F(2x2,3x3), computed in double) as [cout/64][cin/8][i 4][j 4][nt 2][lane 64][4], lane l of
 * (i, j, nt) holding U[i][j] of cout slice*64 + nt*32 + (l & 31), input channel
 * chunk*8 + 4(l >> 5) + e; cout padded to a multiple of 64.  STIF_PACK_WINO_OFFMASK: the same
 * with the OFFMASK row permutation (216 -> 256 rows).  STIF_PACK_WINO_LSTM: the same for the
 * ConvLSTMCell conv (128 -> 256) with packed cout 4h + gate = reference row gate*64 + h (gates
 * i, f, o, g; convlstm.py:49), so one 4-cout quad holds the four gates of hidden channel h.
 * STIF_PACK_WINO* | STIF_PACK_F16X3: U * 2^10 split into fp16 h = rne(U 2^10), l = rne(U 2^10 - h)
 * as [cout/64][cin/16][i 4][j 4][nt 2][plane h|l][lane 64][8 halves], lane l's element e holding
 * input channel 16 q + 8 (e >> 2) + 4 (l >> 5) + (e & 3) (the chunk pair of one f16 MFMA).
 * STIF_PACK_PLAIN | STIF_PACK_F16X3 (64 -> 64 3x3 only: the stif_dcn_nhwc core, and the 3x3
 * stride-2 convs of stif_conv2d_nhwc, with flags = STIF_CONV_F16X3): [group 8][tap pair 5][nt 2][plane h|l][lane 64][8 halves], element e
 * of lane l holding tap 2p + (l >> 5) (tap 9 = 0), input channel 8 group + e.
 * STIF_PACK_DCNSEP | STIF_PACK_F16X3 (conv_offset_mask 64 -> 216, 3x3, for stif_dcn_sep_nhwc): the MFMA
 * A operands [k 36][M-tile m 7][plane h|l][lane 64][8 halves] of W * 2^10, step k = 9 c + tap, lane l
 * holding row i = l & 31 of M-tile m and input channel 16 c + 8 (l >> 5) + e.  Row i is accumulator
 * register r = (i & 3) + 4 (i >> 3) of lane half h = (i >> 2) & 1; half h owns the deformable groups
 * h, h + 2, h + 4, h + 6 and its slot s = 16 m + r < 108 holds component s % 3 (dy, dx, mask) of tap
 * (s % 27) / 3 of group 2 (s / 27) + h (slots 108..111 zero).  Bias: [8][32] in the same row order.
 * STIF_PACK_DCNPAIR | STIF_PACK_F16X3 (the 64 -> 64 3x3 DCN weight of stif_dcn_sep_nhwc): [group pair
 * a 4][tap 9][nt 2][plane h|l][lane 64][8 halves], element e of lane l holding input channel
 * 8 (2 a + (l >> 5)) + e, cout nt * 32 + (l & 31). */
int stif_pack_conv_weight(const float* w_oihw, const float* b, int cout, int cin, int ks, int mode,
                          float* w_dst, float* b_dst);

size_t stif_dec_proj_floats(void);   /* packed fp32 1x1 weight of the LR projection: [25][256][1][8]; the
                                        f16x3 packing: stif_conv_weight_floats(256, 200, 1, STIF_PACK_PLAIN | STIF_PACK_F16X3) */
int stif_pack_dec_proj(const float* feat_w0, const float* feat_b0, const float* flow_w0,
                       const float* enc_w0, float* w_dst, float* b_dst);
/* lr_image bit 0 clear: P2..P4 without the image columns (decoding_test samples a high-resolution
 * image); lr_image | STIF_DEC_REVOLUTIONS: the sine-layer factor is omega_0 / (2 pi) instead of omega_0
 * (pre-activations in revolutions), as the decoder stages run with STIF_CONV_F16X3 expect -- set it iff
 * the mlp was packed with STIF_CONV_F16X3 (the stages cannot check the pairing: a mismatch gives wrong first-layer
 * sines with no error, INTEGRATION.md "Decoder pairing rule"); lr_image | STIF_PACK_F16X3: the PLAIN | F16X3 1x1 packing for stif_conv2d_nhwc with
 * flags = STIF_CONV_F16X3 (split-fp16 k_conv1x1) */
#define STIF_DEC_REVOLUTIONS 2
int stif_pack_dec_proj_ex(const float* feat_w0, const float* feat_b0, const float* flow_w0,
                          const float* enc_w0, int lr_image, float* w_dst, float* b_dst);
size_t stif_dec_mlp_floats(void);
/* Packs every remaining feat/flow/encode_imnet weight (state-dict shapes, see stif_amd.weights)
 * in the order stif_dec_stage1/2 consume them. Pointers follow the Siren layer order:
 * feat: w0,b0,w1,b1,w2,b2,w3,b3; flow: same; enc: w0..w4, b0..b4 interleaved. */
int stif_pack_dec_mlp(const float* const* feat, const float* const* flow, const float* const* enc,
                      float* dst);
/* flags = STIF_CONV_F16X3: every 32x32 MFMA weight tile as a split-fp16 tile ([m 2][plane h|l][lane 64]
 * [8 halves] of W * 2^10, element e of half-tile m = feature F(8m + e, lane >> 5)) and the image tiles
 * scaled by 2^14, and the sine layers scaled by omega_0 / (2 pi) (revolutions: the stages evaluate
 * v_sin_f32(x - rint(x))), for stif_dec_stage1_ex / stif_dec_stage2_ex with the same flag; encode_imnet's
 * tiles are also stored a second time as 16x16x32 A operands for the 16-pixel stage 2 (dec_layout.h Q_*). */
int stif_pack_dec_mlp_ex(const float* const* feat, const float* const* flow, const float* const* enc,
                         float* dst, int flags);

const char* stif_last_error(void);
const char* stif_version(void);

#ifdef __cplusplus
}
#endif
#endif /* STIF_H */
