// Compile-time tuning knobs of the gfx950 kernels, in one place.  Each default is the measured optimum
// of a same-box A/B (DESIGN.md sections 3-5, logs under profiles/); tools/build_obj_variants.sh builds a
// one-object library with any of them overridden (-DNAME=value) for such an A/B.  The *_EXP switches are
// timing probes that skip work and give wrong results; they are never set in a product build.
#pragma once

// ---- k_wino / k_wino_om (wino.hip)
#ifndef WINO_OM
#define WINO_OM 1          // offset/mask conv (f16x3) by k_wino_om; 0 = the per-slice k_wino
#endif
#ifndef WINO_OM_RING
#define WINO_OM_RING 2     // k_wino_om B-operand blocks in flight (4: 158 -> 170-177 us, r02_wino_om_ring_ab.log)
#endif
#ifndef WINO_OM_SCHED
#define WINO_OM_SCHED 1    // a scheduling barrier after every k_wino_om B block (keeps the B loads early)
#endif
#ifndef WINO_UPQ
#define WINO_UPQ 1         // fused x2 upsample expanded by 2 x 2 quads (0: per pixel, k_up2's expression)
#endif
static_assert(WINO_UPQ == 0 || WINO_UPQ == 1, "WINO_UPQ");
#ifndef WINO_NT
#define WINO_NT 0          // cache-policy bits (aux) of the input-halo LDS-DMA (2 = nt)
#endif
#ifndef WINO_TRACE
#define WINO_TRACE 0       // diagnostic: per-wave s_memtime sums of the ResidualBlock conv1 (stif_wino_trace_set)
#endif
#ifndef WINO_EXP
#define WINO_EXP 0         // probes: 1 no LDS-DMA after the first phase, 2 no B refills, 3 no output exchange,
                           // 4 no x2-upsample expansion (in1_mode 2), 5 RELU-epilogue convs store nothing,
                           // 6 k_wino_om stores nothing (out-of-range store offsets), 7 RELU-epilogue convs do a
                           // third chunk-pair pass per phase (1.5x work: a conv1 over its 1-px halo) and store nothing
#endif

// ---- k_dcn (dcn.hip): the DCN core of the two-kernel path and the _ext drop-in at the STIF shape
#ifndef DCN_TH
// waves per workgroup: 4 (8-row two-row tiles, two workgroups per CU whose barriers and memory waits
// overlap): C0 L1 DCN 240 -> 223 us against 8 (r02_dcn_th_ab.log)
#define DCN_TH 4
#endif
#ifndef DCN_M
// staged margin (px) around the 3x3 footprint; samples beyond it use the global-load fallback.
// C0 L1: margin 2 / 3 / 4 / 6 / 8 -> 248 / 250 / 257 / 266 / 289 us (r02_dcn_margin_ab.log)
#define DCN_M 2
#endif
#ifndef DCN_MR2_MIN
#define DCN_MR2_MIN 1024   // two-row kernel from this many workgroups (512 measured no faster)
#endif

// ---- k_dcn_sep (dcnsep.hip): the fused DCN_sep
#ifndef DCNSEP_NW
// waves (= output rows) per tile: 4 -> two 80-KB workgroups per CU; 8 -> one 152-KB workgroup staging the
// next group pair ahead (slower)
#define DCNSEP_NW 4
#endif
#ifndef DCNSEP_WPE
#define DCNSEP_WPE 2       // waves per SIMD the kernel is register-budgeted for
#endif
#ifndef DCNSEP_TAPPIPE
#define DCNSEP_TAPPIPE 0   // diagnostic: phase-2 tap t + 1's corner reads before tap t's blend (review r5 item 4)
#endif
#ifndef DCNSEP_TP_NOFB
#define DCNSEP_TP_NOFB 0   // diagnostic (TAPPIPE): no global-load fallback (wrong results past the margin)
#endif
#ifndef DCNSEP_TP_CHECK
#define DCNSEP_TP_CHECK 0  // diagnostic (TAPPIPE): every staged corner / B fragment read checked against HBM (printf)
#endif
#ifndef DCNSEP_TP_DUMP
#define DCNSEP_TP_DUMP 0   // diagnostic (TAPPIPE): per-thread dump of every tap's blended samples and each pair's accumulators
#endif
#ifndef DCNSEP_PRIO
#define DCNSEP_PRIO 0      // wave priority (s_setprio 2) for phase 2 (1) or phase 1 (2) of the fused DCN_sep
#endif
#ifndef DCNSEP_P2PROG
#define DCNSEP_P2PROG 0    // fused DCN_sep phase 2 (NW 4): 0 = wait for the whole pair stage; 3 / 9 = wait in 3 / 9 steps (the
                           // tile + the first taps' weights, then the next taps'), so the taps start while later weights land
#endif
#ifndef DCNSEP_TRACE
#define DCNSEP_TRACE 0     // diagnostic: per-wave s_memtime sums of k_dcn_sep's waits and phases (stif_dcnsep_trace_set)
#endif
#ifndef DCNSEP_P1_SAFE
#define DCNSEP_P1_SAFE 0   // diagnostic: phase-1 steps behind full drains and __syncthreads
#endif
#ifndef DCNSEP_SOLO
#define DCNSEP_SOLO 0      // diagnostic: 48 KB of padding LDS (one workgroup per CU)
#endif
#ifndef DCNSEP_TP_WAIT
#define DCNSEP_TP_WAIT 0   // diagnostic (TAPPIPE): tap t + 1's corner reads drained before tap t's blend
#endif
#ifndef DCNSEP_WTRIM
#define DCNSEP_WTRIM 0     // phase-1 weight stage without its two all-pad DMA pieces per step (NW 4)
#endif
#ifndef DCNSEP_NT
#define DCNSEP_NT 0        // cache-policy bits (aux) of the feature / input tile LDS-DMA (2 = nt)
#endif
#ifndef DCNSEP_EXP
#define DCNSEP_EXP 0       // probes: 1 no phase 1, 3 no phase 2, 5 no per-pair restaging, 6 offset-free sampling,
                           // 7 phase-1 weights DMA'd for the first two steps only (stale after)
#endif
static_assert(DCNSEP_EXP == 0 || DCNSEP_EXP == 1 || DCNSEP_EXP == 3 || DCNSEP_EXP == 5 || DCNSEP_EXP == 6 ||
                  DCNSEP_EXP == 7,
              "DCNSEP_EXP: only probes 1, 3, 5, 6 and 7 exist (a probe number without code would build the product kernel)");

// ---- k_dec1 / k_dec2 (decoder.hip)
#ifndef DEC1_NW
// k_dec1 waves per workgroup for its four-waves-per-SIMD variants (MODE 0 / 1, no high-resolution image): 4 = four
// 4-wave workgroups per CU.  8 (two 8-wave workgroups, each streaming the MLP weights for 256 pixels instead of 128)
// measured slower: C0 stage 1 686-715 -> 768-784 us, C2 10.9 -> 11.7 ms (profiles/r06_dec_ab.log)
#define DEC1_NW 4
#endif
#ifndef DEC1_OCC
// k_dec1 (MODE 0 / 1) workgroups per CU: 4 (36 KB LDS, 128 registers, the flow projection gathered in four
// 8-load quarters), 3 (52 KB, 168, halves) or 2 (69 KB, 256).  C0 dec1 869 -> 758 us (2 -> 3,
// r04_dec1_occ_ab.log) -> 720 us (3 -> 4; C2 11.6 -> 11.1 ms, r04_dec1_occ4_ab.log); all bit-identical
#define DEC1_OCC 4
#endif
#ifndef DEC2_Q16
// stage 2 (f16x3, LR-projection inputs) by k_dec2q: 16 pixels per wave, 4-wave workgroups, four per CU (40 KB
// LDS, 128 VGPRs); C2 stage 2 17.55-17.79 -> 17.32-17.34 ms (r04_dec2q4_ab.log).  0 = k_dec2 (also the
// fp32 and high-resolution-image stages)
#define DEC2_Q16 1
#endif
#ifndef DEC_TRACE
#define DEC_TRACE 0        // diagnostic: k_dec2q per-wave s_memtime sums (gathers, segment barriers, layers 2/3)
#endif
#ifndef DEC1_RES
#define DEC1_RES 0         // stage 1 (f16x3, LR image) as two persistent resident-weight kernels k_dec1f + k_dec1l
#endif
#ifndef DEC_DMA_LATE
#define DEC_DMA_LATE 0     // decoders: issue the next weight segment's LDS-DMA after the step's first (layer-2) MFMAs, in the
                           // sine / split stretch, instead of right after the segment barrier
#endif
#ifndef DEC2Q_NW
#define DEC2Q_NW 8         // k_dec2q waves per workgroup (8: two 80-KB workgroups per CU; 16: one 160-KB workgroup)
#endif
#ifndef DEC2Q_KTS
#define DEC2Q_KTS (DEC2Q_NW == 16 ? 2 : 1)   // layer-2 tiles per streamed weight segment
#endif
#ifndef DEC2_WPE
#define DEC2_WPE 2         // waves per SIMD k_dec2 is register-budgeted for (2 workgroups/CU, 80 KB LDS each)
#endif
static_assert(DEC1_OCC >= 2 && DEC1_OCC <= 4, "DEC1_OCC: k_dec1 is laid out for 2, 3 or 4 workgroups per CU");
static_assert(DEC2_Q16 == 0 || DEC2_Q16 == 1, "DEC2_Q16: 0 (k_dec2) or 1 (k_dec2q)");
#ifndef DEC_EXP
#define DEC_EXP 0          // probes: 2 segment barriers without the vmcnt(0) wait for the segment, 3 every weight
                           // DMA piece issued out of range (same instructions, no memory traffic, zero weights) --
                           // both with wrong results.  (1, no DMA at all, is gone: the compiler folds the work that
                           // reads never-written LDS, profiles/r06_dec_probe3.log)
#endif
static_assert(DEC_EXP == 0 || DEC_EXP == 2 || DEC_EXP == 3, "DEC_EXP");
