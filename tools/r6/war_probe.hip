// Item-4 probe: does a VALU write to a VGPR that a just-issued XDL MFMA reads as SrcB change the MFMA's
// result on gfx950?  Sequence per wave (fixed registers, one asm block, so no compiler hazard padding):
//   [BUSY independent MFMAs on other accumulators] ; v_mfma_f32_32x32x16_f16 acc, A, B, acc ;
//   D independent VALU fillers ; WRITER overwrites B[2:3] (or A[2:3])
// WRITER = v_pk_mul_f32 (packed fp32) or two v_mul_f32.  The control writes unrelated registers instead.
// Every lane compares its 16 accumulators with the control bit for bit.  Pure register code, no memory
// inside the asm; results go out with ordinary vector stores.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define STR2(x) #x
#define STR(x) STR2(x)
#define F1 "v_mov_b32 v120, v121\n"
#define F2 F1 F1
#define F4 F2 F2
#define F8 F4 F4
#define FILL0 ""
#define FILL1 F1
#define FILL2 F2
#define FILL3 F2 F1
#define FILL4 F4
#define FILL5 F4 F1
#define FILL6 F4 F2
#define FILL7 F4 F2 F1
#define FILL8 F8
#define FILL12 F8 F4
#define FILL16 F8 F8

#define PK_B   "v_pk_mul_f32 v[106:107], v[108:109], v[110:111]\n"
#define PK_A   "v_pk_mul_f32 v[98:99], v[108:109], v[110:111]\n"
#define PK_X   "v_pk_mul_f32 v[112:113], v[108:109], v[110:111]\n"
#define SC_B   "v_mul_f32 v106, v108, v110\nv_mul_f32 v107, v109, v111\n"
#define SC_A   "v_mul_f32 v98, v108, v110\nv_mul_f32 v99, v109, v111\n"
#define SC_X   "v_mul_f32 v112, v108, v110\nv_mul_f32 v113, v109, v111\n"

#define M1 "v_mfma_f32_32x32x16_f16 v[128:143], v[96:99], v[104:107], v[128:143]\n"
#define CHAIN "v_mfma_f32_32x32x16_f16 v[64:79], v[96:99], v[104:107], v[64:79]\n" \
  "v_mfma_f32_32x32x16_f16 v[128:143], v[96:99], v[104:107], v[128:143]\n" \
  "v_mfma_f32_32x32x16_f16 v[64:79], v[96:99], v[104:107], v[64:79]\n" \
  "v_mfma_f32_32x32x16_f16 v[128:143], v[96:99], v[104:107], v[128:143]\n" \
  "v_mfma_f32_32x32x16_f16 v[64:79], v[96:99], v[104:107], v[64:79]\n"
#define BUSY0 ""
#define BUSY1 M1
#define BUSY2 M1 M1
#define BUSY4 M1 M1 M1 M1
#define SEQ(FILL, WR)                                                                              \
  "v_mov_b32 v96, %16\nv_mov_b32 v97, %17\nv_mov_b32 v98, %18\nv_mov_b32 v99, %19\n"               \
  "v_mov_b32 v104, %20\nv_mov_b32 v105, %21\nv_mov_b32 v106, %22\nv_mov_b32 v107, %23\n"           \
  "v_mov_b32 v108, %24\nv_mov_b32 v109, %24\nv_mov_b32 v110, %24\nv_mov_b32 v111, %24\n"          \
  "v_mov_b32 v121, %24\n"                                                                          \
  "v_mov_b32 v64, 0\nv_mov_b32 v65, 0\nv_mov_b32 v66, 0\nv_mov_b32 v67, 0\n"                       \
  "v_mov_b32 v68, 0\nv_mov_b32 v69, 0\nv_mov_b32 v70, 0\nv_mov_b32 v71, 0\n"                       \
  "v_mov_b32 v72, 0\nv_mov_b32 v73, 0\nv_mov_b32 v74, 0\nv_mov_b32 v75, 0\n"                       \
  "v_mov_b32 v76, 0\nv_mov_b32 v77, 0\nv_mov_b32 v78, 0\nv_mov_b32 v79, 0\n"                       \
  "s_nop 7\ns_nop 7\n" BUSYSEQ                                                                    \
  "v_mfma_f32_32x32x16_f16 v[64:79], v[96:99], v[104:107], v[64:79]\n" FILL WR                      \
  "s_nop 7\ns_nop 7\ns_nop 7\ns_nop 7\n"                                                           \
  "v_mov_b32 %0, v64\nv_mov_b32 %1, v65\nv_mov_b32 %2, v66\nv_mov_b32 %3, v67\n"                   \
  "v_mov_b32 %4, v68\nv_mov_b32 %5, v69\nv_mov_b32 %6, v70\nv_mov_b32 %7, v71\n"                   \
  "v_mov_b32 %8, v72\nv_mov_b32 %9, v73\nv_mov_b32 %10, v74\nv_mov_b32 %11, v75\n"                 \
  "v_mov_b32 %12, v76\nv_mov_b32 %13, v77\nv_mov_b32 %14, v78\nv_mov_b32 %15, v79\n"

#define OUTS(r) "=v"(r[0]), "=v"(r[1]), "=v"(r[2]), "=v"(r[3]), "=v"(r[4]), "=v"(r[5]), "=v"(r[6]), "=v"(r[7]), \
  "=v"(r[8]), "=v"(r[9]), "=v"(r[10]), "=v"(r[11]), "=v"(r[12]), "=v"(r[13]), "=v"(r[14]), "=v"(r[15])
#define INS "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(junk)
#define CLOB "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", \
  "v96","v97","v98","v99","v104","v105","v106","v107","v108","v109","v110","v111","v112","v113","v120","v121", \
  "v128","v129","v130","v131","v132","v133","v134","v135","v136","v137","v138","v139","v140","v141","v142","v143"

template <int D, int W>  // W: 0 pk->B, 1 pk->A, 2 scalar->B, 3 scalar->A
__device__ __forceinline__ void run(const unsigned* a, const unsigned* b, unsigned junk, unsigned* r, unsigned* c) {
#define CASE(FILL)                                                                                      \
  if (W == 0) asm volatile(SEQ(FILL, PK_B) : OUTS(r) : INS : CLOB);                                     \
  if (W == 1) asm volatile(SEQ(FILL, PK_A) : OUTS(r) : INS : CLOB);                                     \
  if (W == 2) asm volatile(SEQ(FILL, SC_B) : OUTS(r) : INS : CLOB);                                     \
  if (W == 3) asm volatile(SEQ(FILL, SC_A) : OUTS(r) : INS : CLOB);                                     \
  if (W <= 1) asm volatile(SEQ(FILL, PK_X) : OUTS(c) : INS : CLOB);                                     \
  else asm volatile(SEQ(FILL, SC_X) : OUTS(c) : INS : CLOB);
  if (D == 0) { CASE(FILL0) } else if (D == 1) { CASE(FILL1) } else if (D == 2) { CASE(FILL2) }
  else if (D == 3) { CASE(FILL3) } else if (D == 4) { CASE(FILL4) } else if (D == 5) { CASE(FILL5) }
  else if (D == 6) { CASE(FILL6) } else if (D == 7) { CASE(FILL7) } else if (D == 8) { CASE(FILL8) }
  else if (D == 12) { CASE(FILL12) } else { CASE(FILL16) }
#undef CASE
}

template <int D, int W>
__global__ __launch_bounds__(512) void k_probe(unsigned* bad, int iters, unsigned seed) {
  extern __shared__ char pad[];  // occupancy control only
  if (threadIdx.x == 0xffffffffu) pad[0] = 0;
  unsigned t = blockIdx.x * blockDim.x + threadIdx.x, s = seed ^ (t * 2654435761u);
  unsigned cnt = 0;
  for (int it = 0; it < iters; ++it) {
    unsigned a[4], b[4], r[16], c[16];
    for (int k = 0; k < 4; ++k) {
      s = s * 1664525u + 1013904223u; a[k] = (s >> 1) & 0x3bff3bffu;  // finite f16 pairs
      s = s * 1664525u + 1013904223u; b[k] = (s >> 1) & 0x3bff3bffu;
    }
    run<D, W>(a, b, 0x7f7f7f7fu ^ s, r, c);
    for (int k = 0; k < 16; ++k) cnt += (r[k] != c[k]);
  }
  bad[t] = cnt;
}

template <int D, int W>
static unsigned long long launch(unsigned* dbad, unsigned* hbad, int blocks, int threads, int lds, int iters) {
  hipFuncSetAttribute((const void*)k_probe<D, W>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipLaunchKernelGGL((k_probe<D, W>), dim3(blocks), dim3(threads), lds, 0, dbad, iters, 12345u + D * 7 + W);
  if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); exit(1); }
  hipMemcpy(hbad, dbad, sizeof(unsigned) * blocks * threads, hipMemcpyDeviceToHost);
  unsigned long long n = 0;
  for (int i = 0; i < blocks * threads; ++i) n += hbad[i];
  return n;
}

template <int D>
static void row(unsigned* dbad, unsigned* hbad, int blocks, int threads, int lds, int iters) {
  unsigned long long n0 = launch<D, 0>(dbad, hbad, blocks, threads, lds, iters);
  unsigned long long n1 = launch<D, 1>(dbad, hbad, blocks, threads, lds, iters);
  unsigned long long n2 = launch<D, 2>(dbad, hbad, blocks, threads, lds, iters);
  unsigned long long n3 = launch<D, 3>(dbad, hbad, blocks, threads, lds, iters);
  printf("  D=%2d  pk->B %10llu  pk->A %10llu  2xmul->B %10llu  2xmul->A %10llu\n", D, n0, n1, n2, n3);
}

int main() {
  const int blocks = 2048, iters = 64;
  unsigned* dbad; hipMalloc(&dbad, sizeof(unsigned) * blocks * 512);
  unsigned* hbad = (unsigned*)malloc(sizeof(unsigned) * blocks * 512);
  struct { int threads, lds; const char* name; } occ[] = {
    {256, 160 * 1024, "1 wave/SIMD (256 threads, 1 WG/CU)"},
    {256, 0, "up to 8 waves/SIMD (256-thread WGs, no LDS)"},
    {512, 80 * 1024, "2 waves/SIMD (512 threads, 1 WG/CU)"},
    {256, 80 * 1024, "2 waves/SIMD (2 x 256-thread WGs/CU)"}};
  for (auto& o : occ) {
    printf("%s: %d blocks x %d iters, mismatching accumulators out of %llu\n", o.name, blocks, iters,
           (unsigned long long)blocks * o.threads * iters * 16);
    row<0>(dbad, hbad, blocks, o.threads, o.lds, iters); row<1>(dbad, hbad, blocks, o.threads, o.lds, iters);
    row<2>(dbad, hbad, blocks, o.threads, o.lds, iters); row<3>(dbad, hbad, blocks, o.threads, o.lds, iters);
    row<4>(dbad, hbad, blocks, o.threads, o.lds, iters); row<5>(dbad, hbad, blocks, o.threads, o.lds, iters);
    row<6>(dbad, hbad, blocks, o.threads, o.lds, iters); row<7>(dbad, hbad, blocks, o.threads, o.lds, iters);
    row<8>(dbad, hbad, blocks, o.threads, o.lds, iters); row<12>(dbad, hbad, blocks, o.threads, o.lds, iters);
    row<16>(dbad, hbad, blocks, o.threads, o.lds, iters);
  }
  hipFree(dbad); free(hbad);
  return 0;
}
