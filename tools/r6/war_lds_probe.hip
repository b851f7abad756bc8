// Item-4 probe 2: does an LDS load issued right after a VALU op overwrite that op's source registers before the op
// has read them, for the last lanes?  Per wave and iteration (one asm block, fixed registers):
//   [K independent packed fp32 FMAs (VALU backlog)] ; OP: v[10:11] = fma(v[20:21], v[22:23], v[24:25]) ;
//   ds_read_b128 v[20:23] (the LDS holds other values) ; s_waitcnt lgkmcnt(0) ; result = v[10:11]
// OP = v_pk_fma_f32 or two v_fma_f32.  The control loads into v[40:43] instead.  Mismatching lanes are counted
// per 16-lane quarter.  Register-only arithmetic, LDS reads, plain vector stores of the counters.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define STR2(x) #x
#define STR(x) STR2(x)
#define B1 "v_pk_fma_f32 v[30:31], v[32:33], v[34:35], v[30:31]\n" "v_pk_fma_f32 v[36:37], v[32:33], v[34:35], v[36:37]\n"
#define B4 B1 B1 B1 B1
#define B16 B4 B4 B4 B4
#define S1 "v_fma_f32 v30, v32, v34, v30\n" "v_fma_f32 v31, v33, v35, v31\n" "v_fma_f32 v36, v32, v34, v36\n" "v_fma_f32 v37, v33, v35, v37\n"
#define S4 S1 S1 S1 S1
#define S16 S4 S4 S4 S4
#define MF "v_mfma_f32_32x32x16_f16 v[64:79], v[96:99], v[100:103], v[64:79]\n"
#define M4 MF MF MF MF
#define OP_PK "v_pk_fma_f32 v[10:11], v[20:21], v[22:23], v[24:25]\n"
#define OP_SC "v_fma_f32 v10, v20, v22, v24\n" "v_fma_f32 v11, v21, v23, v25\n"
#define LD_HIT "ds_read_b128 v[20:23], %4\n"
#define LD_CTL "ds_read_b128 v[40:43], %4\n"

#define SEQ(BURST, OP, LD)                                                                         \
  "v_mov_b32 v20, %2\nv_mov_b32 v21, %3\nv_mov_b32 v22, %3\nv_mov_b32 v23, %2\n"                  \
  "v_mov_b32 v24, %2\nv_mov_b32 v25, %3\n"                                                         \
  "v_mov_b32 v30, 0\nv_mov_b32 v31, 0\nv_mov_b32 v36, 0\nv_mov_b32 v37, 0\n"                       \
  "v_mov_b32 v32, %2\nv_mov_b32 v33, %3\nv_mov_b32 v34, %3\nv_mov_b32 v35, %2\n"                  \
  "s_nop 7\n" BURST OP LD "s_waitcnt lgkmcnt(0)\n"                                                  \
  "v_mov_b32 %0, v10\nv_mov_b32 %1, v11\n"

#define CLOB "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", \
  "v79", "v10", "v11", "v20", "v21", "v22", "v23", "v24", "v25", "v30", "v31", "v32", "v33", "v34", "v35", \
  "v36", "v37", "v40", "v41", "v42", "v43", "memory"

template <int MODE>  // 0: pk op, no backlog; 1: pk op after 32 packed FMAs; 2: 2x v_fma, no backlog; 3: 2x v_fma after 64 FMAs
__device__ __forceinline__ void run(float x, float y, unsigned addr, float& r0, float& r1, float& c0, float& c1) {
  if (MODE == 0) {
    asm volatile(SEQ("", OP_PK, LD_HIT) : "=v"(r0), "=v"(r1) : "v"(x), "v"(y), "v"(addr) : CLOB);
    asm volatile(SEQ("", OP_PK, LD_CTL) : "=v"(c0), "=v"(c1) : "v"(x), "v"(y), "v"(addr) : CLOB);
  } else if (MODE == 1) {
    asm volatile(SEQ(B16, OP_PK, LD_HIT) : "=v"(r0), "=v"(r1) : "v"(x), "v"(y), "v"(addr) : CLOB);
    asm volatile(SEQ(B16, OP_PK, LD_CTL) : "=v"(c0), "=v"(c1) : "v"(x), "v"(y), "v"(addr) : CLOB);
  } else if (MODE == 2) {
    asm volatile(SEQ("", OP_SC, LD_HIT) : "=v"(r0), "=v"(r1) : "v"(x), "v"(y), "v"(addr) : CLOB);
    asm volatile(SEQ("", OP_SC, LD_CTL) : "=v"(c0), "=v"(c1) : "v"(x), "v"(y), "v"(addr) : CLOB);
  } else if (MODE == 4) {
    asm volatile(SEQ(M4, OP_PK, LD_HIT) : "=v"(r0), "=v"(r1) : "v"(x), "v"(y), "v"(addr) : CLOB);
    asm volatile(SEQ(M4, OP_PK, LD_CTL) : "=v"(c0), "=v"(c1) : "v"(x), "v"(y), "v"(addr) : CLOB);
  } else if (MODE == 5) {
    asm volatile(SEQ(M4, OP_SC, LD_HIT) : "=v"(r0), "=v"(r1) : "v"(x), "v"(y), "v"(addr) : CLOB);
    asm volatile(SEQ(M4, OP_SC, LD_CTL) : "=v"(c0), "=v"(c1) : "v"(x), "v"(y), "v"(addr) : CLOB);
  } else {
    asm volatile(SEQ(S16, OP_SC, LD_HIT) : "=v"(r0), "=v"(r1) : "v"(x), "v"(y), "v"(addr) : CLOB);
    asm volatile(SEQ(S16, OP_SC, LD_CTL) : "=v"(c0), "=v"(c1) : "v"(x), "v"(y), "v"(addr) : CLOB);
  }
}

template <int MODE, int STORM>
__global__ __launch_bounds__(512) void k_probe(unsigned* bad, int iters) {
  __shared__ __attribute__((aligned(16))) float lds[512 * 4];
  extern __shared__ char pad[];
  if (threadIdx.x == 0xffffffffu) pad[0] = 0;
  const int tid = threadIdx.x, lane = tid & 63;
  for (int k = 0; k < 4; ++k) lds[tid * 4 + k] = 1000.f + tid * 4 + k;
  __syncthreads();
  const unsigned addr = (unsigned)(uintptr_t)(&lds[tid * 4]);
  unsigned cnt = 0;
  if (STORM && ((tid >> 6) & 1)) {   // odd waves: an MFMA + packed-fp32 storm beside the probing waves (wave-uniform)
    for (int it = 0; it < iters * 4; ++it)
      asm volatile(M4 B4 ::: "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76",
                   "v77", "v78", "v79", "v30", "v31", "v36", "v37");
    bad[blockIdx.x * blockDim.x + tid] = 0;
    return;
  }
  for (int it = 0; it < iters; ++it) {
    const float x = 1.0f + 0.001f * (lane + it), y = 2.0f - 0.0005f * (lane + 3 * it);
    float r0, r1, c0, c1;
    run<MODE>(x, y, addr, r0, r1, c0, c1);
    cnt += (__builtin_bit_cast(unsigned, r0) != __builtin_bit_cast(unsigned, c0)) |
           (__builtin_bit_cast(unsigned, r1) != __builtin_bit_cast(unsigned, c1));
  }
  bad[blockIdx.x * blockDim.x + tid] = cnt;
}

template <int MODE, int STORM>
static void launch(unsigned* dbad, unsigned* hbad, int blocks, int threads, int lds, int iters, unsigned long long q[4]) {
  (void)hipFuncSetAttribute((const void*)k_probe<MODE, STORM>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
  hipLaunchKernelGGL((k_probe<MODE, STORM>), dim3(blocks), dim3(threads), lds, 0, dbad, iters);
  if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); exit(1); }
  (void)hipMemcpy(hbad, dbad, sizeof(unsigned) * blocks * threads, hipMemcpyDeviceToHost);
  for (int i = 0; i < 4; ++i) q[i] = 0;
  for (int i = 0; i < blocks * threads; ++i) q[(i & 63) >> 4] += hbad[i];
}

int main() {
  const int blocks = 2048, iters = 256;
  unsigned* dbad; (void)hipMalloc(&dbad, sizeof(unsigned) * blocks * 512);
  unsigned* hbad = (unsigned*)malloc(sizeof(unsigned) * blocks * 512);
  struct { int threads, lds; const char* name; } occ[] = {
    {256, 140 * 1024, "1 wave/SIMD"}, {512, 140 * 1024, "2 waves/SIMD (1 WG of 8 waves)"},
    {256, 60 * 1024, "2 waves/SIMD (2 WGs of 4 waves)"}, {256, 0, "up to 8 waves/SIMD"}};
  const char* mname[] = {"v_pk_fma_f32            ", "v_pk_fma_f32 after 32 pk", "2x v_fma_f32            ", "2x v_fma_f32 after 64   ",
                         "v_pk_fma_f32 after 4 MFMA", "2x v_fma_f32 after 4 MFMA"};
  for (auto& o : occ) {
    printf("%s: %d blocks x %d threads x %d iters; iterations whose result differs from the control, per lane quarter\n",
           o.name, blocks, o.threads, iters);
    unsigned long long q[4];
#define ROW(MODE, STORM) launch<MODE, STORM>(dbad, hbad, blocks, o.threads, o.lds, iters, q); \
    printf("  %s%s %llu %llu %llu %llu\n", mname[MODE], STORM ? " +storm" : "       ", q[0], q[1], q[2], q[3]);
    ROW(0, 0) ROW(1, 0) ROW(2, 0) ROW(3, 0) ROW(4, 0) ROW(5, 0)
    ROW(0, 1) ROW(1, 1) ROW(2, 1) ROW(4, 1) ROW(5, 1)
  }
  (void)hipFree(dbad); free(hbad);
  return 0;
}
