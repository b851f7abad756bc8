"""Build tools/exp_dectrace.so: the engine library with k_dec2 (f16x3) instrumented by a per-wave s_memtime event
trace, patched into a temporary copy of decoder.hip and linked with the in-tree objects (make first; the product
kernel carries no trace hooks).  Every 4th workgroup (up to 4,096 of them) records (cycle << 8 | tag) for tags
0 start, 1 P3 gathered, 2 P4 gathered + layer-0 LR terms, 3 HRfeat(grid 1) gathered, 4 after the layer-0 weight
barrier, 5 layer-0 MFMAs of q_feat1, 6 HRfeat(grid 2) gathered, 7 layer 0 done, 8 after the layer-1 barrier,
9 layer 1 done; per layer-2/3 step 10 before its barrier, 11 after it, 12 layer-2 tile + sine + split, 13 its
layer-3 MFMAs; 14 after the layer-4 barrier, 15 layer 4 done, 16 stored.  Read with tools/r4/trace_dec.py."""
import os
import shutil
import subprocess
import tempfile

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(R, "stif-continuous-video-representation_amd")
T = tempfile.mkdtemp()
shutil.copytree(os.path.join(PKG, "csrc"), os.path.join(T, "csrc"))
p = os.path.join(T, "csrc", "decoder.hip")
s = open(p).read()


def sub(old, new, count=1):
    global s
    assert s.count(old) == count, (old, s.count(old))
    s = s.replace(old, new)


sub("template <bool HRIMG, int F16>\n__global__", '''__device__ unsigned long long g_dtrace[4096 * 4 * 64];
#define DTR(tag)                                                                                           \\
  do {                                                                                                     \\
    if (F16 && (blockIdx.x & 3) == 0 && (blockIdx.x >> 2) < 4096 && lane == 0 && ntr < 64)                 \\
      g_dtrace[((blockIdx.x >> 2) * 4 + wv) * 64 + ntr] = (__builtin_amdgcn_s_memtime() << 8) | (tag);     \\
    ++ntr;                                                                                                 \\
  } while (0)
template <bool HRIMG, int F16>
__global__''')
sub('''  const float* HRF = hrfeat + (size_t)item * HH * WW * 64;
''', '''  const float* HRF = hrfeat + (size_t)item * HH * WW * 64;
  int ntr = 0;
  DTR(0);
''')
sub('''    gather64(z, P, PROJ_C, 128, bilin(g1x, g1y, w, h), hf);
    asm volatile("" ::: "memory");
    gather64(q, P, PROJ_C, 192, bilin(g2x, g2y, w, h), hf);''', '''    gather64(z, P, PROJ_C, 128, bilin(g1x, g1y, w, h), hf);
    DTR(1);
    asm volatile("" ::: "memory");
    gather64(q, P, PROJ_C, 192, bilin(g2x, g2y, w, h), hf);''')
sub('''    asm volatile("" ::: "memory");
    gather64(q, HRF, 64, 0, bilin(g1x, g1y, WW, HH), hf);   // q_feat1 -> W0 columns 0..63
    lds_dma_barrier();''', '''    DTR(2);
    asm volatile("" ::: "memory");
    gather64(q, HRF, 64, 0, bilin(g1x, g1y, WW, HH), hf);   // q_feat1 -> W0 columns 0..63
    DTR(3);
    lds_dma_barrier();
    DTR(4);''')
sub('''    asm volatile("" ::: "memory");
    gather64(q, HRF, 64, 0, bilin(g2x, g2y, WW, HH), hf);   // q_feat2 -> W0 columns 64..127''', '''    DTR(5);
    asm volatile("" ::: "memory");
    gather64(q, HRF, 64, 0, bilin(g2x, g2y, WW, HH), hf);   // q_feat2 -> W0 columns 64..127
    DTR(6);''')
sub('''  lds_dma_barrier();
  const Bias32 eb1[2] = {bias_ld(mlp + E_B1, hf), bias_ld(mlp + E_B1 + 32, hf)};   // before the DMA''', '''  DTR(7);
  lds_dma_barrier();
  DTR(8);
  const Bias32 eb1[2] = {bias_ld(mlp + E_B1, hf), bias_ld(mlp + E_B1 + 32, hf)};   // before the DMA''')
sub('''  const XT<F16> x1s[2] = {xop<F16>(x1[0]), xop<F16>(x1[1])};
  // layer 2 (64 -> 256, sine) streamed tile by tile''', '''  const XT<F16> x1s[2] = {xop<F16>(x1[0]), xop<F16>(x1[1])};
  DTR(9);
  // layer 2 (64 -> 256, sine) streamed tile by tile''')
sub('''  auto l23_step = [&](int kt, bool last) {   // kt = 7 peeled (see k_dec1's feat_step)
    lds_dma_barrier();''', '''  auto l23_step = [&](int kt, bool last) {   // kt = 7 peeled (see k_dec1's feat_step)
    DTR(10);
    lds_dma_barrier();
    DTR(11);''')
sub('''    const XT<F16> h2 = xop<F16>(bias_sin<F16>(acc, b2));
#pragma unroll
    for (int ot = 0; ot < 8; ++ot) tile_mma<F16>(a3[ot], cur + (2 + ot) * T, h2, lane);
  };''', '''    const XT<F16> h2 = xop<F16>(bias_sin<F16>(acc, b2));
    DTR(12);
#pragma unroll
    for (int ot = 0; ot < 8; ++ot) tile_mma<F16>(a3[ot], cur + (2 + ot) * T, h2, lane);
    DTR(13);
  };''')
sub('''  lds_dma_barrier();
  float o4[3] = {0.f, 0.f, 0.f};''', '''  lds_dma_barrier();
  DTR(14);
  float o4[3] = {0.f, 0.f, 0.f};''')
sub('''  for (int c = 0; c < 3; ++c) o4[c] += __shfl_xor(o4[c], 32);   // the other lane half's 128 features
  if (valid && hf == 0) {
    const size_t plane = (size_t)HH * WW;''', '''  for (int c = 0; c < 3; ++c) o4[c] += __shfl_xor(o4[c], 32);   // the other lane half's 128 features
  DTR(15);
  if (valid && hf == 0) {
    const size_t plane = (size_t)HH * WW;''')
sub('''    if (F16) report_range(status, bad);
  }
}''', '''    if (F16) report_range(status, bad);
  }
  DTR(16);
}''')
s += '''
extern "C" int stif_exp_dec_trace(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dtrace), sizeof(g_dtrace)) == hipSuccess ? 0 : -1;
}
'''
open(p, "w").write(s)
subprocess.check_call(["make", "-s", "-C", R])
obj = os.path.join(T, "decoder.o")
subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                       "-I" + os.path.join(R, "include"), "-I" + os.path.join(T, "csrc"), "-Wno-unused-function",
                       "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops", "-c", "-o", obj, p])
objs = [os.path.join(R, "build", f) for f in sorted(os.listdir(os.path.join(R, "build")))
        if f.endswith(".o") and not f.startswith("exp_") and f != "decoder.o"]
out = os.path.join(R, "tools", "exp_dectrace.so")
subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-o", out] + objs + [obj])
shutil.rmtree(T)
print("built", out)
