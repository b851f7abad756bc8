"""Build tools/exp_trace.so: the engine library with k_wino (F16 path) instrumented by a per-wave
s_memtime event trace, patched into a temporary copy of the sources (the product kernel carries no
trace hooks).  Tags: 1 tile start, 6 before a phase's wait+barrier, 2 after it, 3 after an exchange
barrier, 5 before the closing barrier, 4 after it, 7 tile setup done (accumulators zeroed), 8 / 9 after sub-phase 0 / 1 of a phase.  Read with tools/experiments/trace_wino.py."""
import os
import shutil
import subprocess
import sys
import tempfile

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(R, "stif-continuous-video-representation_amd")
T = tempfile.mkdtemp()
shutil.copytree(os.path.join(PKG, "csrc"), os.path.join(T, "csrc"))
p = os.path.join(T, "csrc", "wino.hip")
s = open(p).read()


def sub(old, new, count=1):
    global s
    assert s.count(old) == count, (old, s.count(old))
    s = s.replace(old, new)


sub("struct Tile {\n", '''__device__ unsigned long long g_wtrace[512 * 4 * 128];
#define WTR(tag)                                                                                   \\
  do {                                                                                             \\
    if (F16 && ntr < 127 && blockIdx.x < 512 && lane == 0)                                         \\
      g_wtrace[(blockIdx.x * 4 + wi) * 128 + ntr] = (__builtin_amdgcn_s_memtime() << 8) | (tag);   \\
    ++ntr;                                                                                         \\
  } while (0)

struct Tile {
''')
sub('''  if (T >= tend) return;
  Tile cur = tile_of(T);
  const float* wsl = wbase(cur);''', '''  if (T >= tend) return;
  int ntr = 0;
  if (F16 && blockIdx.x < 512 && lane == 0) {   // slot 127: hardware placement (HW_ID, XCC_ID)
    const unsigned hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));
    const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11));
    g_wtrace[(blockIdx.x * 4 + wi) * 128 + 127] = ((unsigned long long)xcc << 32) | hw;
  }
  Tile cur = tile_of(T);
  const float* wsl = wbase(cur);''')
sub('''  for (;;) {
    const int Tn = T + nl;
    const bool has_next = Tn < tend;
    const Tile nxt = tile_of(has_next ? Tn : T);
    const float* wnx = wbase(nxt);
''', '''  for (;;) {
    WTR(1);
    const int Tn = T + nl;
    const bool has_next = Tn < tend;
    const Tile nxt = tile_of(has_next ? Tn : T);
    const float* wnx = wbase(nxt);
''')
sub('''        // every load older than the last two blocks' B refills (8) -- the phase's LDS-DMA among
        // them -- has landed
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        __syncthreads();''', '''        WTR(6);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        __syncthreads();
        WTR(2);''')
sub('''          wb[((r & 3) + 8 * (r >> 2)) * 32 + ((r & 1) ? -fl : fl)] = yv[nt][b][r];
      }
      __syncthreads();''', '''          wb[((r & 3) + 8 * (r >> 2)) * 32 + ((r & 1) ? -fl : fl)] = yv[nt][b][r];
      }
      __syncthreads();
      WTR(3);''')
sub('''    if (F16) report_range(a.status, not_finite(chk));   // a non-finite output makes the sum non-finite
    __syncthreads();   // exchange buffer free for the next tile's staging''', '''    if (F16) report_range(a.status, not_finite(chk));   // a non-finite output makes the sum non-finite
    WTR(5);
    STORE_WAIT
    __syncthreads();   // exchange buffer free for the next tile's staging
    WTR(4);''')
sub('''            __builtin_amdgcn_sched_barrier(0);
          }
        }
        WTR(6);''', '''            __builtin_amdgcn_sched_barrier(0);
          }
          WTR(8 + sp);
        }
        WTR(6);''')
sub('''    if constexpr (F16) {
      for (int p = 0; p < NP; ++p, ++gp) {''', '''    if constexpr (F16) {
      WTR(7);
      for (int p = 0; p < NP; ++p, ++gp) {''')
# STORE_WAIT=1: drain the tile's output stores before the closing barrier (probe of store latency)
s = s.replace("STORE_WAIT", 'asm volatile("s_waitcnt vmcnt(0)" ::: "memory");' if os.environ.get("STORE_WAIT") else "")
s += '''
extern "C" int stif_exp_wino_trace(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_wtrace), sizeof(g_wtrace)) == hipSuccess ? 0 : -1;
}
'''
open(p, "w").write(s)
src = [os.path.join(T, "csrc", f) for f in sorted(os.listdir(os.path.join(T, "csrc"))) if f.endswith(".hip")]
src.append(os.path.join(T, "csrc", "pack.cpp"))
out = os.path.join(R, "tools", os.environ.get("OUT", "exp_trace.so"))
subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                       "-I" + os.path.join(R, "include"), "-I" + os.path.join(T, "csrc"), "-shared", "-o", out] + src)
shutil.rmtree(T)
print("built", out)
