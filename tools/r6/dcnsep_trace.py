"""Where a k_dcn_sep<0> launch's wave time goes (DCNSEP_TRACE build): per wave, s_memtime sums of phase 1's vmcnt waits
and barriers, phase 2's pair stage + wait, and the phase / epilogue spans.  Re-runs the C0 window's largest fused
launch (8 weight sets x 6 items x 128 x 128) 3x with the trace on, once with it off (HIP events)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import stif_pkg  # noqa: E402

stif = stif_pkg.load()
print("library:", stif._lib.LIB_PATH)
h = stif._lib.lib()
h.stif_dcnsep_trace_set.argtypes = [ctypes.c_void_p]
sd = {k: torch.from_numpy(v) for k, v in stif.weights.make_state_dict(0).items()}
fr = torch.empty(7, 3, 128, 128)
for i in range(7):
    fr[i] = torch.rand(3, 128, 128, generator=torch.Generator().manual_seed(1234 + i))
fr = fr.cuda()
ops = stif.ops
orig = ops.dcn_sep
caught = []


def catch(groups, epi=0, status=None):
    orig(groups, epi=epi, status=status)
    caught.append(([{k: (v.clone() if torch.is_tensor(v) else v) for k, v in g.items()} for g in groups], epi))


ops.dcn_sep = catch
m = stif.LunaTokis(64, 6, 8, 5, 40, mfma="f16x3", range_check="off")
m.load_state_dict(sd, strict=True)
m.eval()
with torch.no_grad():
    m.gen_feat_window(fr)
ops.dcn_sep = orig
NW = 4
big = max(range(len(caught)), key=lambda i: len(caught[i][0]) * caught[i][0][0]["out"].numel())
groups, epi = caught[big]
o = groups[0]["out"]
N, H, W = o.shape[0], o.shape[1], o.shape[2]
wgs = ((W + 31) // 32) * ((H + NW - 1) // NW) * len(groups) * N
print(f"launch {big}: {len(groups)} weight sets, out {tuple(o.shape)}, {wgs} workgroups")
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for rep in range(4):
    tr = torch.zeros(wgs * NW * 8, dtype=torch.int32, device="cuda")
    h.stif_dcnsep_trace_set(tr.data_ptr() if rep else None)
    g2 = [dict(g, out=torch.empty_like(g["out"])) for g in groups]
    torch.cuda.synchronize()
    ev0.record()
    orig(g2, epi=epi)
    ev1.record()
    torch.cuda.synchronize()
    h.stif_dcnsep_trace_set(None)
    ms = ev0.elapsed_time(ev1)
    if rep == 0:
        print(f"  untraced: {ms * 1e3:.1f} us")
        continue
    t = tr.view(wgs * NW, 8).cpu().to(torch.int64) & 0xFFFFFFFF
    t0, p1e, p2e, end, vm, bar, p2w = (t[:, i].double() for i in range(7))
    span = (t0 + end).max() - t0.min()
    life = end.mean()
    print(f"  traced: {ms * 1e3:.1f} us; launch span {span / 1e3:.1f} k-cycles, mean wave life {life / 1e3:.1f} k-cycles "
          f"({life / span * 100:.1f} % of the span; {(end.sum() / span / 1024):.2f} waves per SIMD on average)")
    print(f"    phase 1 {p1e.mean() / life * 100:5.1f} % of a wave's life  (vmcnt waits {vm.mean() / life * 100:5.1f} %, "
          f"barriers {bar.mean() / life * 100:5.1f} %, rest = MFMA / LDS / DMA issue {(p1e - vm - bar).mean() / life * 100:5.1f} %)")
    print(f"    phase 2 {(p2e - p1e).mean() / life * 100:5.1f} %  (pair stage + DMA wait {p2w.mean() / life * 100:5.1f} %, "
          f"sampling + MFMA {(p2e - p1e - p2w).mean() / life * 100:5.1f} %)")
    print(f"    epilogue {(end - p2e).mean() / life * 100:5.1f} %;  per K step: vm wait {vm.mean() / 36:.0f}, barrier "
          f"{bar.mean() / 36:.0f}, rest {(p1e - vm - bar).mean() / 36:.0f} cycles; per pair: stage+wait {p2w.mean() / 4:.0f}, "
          f"rest {(p2e - p1e - p2w).mean() / 4:.0f} cycles")
