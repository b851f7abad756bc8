"""Where a ResidualBlock conv1 (k_wino<0, 2, 1>, f16x3) wave's time goes (WINO_TRACE build): per wave over the last
such launch of a C0 window -- phase-end waits (vmcnt(8) + barrier), the epilogue (output-transform LDS exchange, bias,
ReLU, stores), the rest (staging issue, transform, split, MFMA)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import stif_pkg  # noqa: E402

stif = stif_pkg.load()
print("library:", stif._lib.LIB_PATH)
h = stif._lib.lib()
h.stif_wino_trace_set.argtypes = [ctypes.c_void_p]
sd = {k: torch.from_numpy(v) for k, v in stif.weights.make_state_dict(0).items()}
fr = torch.empty(7, 3, 128, 128)
for i in range(7):
    fr[i] = torch.rand(3, 128, 128, generator=torch.Generator().manual_seed(1234 + i))
m = stif.LunaTokis(64, 6, 8, 5, 40, mfma="f16x3", range_check="off", trunk_lanes=1)
m.load_state_dict(sd, strict=True)
m.eval()
with torch.no_grad():
    for rep in range(3):
        tr = torch.zeros(512 * 4 * 4, dtype=torch.int32, device="cuda")
        h.stif_wino_trace_set(tr.data_ptr())
        m.gen_feat_window(fr.cuda())
        torch.cuda.synchronize()
        h.stif_wino_trace_set(None)
        t = (tr.view(-1, 4).cpu().to(torch.int64) & 0xFFFFFFFF).double()
        t = t[t[:, 3] > 0]
        life, wait, epi, nt = t[:, 0], t[:, 1], t[:, 2], t[:, 3]
        print(f"rep {rep}: {t.shape[0]} waves, {nt.mean():.1f} tiles per wave, mean life {life.mean() / 1e3:.1f} k-ticks "
              f"({life.mean() / nt.mean() / 1e3:.2f} per tile): phase-end waits {wait.mean() / life.mean() * 100:5.1f} %, "
              f"epilogue {epi.mean() / life.mean() * 100:5.1f} %, rest {(life - wait - epi).mean() / life.mean() * 100:5.1f} %")
