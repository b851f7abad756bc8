"""Where a k_dec2q wave's time goes (DEC_TRACE build): s_memtime sums per wave over the C0 window's stage-2 launch --
gathers (the flow load and the four bilinear gathers, waits included), segment-barrier waits, the layer-2/3 span."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import stif_pkg  # noqa: E402

stif = stif_pkg.load()
print("library:", stif._lib.LIB_PATH)
h = stif._lib.lib()
h.stif_dec_trace_set.argtypes = [ctypes.c_void_p]
sd = {k: torch.from_numpy(v) for k, v in stif.weights.make_state_dict(0).items()}
fr = torch.empty(7, 3, 128, 128)
for i in range(7):
    fr[i] = torch.rand(3, 128, 128, generator=torch.Generator().manual_seed(1234 + i))
m = stif.LunaTokis(64, 6, 8, 5, 40, mfma="f16x3", range_check="off")
m.load_state_dict(sd, strict=True)
m.eval()
NW, total = 8, 6 * 512 * 512
waves = (total + NW * 16 - 1) // (NW * 16) * NW
with torch.no_grad():
    m.gen_feat_window(fr.cuda())
    for rep in range(3):
        tr = torch.zeros(waves * 8, dtype=torch.int32, device="cuda")
        h.stif_dec_trace_set(tr.data_ptr())
        m.decoding([torch.tensor([[0.5]])])
        torch.cuda.synchronize()
        h.stif_dec_trace_set(None)
        t = (tr.view(waves, 8).cpu().to(torch.int64) & 0xFFFFFFFF).double()
        life, g, b, l23 = t[:, 0], t[:, 1], t[:, 2], t[:, 3]
        print(f"rep {rep}: mean wave life {life.mean() / 1e3:.1f} k-ticks; gathers {g.mean() / life.mean() * 100:5.1f} %, "
              f"segment-barrier waits {b.mean() / life.mean() * 100:5.1f} %, layers 2/3 span {l23.mean() / life.mean() * 100:5.1f} % "
              f"(of which barrier waits ~{(b.mean() * 8 / 10) / life.mean() * 100:4.1f} %); layers 2/3 per segment "
              f"{l23.mean() / 8 / 1e3:.2f} k-ticks")
