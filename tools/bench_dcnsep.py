"""Microbenchmark of DCN_sep at one map shape: the fused kernel (k_dcn_sep, FUSED=1) or the two-kernel
path (k_wino_om -> 216-ch map -> k_dcn, FUSED=0).  N maps of HW x HW, offset-branch features N(0, 1) x
OSCALE / 23 (the generated conv_offset_mask weights give offsets of std ~23 px per unit feature, so
OSCALE ~ the offsets' std in px).  Prints the average launch time (HIP events)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import stif_pkg  # noqa: E402

N, HW = int(os.environ.get("N", 48)), int(os.environ.get("HW", 128))
OSCALE = float(os.environ.get("OSCALE", 2.0))
FUSED = int(os.environ.get("FUSED", 1))
REPS = int(os.environ.get("REPS", 20))
stif = stif_pkg.load()
L, ops = stif._lib, stif.ops
sd = stif.weights.make_state_dict(0)
p = "pcd_align.L1_dcnpack_1"
g = torch.Generator(device="cuda").manual_seed(0)
fea = torch.randn(N, HW, HW, 64, device="cuda", generator=g) * (OSCALE / 23.0)
inp = torch.randn(N, HW, HW, 64, device="cuda", generator=g)
out = torch.empty_like(inp)
core = ops.pack_conv(sd[p + ".weight"], sd[p + ".bias"], (L.PACK_DCNPAIR if FUSED else L.PACK_PLAIN) | L.PACK_F16X3)
if FUSED:
    om = ops.pack_conv(sd[p + ".conv_offset_mask.weight"], sd[p + ".conv_offset_mask.bias"],
                       L.PACK_DCNSEP | L.PACK_F16X3, range_fallback=False)
    run = lambda: ops.dcn_sep([dict(om_layer=om, layer=core, fea=fea, inp=inp, out=out)])
else:
    omw = ops.pack_conv(sd[p + ".conv_offset_mask.weight"], sd[p + ".conv_offset_mask.bias"],
                        L.PACK_WINO_OFFMASK | L.PACK_F16X3)
    omap = torch.empty(N, HW, HW, 216, device="cuda")

    def run():
        ops.conv2d([dict(layer=omw, in0=fea, out=omap)], epi=L.EPI_OFFMASK)
        ops.dcn([dict(layer=core, inp=inp, offmask=omap, out=out)])
for _ in range(3):
    run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(REPS):
    run()
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / REPS * 1e3
px = N * HW * HW
print(f"{'fused k_dcn_sep' if FUSED else 'k_wino_om + k_dcn'}: N={N} HW={HW} OSCALE={OSCALE}: {us:.1f} us per DCN_sep "
      f"({px / us:.1f} Mpx/s, {2 * 280 * 576 * px / us * 1e-6:.1f} TFLOP/s)")
