"""Round-5 review item 4: why the tap-pipelined fused DCN_sep (DCNSEP_TAPPIPE=1) gave batch-dependent C0 outputs.

Runs the C0 window batched and its pairs alone (tests/test_gpu_configs.py::test_c0_window_pairs_equal_single_pairs)
under the library STIF_HIP_LIB points at, and reports: the model's f16x3 range re-runs (a non-finite value in a
fused launch's range sum makes the model re-run the whole call in fp32), per fused launch the status word and
whether a re-run of the same launch is bit-identical, and the batched-vs-single comparison with the range guard
off (range_check='off')."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import stif_pkg  # noqa: E402

stif = stif_pkg.load()
print("library:", stif._lib.LIB_PATH)
sd = {k: torch.from_numpy(v) for k, v in stif.weights.make_state_dict(0).items()}


def synth(first, count, H, W):
    out = torch.empty(count, 3, H, W)
    for i in range(count):
        out[i] = torch.rand(3, H, W, generator=torch.Generator().manual_seed(1234 + first + i))
    return out.cuda()


fr = synth(0, 7, 128, 128)
for rc in (() if os.environ.get("QUICK") else ("rerun", "off")):
    m = stif.LunaTokis(64, 6, 8, 5, 40, mfma="f16x3", range_check=rc)
    m.load_state_dict(sd, strict=True)
    m.eval()
    with torch.no_grad():
        m.gen_feat_window(fr)
        win = m.decoding([torch.tensor([[0.5]])])[0].clone()
        r_win = m.range_reruns
        res = []
        for p in range(6):
            r0 = m.range_reruns
            one = m(torch.stack([fr[p], fr[p + 1]])[None], [0.5])[0]
            res.append((p, bool(torch.equal(win[p:p + 1], one)), float((win[p:p + 1] - one).abs().max()),
                        m.range_reruns - r0, bool(torch.isfinite(one).all())))
    print(f"range_check={rc}: window range re-runs {r_win}, window finite {bool(torch.isfinite(win).all())}")
    for r in res:
        print(f"  pair {r[0]}: equal {r[1]} max|diff| {r[2]:.3e} re-runs {r[3]} finite {r[4]}")

# per fused launch: status word, bit-identical re-runs, non-finite outputs
ops = stif.ops
orig = ops.dcn_sep
rows = []


def traced(groups, epi=0, status=None):
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    orig(groups, epi=epi, status=st)
    ref = [g["out"].clone() for g in groups]
    same, stats = [], [int(st.item())]
    diffs = []
    for _ in range(3):
        st2 = torch.zeros(1, dtype=torch.int32, device="cuda")
        g2 = [dict(g, out=torch.full_like(g["out"], float("nan"))) for g in groups]
        orig(g2, epi=epi, status=st2)
        same.append(all(torch.equal(a["out"], b) for a, b in zip(g2, ref)))
        if os.environ.get("DIFF"):
            for gi, (a, b) in enumerate(zip(g2, ref)):
                d = (a["out"] - b).abs()
                if bool((d > 0).any()):
                    nz = (d > 0).nonzero()
                    H, W = b.shape[1], b.shape[2]
                    diffs.append(f"g{gi}: {int(nz.shape[0])} el, max|d| {float(d.max()):.3e} (max|out| {float(b.abs().max()):.2e}), "
                                 f"max rel {float((d / b.abs().clamp_min(1e-6)).max()):.2e}; ch<32 {int((nz[:, 3] < 32).sum())}, "
                                 f"row%4 {torch.bincount(nz[:, 1] % 4, minlength=4).tolist()}, x%32<8 {int((nz[:, 2] % 32 < 8).sum())}, "
                                 f"border(<=2 px) {int(((nz[:, 1] <= 2) | (nz[:, 1] >= H - 3) | (nz[:, 2] <= 2) | (nz[:, 2] >= W - 3)).sum())}, "
                                 f"items {torch.bincount(nz[:, 0], minlength=b.shape[0]).tolist()}")
        stats.append(int(st2.item()))
    nonfin = sum(int((~torch.isfinite(r)).sum()) for r in ref)
    rows.append((len(groups), tuple(groups[0]["out"].shape), stats, same, nonfin, diffs[:4]))
    if status is not None and stats[0]:
        status.fill_(1)


ops.dcn_sep = traced
m = stif.LunaTokis(64, 6, 8, 5, 40, mfma="f16x3", range_check="off")
m.load_state_dict(sd, strict=True)
try:
    with torch.no_grad():
        m.gen_feat_window(fr)
finally:
    ops.dcn_sep = orig
for r in rows:
    print(f"  launch groups={r[0]} out={r[1]} status(run, reruns)={r[2]} identical={r[3]} nonfinite={r[4]}")
    for d in r[5]:
        print("      diff", d)
