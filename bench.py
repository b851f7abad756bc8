"""Benchmark of the STIF LunaTokis forward on MI355X (BASELINE.json metric).

Workload (default c0 = the metric's own config, BASELINE.json "7x128x128 -> 4x"): a synthetic
7-frame 3x128x128 window = 6 adjacent pairs, 4x spatial, one interpolated time t = 0.5 -> 6 x
512x512 output pixels per GPU per step.  A step = the encoder over the window (per-frame encoder,
PCD alignment, Bi-Deformable-ConvLSTM, 40-block trunk) + the implicit decoder, with inputs already
resident in HBM.

Multi-GPU (one process per GPU, RCCL): c0-c2 are weak-scaled -- rank r owns frames [6r, 6r+6] of
one (6N+1)-frame sequence -- and c3 / c4 strong-scaled -- one fixed sequence (64 frames at 720p /
9 frames at 1080p) split into contiguous pair shards (8,8,...,7 at 8 ranks).  Neighbouring shards
share one boundary frame; its per-frame encoder features come from rank r+1 by a point-to-point
halo exchange inside the timed step (--halo recompute recomputes them instead).  Rank 0 prints one
JSON line; at N = 1 it also carries the CPU baseline, a parity check of the same pair against the
CPU oracle (max error, PSNR), the fp32-MFMA value and the C1 / C2 lines.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c0|c1|c2|c3|c4]
"""
import argparse
import glob
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

BASE = json.load(open(os.path.join(REPO, "BASELINE.json")))
CONFIGS = {
    # name: (frames, H, W, (HH, WW) per LR (H, W), times, scaling); weak: frames per rank
    "c0": (7, 128, 128, 4.0, [0.5], "weak"),
    "c1": (7, 256, 256, 4.0, [0.5], "weak"),
    "c2": (7, 540, 960, 4.0, [0.25, 0.5, 0.75], "weak"),
    "c3": (64, 720, 1280, 4.0, [0.0, 0.5], "strong"),
    "c4": (9, 1080, 1920, 2.5, [0.0, 0.25, 0.5, 0.75], "strong"),
}
# the reference's own CPU path (torch 2.10 + mkldnn, 8 threads, the survey container; BASELINE.md
# section 2): one 128x128 pair -> 512x512 at one t in 3.69 s
REF_TORCH_CPU_MPIX_S = 0.0711
FP32_PEAK_TFLOPS = 157.3   # MI355X dense fp32 MFMA (MI355X_MICROARCH.md, chip-level parameters)
# f16x3 operand mode: one fp32-class product = 3 products on the dense fp16 MFMA pipe (~2.5 PF/s)
F16X3_PEAK_TFLOPS = 2500.0 / 3.0
WINO_GAIN = 36.0 / 16.0    # F(2x2,3x3): 16 transformed-domain MACs per 36 direct MACs
EPI_NAMES = {0: "NONE", 1: "LRELU", 2: "RELU", 3: "RES", 4: "OFFMASK", 5: "LSTM"}


def kernel_desc(kind, mfma="f32"):
    """(kernel name as rocprof shows it, description, peak in algorithmic TFLOP/s) of a launch kind."""
    f16 = mfma == "f16x3"
    if kind and kind[-1] == "lane":   # a launch on a side stream (KernelTimer)
        kind = kind[:-1]
    if kind[0] == "wino":
        _, ks, s, epi, in1, cout = kind
        if f16 and epi == 4 and not in1:
            return ("k_wino_om<4>", f"3x3 64->{cout} conv, EPI_OFFMASK, Winograd F(2x2,3x3) on split-fp16 MFMA, all "
                    "couts per tile (3 fp16 products per fp32-class product); algorithmic = direct-conv FLOPs, peak = "
                    "fp16 MFMA dense peak / 3 x 36/16", F16X3_PEAK_TFLOPS * WINO_GAIN)
        if f16:
            return (f"k_wino<{in1}, {epi}, 1>", f"3x3 {64 * (2 if in1 else 1)}->{cout} conv, EPI_{EPI_NAMES[epi]}, "
                    "Winograd F(2x2,3x3) on split-fp16 MFMA (3 fp16 products per fp32-class product); algorithmic = "
                    "direct-conv FLOPs, peak = fp16 MFMA dense peak / 3 x 36/16", F16X3_PEAK_TFLOPS * WINO_GAIN)
        return (f"k_wino<{in1}, {epi}, 0>", f"3x3 {64 * (2 if in1 else 1)}->{cout} conv, EPI_{EPI_NAMES[epi]}, "
                f"Winograd F(2x2,3x3) on fp32 MFMA; algorithmic = direct-conv FLOPs, peak = fp32 MFMA peak x 36/16",
                FP32_PEAK_TFLOPS * WINO_GAIN)
    if kind[0] == "conv":
        _, ks, s, epi, in1, cout = kind
        return (f"k_conv<{ks}, {s}, ...>", f"{ks}x{ks}/s{s} conv -> {cout}, in1 mode {in1}, EPI_{EPI_NAMES[epi]}, "
                "direct implicit GEMM on fp32 MFMA", FP32_PEAK_TFLOPS)
    if kind[0] == "dcnsep":
        return (f"k_dcn_sep<{kind[1]}>", "fused DCN_sep: offset/mask conv (direct, split-fp16 MFMA, offsets kept in the "
                "accumulators) + sigmoid + modulated deformable conv; algorithmic = both convolutions' FLOPs, peak = fp16 "
                "MFMA dense peak / 3", F16X3_PEAK_TFLOPS)
    if kind[0] == "dcn":
        if f16:
            return (f"k_dcn<{kind[1]}, 1>", "fused modulated deformable conv, split-fp16 MFMA (peak = fp16 MFMA / 3)",
                    F16X3_PEAK_TFLOPS)
        return (f"k_dcn<{kind[1]}, 0>", "fused modulated deformable conv", FP32_PEAK_TFLOPS)
    if f16:
        # stage 2 of LunaTokis.decoding in f16x3 is k_dec2q (16 pixels per wave); k_dec2 runs the fp32 and the
        # high-resolution-image variants (decoder.hip, stif_dec_stage2_ex)
        name = "k_dec2q" if kind[0] == "dec2" else f"k_{kind[0]}"
        return (name, "SIREN decoder stage, split-fp16 MFMA (peak = fp16 MFMA / 3)", F16X3_PEAK_TFLOPS)
    return (f"k_{kind[0]}", "SIREN decoder stage", FP32_PEAK_TFLOPS)


class KernelTimer:
    """HIP-event timing of the launches of one kernel variant (or of all, kind=None), on the launch
    stream: every ``every``-th launch of the variant (default all; every = 4 measured 91.5 vs 91.1
    Mpix/s for all, within the box's noise, so the headline times every launch)."""

    def __init__(self, kind, every=1):
        self.kind = kind
        self.every = max(1, int(every))
        # launches issued on another stream than this one (the model's trunk lanes) overlap that stream's
        # kernels, so their event intervals include the overlap: they are kept apart (kind + ("lane",)) and
        # never picked as the dominant kernel
        self.main = torch.cuda.current_stream() if torch.cuda.is_available() else None
        self.seen = 0
        self.nbytes = []
        self.rec = []
        self.all = []
        self._cur = None

    kinds = None

    def begin(self, kind, flops, nbytes=0.0):
        base = tuple(kind)
        if self.main is not None and torch.cuda.current_stream() != self.main:
            kind = base + ("lane",)
        # a named kind is timed on whichever stream it is launched (the events record on that stream)
        if self.kind is None or kind == self.kind or base == tuple(self.kind):
            self.seen += 1
            if (self.seen - 1) % self.every:
                return
            if self.kinds is None:
                self.kinds = []
            self.kinds.append(kind)
            self.nbytes.append(nbytes)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            self._cur = (e0, e1, flops)

    def end(self):
        if self._cur is not None:
            self._cur[1].record()
            self.rec.append(self._cur)
            self._cur = None

    def per_kind(self):
        """kind -> [launches, total ms, total FLOP, total algorithmic bytes]"""
        agg = {}
        for (a, b, f), k, nb in zip(self.rec, self.kinds, self.nbytes):
            d = agg.setdefault(k, [0, 0.0, 0.0, 0.0])
            d[0] += 1
            d[1] += a.elapsed_time(b)
            d[2] += f
            d[3] += nb
        return agg

    def dominant(self):
        """the launch kind with the largest total time (launches on the main stream; run_config probes a
        single-stream step, so every launch is there; with none, any stream; ("none",) for an empty probe)"""
        agg = self.per_kind()
        main = {k: v for k, v in agg.items() if k[-1] != "lane"} or {k[:-1] if k[-1] == "lane" else k: v
                                                                    for k, v in agg.items()}
        return max(main.items(), key=lambda kv: kv[1][1])[0] if main else ("none",)

    def report(self):
        """per-kind launches / avg us / TFLOP/s (all-kinds mode); kinds tagged 'lane' ran on a side stream
        beside another stream's kernels (their intervals include the overlap)"""
        agg = self.per_kind()
        for k, (nl, ms, fl, _) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            print(f"  {str(k):40s} {nl:5d} launches {ms / nl * 1e3:9.1f} us avg {fl / (ms * 1e-3) / 1e12:7.1f} TFLOP/s"
                  f"  {ms:8.2f} ms total", file=sys.stderr)

    def summary(self):
        ms = [a.elapsed_time(b) for a, b, _ in self.rec]
        fl = [f for _, _, f in self.rec]
        nb = self.nbytes[:len(ms)]
        return (len(ms), float(np.mean(ms)) if ms else 0.0, float(np.mean(fl)) if fl else 0.0,
                float(np.mean(nb)) if nb else 0.0)


HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E (MI355X_MICROARCH.md)


def roofline(kname, kdesc, dom, peak_tflops, achieved_tflops, avg_ms, avg_flops, avg_bytes, n_launch, traffic,
             n_timed=None):
    """Roofline record of the dominant kernel.  The bound is the kernel's algorithmic intensity (direct
    FLOPs / algorithmic HBM bytes per launch) against the ridge of the pipe it runs on (peak FLOP/s /
    8 TB/s): below the ridge it is HBM-bound and `achieved` is algorithmic GB/s, above it MFMA-bound and
    `achieved` is algorithmic TFLOP/s; both views are kept."""
    gbps = avg_bytes / (avg_ms * 1e-3) / 1e9 if avg_ms and avg_bytes else 0.0
    intensity = avg_flops / avg_bytes if avg_bytes else float("inf")
    ridge = peak_tflops * 1e12 / (HBM_PEAK_GBPS * 1e9)
    hbm = intensity < ridge
    rec = {"bound": "hbm" if hbm else "mfma", "kernel": f"{kname} ({kdesc})", "kind": list(dom)}
    if hbm:
        rec.update(achieved=round(gbps, 1), peak=HBM_PEAK_GBPS, unit="GB/s", frac=round(gbps / HBM_PEAK_GBPS, 4))
    else:
        rec.update(achieved=round(achieved_tflops, 3), peak=round(peak_tflops, 2), unit="TFLOP/s",
                   frac=round(achieved_tflops / peak_tflops, 4))
    rec.update(traffic=traffic, launches=n_launch, timed_launches=n_launch if n_timed is None else n_timed,
               avg_launch_us=round(avg_ms * 1e3, 2),
               flops_per_launch=avg_flops, algorithmic_bytes_per_launch=round(avg_bytes),
               intensity_flop_per_byte=round(intensity, 1), ridge_flop_per_byte=round(ridge, 1),
               mfma_view={"achieved": round(achieved_tflops, 3), "peak": round(peak_tflops, 2), "unit": "TFLOP/s",
                          "frac": round(achieved_tflops / peak_tflops, 4)},
               hbm_view={"achieved": round(gbps, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(gbps / HBM_PEAK_GBPS, 4)})
    return rec


def kernel_table(probe, mfma, top=4):
    """The `top` launch kinds of one step by total time (HIP events on the launch stream, one untimed
    step, single-stream): launches, avg us, share of the step's kernel time, and each kind's roofline fraction on the
    bound its intensity picks (roofline())."""
    # launches on the model's side streams (the trunk lanes) overlap each other, so their event intervals
    # are not kernel times: left out here (their kernel times are in the rocprof summary)
    agg = {k: v for k, v in probe.per_kind().items() if k[-1] != "lane"}
    tot = sum(v[1] for v in agg.values()) or 1.0
    out = []
    for k, (nl, ms, fl, nb) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        kname, kdesc, peak = kernel_desc(k, mfma)
        tf = fl / (ms * 1e-3) / 1e12 if ms else 0.0
        r = roofline(kname, kdesc, k, peak, tf, ms / nl, fl / nl, nb / nl, nl, None)
        out.append({"kind": list(k), "kernel": kname, "launches": nl, "avg_us": round(ms / nl * 1e3, 1),
                    "share": round(ms / tot, 3), "bound": r["bound"], "frac": r["frac"],
                    "hbm_frac": r["hbm_view"]["frac"], "mfma_frac": r["mfma_view"]["frac"]})
    return out


def hot_path_kernels(probe, mfma):
    """The north star's DCNv2 + implicit-decoder kernels, from the last warm-up step (HIP events on
    the launch stream): per kind avg time and TFLOP/s; for the DCN core also its algorithmic HBM
    bytes (input + offset/mask + output per pixel) as GB/s and fraction of the HBM peak; for the
    decoder stages the fraction of the MFMA peak of their operand mode."""
    dec_peak = 2500.0 / 3 if mfma == "f16x3" else 157.3
    out = {}
    for k, (nl, ms, fl, nb) in probe.per_kind().items():
        if k[0] not in ("dcn", "dcnsep", "dec1", "dec2") or not ms:
            continue
        e = {"kernel": kernel_desc(k, mfma)[0], "launches": nl, "avg_us": round(ms / nl * 1e3, 1),
             "tflops": round(fl / (ms * 1e-3) / 1e12, 1)}
        if nb:
            gbps = nb / (ms * 1e-3) / 1e9
            e.update(hbm_gbps_algorithmic=round(gbps, 1), hbm_frac=round(gbps / HBM_PEAK_GBPS, 3))
        if k[0] != "dcn":
            e["mfma_frac"] = round(fl / (ms * 1e-3) / 1e12 / dec_peak, 3)   # dcnsep / decoder: split-fp16 pipe
        out["_".join(str(x) for x in k)] = e
    return out


def synth_frames(first, count, H, W, device):
    """Deterministic synthetic frames: frame k = U[0,1) from a generator seeded by its global index."""
    out = torch.empty(count, 3, H, W)
    for i in range(count):
        g = torch.Generator().manual_seed(1234 + first + i)
        out[i] = torch.rand(3, H, W, generator=g)
    return out.to(device)


# moving gratings (synthetic input (ii)): channel c of frame k is
# 0.5 + 0.5 sin(2 pi (F_c x + G_c y) + PHI_c + V_c k), x / y in LR pixel units -- real, known motion,
# and a ground truth at any HR pixel and continuous time (gratings_gt)
GRATING_F = (0.05, 0.07, 0.03)
GRATING_G = (0.04, -0.02, 0.06)
GRATING_PHI = (0.0, 1.0, 2.0)
GRATING_V = (0.3, -0.2, 0.25)


def _grating(y, x, k):
    return np.stack([0.5 + 0.5 * np.sin(2 * np.pi * (GRATING_F[c] * x + GRATING_G[c] * y) + GRATING_PHI[c]
                                        + GRATING_V[c] * k) for c in range(3)])


def gratings(first, count, H, W):
    """frames [count, 3, H, W] (float32) of the moving gratings, frames first .. first + count - 1"""
    y, x = np.meshgrid(np.arange(H, dtype=np.float64), np.arange(W, dtype=np.float64), indexing="ij")
    return np.stack([_grating(y, x, first + i) for i in range(count)]).astype(np.float32)


def gratings_gt(k0, t, H, W, HH, WW):
    """ground truth [3, HH, WW] of the pair (k0, k0 + 1) at time t: the pattern at the HR pixel centres
    ((X + 0.5) W / WW - 0.5 in LR units) and frame time k0 + t"""
    yy = (np.arange(HH) + 0.5) * (H / HH) - 0.5
    xx = (np.arange(WW) + 0.5) * (W / WW) - 0.5
    y, x = np.meshgrid(yy, xx, indexing="ij")
    return _grating(y, x, k0 + t)


def _threads():
    try:
        from threadpoolctl import threadpool_info
        return max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    except Exception:
        return int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


CPU_SAMPLE = 96   # LR crop of the CPU-baseline sample (FLOP per output pixel does not depend on it)


def _oracle_timed(threads=None):
    """time the numpy oracle on the sample pair (frames 0-1 of the window cropped to CPU_SAMPLE^2,
    4x, t = 0.5); threads=None: the process's BLAS pool as configured"""
    from oracle import stif_oracle as O
    sd = __import__("stif_pkg").load().weights.make_state_dict(seed=0)
    x = np.ascontiguousarray(synth_frames(0, 2, 128, 128, "cpu")[:, :, :CPU_SAMPLE, :CPU_SAMPLE].numpy()[None])
    ctx = None
    if threads:
        from threadpoolctl import threadpool_limits
        ctx = threadpool_limits(threads)
    t0 = time.perf_counter()
    O.forward(x, [0.5], sd, dtype=np.float32)
    dt = time.perf_counter() - t0
    if ctx is not None:
        ctx.unregister()
    return dt


def _pinned_child():
    """child process: pinned to CPUs 0-7 (as taskset -c 0-7), 8 BLAS threads; prints the seconds"""
    os.sched_setaffinity(0, range(8))
    print(json.dumps({"s": _oracle_timed(8)}), flush=True)


def cpu_baseline():
    """The numpy oracle (fp32) on a bounded sample of the same workload -- one pair of the window
    cropped to CPU_SAMPLE x CPU_SAMPLE LR pixels, 4x, t = 0.5 -- on the process's BLAS pool (its thread
    count stated as `cores`, next to the host's CPU count and the process affinity), and again
    in a child process pinned to 8 cores (the survey container's count, where the reference's own torch
    CPU path was timed).  The child is a fresh interpreter that never touches the GPU."""
    import subprocess
    dt = _oracle_timed()
    mpix = 16 * CPU_SAMPLE * CPU_SAMPLE / 1e6
    pinned = None
    try:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--cpu-pinned-child"], capture_output=True,
                           text=True, timeout=300, env=dict(os.environ, HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="8"))
        pinned = json.loads(r.stdout.strip().splitlines()[-1])["s"]
    except Exception as e:  # noqa: BLE001 -- the pinned leg is informational
        print(f"pinned CPU baseline failed: {e}", file=sys.stderr)
    sample = (f"1 pair (frames 0-1) of the window cropped to {CPU_SAMPLE}x{CPU_SAMPLE} -> {4 * CPU_SAMPLE}x"
              f"{4 * CPU_SAMPLE}, t=0.5, numpy fp32 restatement (oracle/stif_oracle.py)")
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    nthr = _threads()
    rec = {"value": round(mpix / dt, 6), "unit": "Mpix/s", "cores": nthr, "kind": "port",
           "sample": f"{sample}, {dt:.1f} s on {nthr} BLAS threads",
           "threads_note": "the BLAS pool the process was given (OMP_NUM_THREADS: the GPU box's per-GPU CPU share, "
                           "16, which the pool's rules say to leave as set), not every CPU of the host",
           "cpu_model": cpu_model(), "host_cpus": os.cpu_count(), "affinity_cpus": affinity,
           "pinned_8_cores": None if pinned is None else {
               "value": round(mpix / pinned, 6), "unit": "Mpix/s", "cores": 8, "seconds": round(pinned, 2),
               "how": "child process, sched_setaffinity CPUs 0-7 (as taskset -c 0-7), 8 BLAS threads"},
           "reference_torch_cpu": {"value": REF_TORCH_CPU_MPIX_S, "unit": "Mpix/s", "cores": 8,
                                   "note": "the reference's own torch CPU path (Sakuya_arch_test.LunaTokis, torch 2.10 "
                                           "+ mkldnn, 8 threads), one 128x128 pair -> 512x512 at t=0.5, measured in the "
                                           "survey container (BASELINE.md section 2); not re-run on the GPU box, where "
                                           "the reference is absent"}}
    return rec


def _psnr(x, gt):
    m = float(np.mean((np.asarray(x, np.float64) - gt) ** 2))
    return 10 * np.log10(1.0 / m) if m > 0 else float("inf")


def parity_record(out, ref, gt, what, gt_desc):
    """GPU output vs the reference model's own output on the same pair (fixture made by running the
    reference here, tests/golden/make_golden.py): max errors, the north star's elementwise bar
    (|a - b| <= 1e-4 |b| + 1e-6), PSNR vs the reference, and the PSNR criterion: both PSNRs against a
    ground truth (calc_psnr form, myutils.py:269-271, data range 1) and their difference."""
    a = np.asarray(out, np.float64)
    b = np.asarray(ref, np.float64)
    d = np.abs(a - b)
    ok = d <= 1e-4 * np.abs(b) + 1e-6
    mse = float(np.mean(d ** 2))
    return {"pair": what, "vs": "the reference model's own output (tests/golden)", "max_abs_err": float(d.max()),
            "max_err_rel_to_max_ref": float(d.max() / np.abs(b).max()),
            "elementwise_rtol1e-4_atol1e-6_frac": float(ok.mean()),
            "psnr_vs_reference_db": round(10 * np.log10(1.0 / mse), 2) if mse > 0 else None,
            "psnr_gpu_vs_gt_db": round(_psnr(a, gt), 6), "psnr_reference_vs_gt_db": round(_psnr(b, gt), 6),
            "psnr_delta_db": abs(_psnr(a, gt) - _psnr(b, gt)), "gt": gt_desc}


def parity_records(stif, sd, device, mfma):
    """the metric's pair (U[0,1) frames 0-1 at 128x128) and the moving-grating pair, 4x, t = 0.5"""
    m = stif.LunaTokis(64, 6, 8, 5, 40, device=device, mfma=mfma)
    m.load_state_dict(sd, strict=True)
    recs = []
    gd = os.path.join(REPO, "tests", "golden")
    for name, what in (("c0_pair_128", "frames 0-1 of the C0 window (U[0,1), 128x128)"),
                       ("gratings_128", "moving gratings, frames 0-1 (128x128)")):
        g = np.load(os.path.join(gd, name + ".npz"))
        with torch.no_grad():
            out = m(torch.from_numpy(g["x"]).to(device), [0.5])[0][0].cpu().numpy()
        ref = g["out"]
        if name == "gratings_128":
            gt, desc = gratings_gt(0, 0.5, 128, 128, 512, 512), "analytic moving-grating pattern at t = 0.5 (gratings_gt)"
        else:
            gt = np.round(np.clip(ref.astype(np.float64), 0, 1) * 255) / 255
            desc = "the reference output quantised to 8-bit levels (the harness's uint8 output precision)"
        recs.append(parity_record(out, ref, gt, what, desc))
    return recs


def run_config(stif, sd, cfg, args, world, rank, device, dist, mfma, trace_dom=True):
    """Warm up, time args.steps steps of one config; returns (elapsed s, probe, timer, model, frames, tq,
    out_pix per step over all ranks)."""
    nframes, H, W, scale, times, scaling = CONFIGS[cfg]
    P = stif.parallel
    if scaling == "weak":
        pairs = nframes - 1
        total_frames = pairs * world + 1
        shards = P.pair_shards(total_frames, world)
    else:
        total_frames = nframes
        shards = P.pair_shards(total_frames, world)
    a, b = shards[rank]
    total_pairs = total_frames - 1
    HH, WW = int(round(H * scale)), int(round(W * scale))
    model = stif.LunaTokis(64, 6, 8, 5, 40, device=device, mfma=mfma, lanes=args.lanes, trunk_lanes=args.trunk_lanes,
                           dec_lanes=args.dec_lanes, lstm_lanes=args.lstm_lanes, pcd_streams=args.pcd_streams,
                           range_check=getattr(args, "range_check", "rerun"), fused_dcn=bool(args.fused_dcn))
    model.load_state_dict(sd, strict=True)
    frames = synth_frames(a, b - a, H, W, device) if b > a else None
    tq = [torch.tensor([[t]], device=device) for t in times]
    exchange = args.halo == "exchange"

    def step():
        # every rank calls gen_feat_shard (an empty shard only joins its first-call barrier)
        P.gen_feat_shard(model, frames, rank, world, shards=shards, exchange=exchange)
        if frames is None:
            return None
        return model.decoding(tq, None if scale == 4.0 else (HH, WW))

    # the kernel-table probe (the last warm-up step) runs every launch on one stream: outputs are bit-identical
    # for any lane setting, and HIP-event intervals of launches overlapping on side streams are not kernel times
    knobs = ("lanes", "trunk_lanes", "dec_lanes", "lstm_lanes", "pcd_streams")
    with torch.no_grad():
        probe = KernelTimer(None)
        for i in range(max(1, args.warmup)):
            step()
        if trace_dom:   # one more untimed step, single-stream, traced
            keep = {k: getattr(model, k) for k in knobs}
            for k in knobs:
                setattr(model, k, 1)
            stif.ops.TRACE = probe
            try:
                step()
            finally:
                stif.ops.TRACE = None
                for k, v in keep.items():
                    setattr(model, k, v)
            step()   # and the timed configuration once more, so the timed region starts warm
        stif.ops.TRACE = None
        torch.cuda.synchronize()
        timer = KernelTimer(probe.dominant() if (trace_dom and probe.rec) else ("none",), every=args.time_every)
        stif.ops.TRACE = timer if trace_dom else None
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        stif.ops.TRACE = None
    out_pix = total_pairs * len(times) * HH * WW
    return elapsed, probe, timer, model, frames, tq, out_pix


def host_inclusive(stif, sd, cfg, device, mfma, steps=3):
    """End to end with the PCIe legs: the window's frames start in pinned host memory and every output
    frame is copied back to pinned host memory inside the timed region (H2D + encoder + decoder + D2H);
    not the headline value, whose inputs are resident in HBM."""
    nframes, H, W, scale, times, _ = CONFIGS[cfg]
    HH, WW = int(round(H * scale)), int(round(W * scale))
    m = stif.LunaTokis(64, 6, 8, 5, 40, device=device, mfma=mfma)
    m.load_state_dict(sd, strict=True)
    host = synth_frames(0, nframes, H, W, "cpu").pin_memory()
    outs = [torch.empty(nframes - 1, 3, HH, WW).pin_memory() for _ in times]
    tq = [torch.tensor([[t]], device=device) for t in times]

    def step():
        fr = host.to(device, non_blocking=True)
        m.gen_feat_window(fr)
        for o, d in zip(outs, m.decoding(tq, None if scale == 4.0 else (HH, WW))):
            o.copy_(d, non_blocking=True)

    with torch.no_grad():
        step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    px = (nframes - 1) * len(times) * HH * WW
    return {"value": round(px * steps / el / 1e6, 4), "unit": "Mpix/s", "ms_per_step": round(el / steps * 1e3, 3),
            "steps": steps, "h2d_bytes": host.numel() * 4, "d2h_bytes": sum(o.numel() for o in outs) * 4,
            "note": "frames H2D from pinned host memory and outputs D2H to pinned host memory inside the timed region"}


def main():
    if sys.argv[1:] == ["--cpu-pinned-child"]:
        _pinned_child()
        return
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c0", choices=sorted(CONFIGS))
    ap.add_argument("--halo", default="exchange", choices=["exchange", "recompute"],
                    help="boundary frame of a shard: features from rank r+1 (P2P) or recomputed")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="N=1: skip the fp32-MFMA and C1/C2 lines")
    ap.add_argument("--traffic", default=None,
                    help="PMC summary (tools/pmc_summary.py) giving the dominant kernel's HBM bytes/dispatch; "
                         "default: the newest profiles/pmc_rNN_<config>.json")
    ap.add_argument("--mfma", default="f16x3", choices=["f32", "f16x3"],
                    help="operand mode of the contractions (model.LunaTokis mfma=)")
    ap.add_argument("--kernel-report", action="store_true", help="time every launch kind (stderr)")
    ap.add_argument("--range-check", default="rerun", choices=["rerun", "raise", "off"],
                    help="LunaTokis range_check (timing probes with wrong results use 'off')")
    ap.add_argument("--time-every", type=int, default=1,
                    help="HIP-event-time every N-th launch of the dominant kernel in the timed region")
    ap.add_argument("--fused-dcn", type=int, default=1, choices=[0, 1],
                    help="f16x3: DCN_sep as one kernel (k_dcn_sep, default) or offset/mask conv + DCN core (0)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="N>1 process group: nccl (= RCCL over xGMI, one GPU per rank) or gloo (host-staged halo; "
                         "ranks may share a GPU -- the multi-rank GPU test on a one-GPU box)")
    ap.add_argument("--trunk-lanes", type=int, default=2,
                    help="HIP streams the recon trunk's items are split over (LunaTokis trunk_lanes)")
    ap.add_argument("--pcd-streams", type=int, default=1,
                    help="PCD alignment: 2 = the DCN / feature branch on a second stream (LunaTokis pcd_streams)")
    ap.add_argument("--dynamic-tiles", type=int, default=0,
                    help="persistent Winograd conv: 1 = dynamic per-XCD tile counters, 0 = static schedule")
    ap.add_argument("--lstm-lanes", type=int, default=1,
                    help="streams for the BiConvLSTM's two directions (LunaTokis lstm_lanes: 1 or 2)")
    ap.add_argument("--dec-lanes", type=int, default=None,
                    help="HIP streams decoding's pairs are split over (LunaTokis dec_lanes; default: --lanes)")
    ap.add_argument("--lanes", type=int, default=1,
                    help="concurrent HIP streams per rank, each a contiguous range of the pairs (LunaTokis lanes)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    td = None
    if args.backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    # a torchrun launch (MASTER_ADDR set) initialises the process group even at world size 1, so the
    # N = 1 run of a scaling sweep goes through the same init / all_reduce / teardown as N > 1
    if world > 1 or "MASTER_ADDR" in os.environ:
        import torch.distributed as td
        torch.cuda.set_device(local)
        if args.backend == "nccl":
            # eager communicator (device_id): the halo exchange's batch_isend_irecv is not every rank's
            # first collective (parallel.halo_exchange)
            td.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            td.init_process_group("gloo")
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    import stif_pkg
    stif = stif_pkg.load()
    stif.ops.DYNAMIC_TILES = bool(args.dynamic_tiles)
    sd = stif.weights.make_state_dict(seed=0)
    nframes, H, W, scale, times, scaling = CONFIGS[args.config]
    elapsed, probe, timer, model, frames, tq, out_pix = run_config(stif, sd, args.config, args, world, rank, device,
                                                                   td, args.mfma)
    dom = timer.kind
    hot = hot_path_kernels(probe, args.mfma)
    if td is not None:
        t = torch.tensor([elapsed], device=device if args.backend == "nccl" else "cpu", dtype=torch.float64)
        td.all_reduce(t, op=td.ReduceOp.MAX)
        elapsed = float(t.item())
    n_launch, avg_ms, avg_flops, avg_bytes = timer.summary()
    if args.kernel_report and rank == 0 and frames is not None:
        with torch.no_grad():
            rep = KernelTimer(None)
            stif.ops.TRACE = rep
            model.gen_feat_window(frames)
            model.decoding(tq)
            torch.cuda.synchronize()
            stif.ops.TRACE = None
        print("launch report (one extra step, not timed):", file=sys.stderr)
        rep.report()

    value = out_pix * args.steps / elapsed / 1e6
    res = None
    if rank == 0:
        achieved = avg_flops / (avg_ms * 1e-3) / 1e12 if avg_ms else 0.0
        kname, kdesc, peak = kernel_desc(dom, args.mfma)
        traffic = None
        # HBM bytes per dispatch of the same kernel from the committed PMC passes over this bench at this
        # config (tools/pmc_summary.py; FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md HBM section)
        found = sorted(glob.glob(os.path.join(REPO, "profiles", f"pmc_r[0-9][0-9]_{args.config}.json")))
        tpath = args.traffic or (found[-1] if found else "")
        if os.path.exists(tpath) and args.mfma == "f16x3":
            try:
                pmc = json.load(open(tpath))["per_kernel"]
                hits = [v for k, v in pmc.items() if kname in k]
                if len(hits) == 1:
                    traffic = round(hits[0]["hbm_bytes_per_dispatch"])
            except Exception:
                traffic = None
        res = {
            "metric": BASE["metric"],
            "value": round(value, 4),
            "unit": "Mpix/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": args.mfma,
            "mfma_operands": ("f16x3: every contraction (Winograd convs, stride-2 convs, the DCN core, the SIREN decoder "
                              "layers) runs its fp32 products as 3 fp16 MFMA products on split operands (x = h + l, "
                              "~22-bit operands, fp32 accumulation; outputs within 1e-4 of the fp32 reference, "
                              "DESIGN.md section 3a); 1x1 convs and all elementwise/sampling math in fp32")
                             if args.mfma == "f16x3" else "f32: every contraction on fp32 MFMA",
            "data": "synthetic (U[0,1) frames, seeded; deterministic generated weights: checkpoint not in tree)",
            "config": {"workload": f"{'per GPU ' if scaling == 'weak' else ''}{nframes}x3x{H}x{W} "
                                   f"{'window' if scaling == 'weak' else 'sequence'} ({nframes - 1} pairs), "
                                   f"{scale}x spatial, t={times}",
                       "name": args.config, "frames": nframes, "lr_hw": [H, W], "scale": scale, "times": times,
                       "parallelism": (f"sequence pair-sharded x{world}, boundary-frame features by "
                                       f"{('RCCL P2P halo exchange' if args.backend == 'nccl' else 'gloo host-staged halo exchange') if args.halo == 'exchange' else 'recompute'}"
                                       if world > 1 else "1 GPU")},
            "roofline": roofline(kname, kdesc, dom, peak, achieved, avg_ms, avg_flops, avg_bytes, timer.seen,
                                 traffic, n_timed=n_launch),
            "hot_path_kernels": hot,
            # every kernel kind's share of the last warm-up step and its roofline fraction (the headline
            # `roofline` above is the dominant kind's, timed over the whole timed region)
            "top_kernels": kernel_table(probe, args.mfma, top=6) if probe.rec else [],
        }
    if world == 1 and not args.no_extras and td is None:
        # the same workload with every contraction on fp32 MFMA and without the per-call f16x3 range sync,
        # then the other configs on this one GPU (C3 / C4: the whole sequence -- the 1-GPU denominators
        # of the strong-scaling runs), and the host-inclusive line (frames from host memory, outputs back)
        extras = {}
        runs = [(args.config, "f32" if args.mfma == "f16x3" else "f16x3", "rerun")]
        if args.mfma == "f16x3":
            runs.append((args.config, "f16x3", "off"))
        runs += [(c, args.mfma, "rerun") for c in ("c1", "c2", "c3", "c4") if c != args.config]
        # the other operand mode / the range-sync-free line of the metric's own config over 10 steps (review r5: the
        # 3-step fp32 line moved by a few % between runs); the large configs keep 1-3 steps (seconds each)
        reps = {"c0": (10, 2), "c1": (3, 1), "c2": (2, 1), "c3": (1, 1), "c4": (1, 1)}
        for cfg, mf, rc in runs:
            a2 = argparse.Namespace(**vars(args))
            a2.steps, a2.warmup = reps[cfg]
            a2.range_check = rc
            del model
            torch.cuda.empty_cache()
            el, _, _, model, fr2, tq2, px = run_config(stif, sd, cfg, a2, 1, 0, device, None, mf, trace_dom=False)
            key = f"{cfg}_{mf}" + ("_range_check_off" if rc == "off" else "")
            extras[key] = {"value": round(px * a2.steps / el / 1e6, 4), "unit": "Mpix/s",
                           "ms_per_step": round(el / a2.steps * 1e3, 3), "steps": a2.steps}
            if cfg in ("c1", "c2") and mf == "f16x3":
                # the config's own top kernels and their roofline fractions (one more, untimed step)
                probe2 = KernelTimer(None)
                with torch.no_grad():
                    stif.ops.TRACE = probe2
                    model.gen_feat_window(fr2)
                    model.decoding(tq2)
                    torch.cuda.synchronize()
                    stif.ops.TRACE = None
                extras[key]["top_kernels"] = kernel_table(probe2, mf)
                del fr2
            if cfg in ("c3", "c4"):
                extras[key]["workload"] = (f"{CONFIGS[cfg][0]}-frame {CONFIGS[cfg][1]}x{CONFIGS[cfg][2]} sequence "
                                           f"({CONFIGS[cfg][0] - 1} pairs), {CONFIGS[cfg][3]}x, t={CONFIGS[cfg][4]}, "
                                           "all on 1 GPU (strong-scaling denominator)")
        del model
        torch.cuda.empty_cache()
        extras[f"{args.config}_host_inclusive"] = host_inclusive(stif, sd, args.config, device, args.mfma)
        res["extra_lines"] = extras
    if rank == 0 and world == 1 and td is None and not args.no_cpu_baseline:
        res["parity"], res["parity_gratings"] = parity_records(stif, sd, device, args.mfma)
        res["cpu_baseline"] = cpu_baseline()
    if rank == 0:
        print(json.dumps(res), flush=True)
    if td is not None:
        td.destroy_process_group()


if __name__ == "__main__":
    main()
