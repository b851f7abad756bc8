"""Benchmark of the STIF LunaTokis forward on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): a synthetic 7-frame 3x256x256 window = 6
adjacent pairs, 4x spatial, one interpolated time t=0.5 -> 6 x 1024x1024 output
pixels per GPU per step.  A step = gen_feat over the window (per-frame encoder,
PCD alignment, Bi-Deformable-ConvLSTM, 40-block trunk) + the implicit decoder,
with inputs already resident in HBM.  Multi-GPU: one process per GPU; rank r owns
frames [6r, 6r+6] of a (6N+1)-frame sequence (the shared boundary frame is the
temporal halo), so per-GPU work is fixed (weak scaling) and no collective is on
the data path.  Rank 0 prints one JSON line.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c1|c0|c2]
"""
import argparse
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
    # name: (frames, H, W, scale, times)
    "c0": (7, 128, 128, 4, [0.5]),
    "c1": (7, 256, 256, 4, [0.5]),
    "c2": (7, 540, 960, 4, [0.25, 0.5, 0.75]),
}
FP32_PEAK_TFLOPS = 157.3   # MI355X dense fp32 MFMA (MI355X_MICROARCH.md, chip-level parameters)
# f16x3 operand mode: one fp32-class product = 3 products on the dense fp16 MFMA pipe (~2.5 PF/s)
F16X3_PEAK_TFLOPS = 2500.0 / 3.0
WINO_GAIN = 36.0 / 16.0    # F(2x2,3x3): 16 transformed-domain MACs per 36 direct MACs
EPI_NAMES = {0: "NONE", 1: "LRELU", 2: "RELU", 3: "RES", 4: "OFFMASK", 5: "LSTM"}


def kernel_desc(kind, mfma="f32"):
    """(kernel name as rocprof shows it, description, peak in algorithmic TFLOP/s) of a launch kind."""
    f16 = mfma == "f16x3"
    if kind[0] == "wino":
        _, ks, s, epi, in1, cout = kind
        if f16:
            return (f"k_wino<{in1}, {epi}, 0, 1>", f"3x3 {64 * (2 if in1 else 1)}->{cout} conv, EPI_{EPI_NAMES[epi]}, "
                    "Winograd F(2x2,3x3) on split-fp16 MFMA (3 fp16 products per fp32-class product); algorithmic = "
                    "direct-conv FLOPs, peak = fp16 MFMA dense peak / 3 x 36/16", F16X3_PEAK_TFLOPS * WINO_GAIN)
        return (f"k_wino<{in1}, {epi}, 0, 0>", f"3x3 {64 * (2 if in1 else 1)}->{cout} conv, EPI_{EPI_NAMES[epi]}, "
                f"Winograd F(2x2,3x3) on fp32 MFMA; algorithmic = direct-conv FLOPs, peak = fp32 MFMA peak x 36/16",
                FP32_PEAK_TFLOPS * WINO_GAIN)
    if kind[0] == "conv":
        _, ks, s, epi, in1, cout = kind
        return (f"k_conv<{ks}, {s}, ...>", f"{ks}x{ks}/s{s} conv -> {cout}, in1 mode {in1}, EPI_{EPI_NAMES[epi]}, "
                "direct implicit GEMM on fp32 MFMA", FP32_PEAK_TFLOPS)
    if kind[0] == "dcn":
        if f16:
            return (f"k_dcn<{kind[1]}, 1>", "fused modulated deformable conv, split-fp16 MFMA (peak = fp16 MFMA / 3)",
                    F16X3_PEAK_TFLOPS)
        return (f"k_dcn<{kind[1]}, 0>", "fused modulated deformable conv", FP32_PEAK_TFLOPS)
    if f16:
        return (f"k_{kind[0]}", "SIREN decoder stage, split-fp16 MFMA (peak = fp16 MFMA / 3)", F16X3_PEAK_TFLOPS)
    return (f"k_{kind[0]}", "SIREN decoder stage", FP32_PEAK_TFLOPS)


class KernelTimer:
    """HIP-event timing of every launch of one kernel variant (or of all, kind=None), on the
    launch stream."""

    def __init__(self, kind):
        self.kind = kind
        self.nbytes = []
        self.rec = []
        self.all = []
        self._cur = None

    kinds = None

    def begin(self, kind, flops, nbytes=0.0):
        if self.kind is None or kind == self.kind:
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
        """the launch kind with the largest total time"""
        return max(self.per_kind().items(), key=lambda kv: kv[1][1])[0]

    def report(self):
        """per-kind launches / avg us / TFLOP/s (all-kinds mode)"""
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


def hot_path_kernels(probe, mfma):
    """The north star's DCNv2 + implicit-decoder kernels, from the last warm-up step (HIP events on
    the launch stream): per kind avg time and TFLOP/s; for the DCN core also its algorithmic HBM
    bytes (input + offset/mask + output per pixel) as GB/s and fraction of the HBM peak; for the
    decoder stages the fraction of the MFMA peak of their operand mode."""
    dec_peak = 2500.0 / 3 if mfma == "f16x3" else 157.3
    out = {}
    for k, (nl, ms, fl, nb) in probe.per_kind().items():
        if k[0] not in ("dcn", "dec1", "dec2") or not ms:
            continue
        e = {"launches": nl, "avg_us": round(ms / nl * 1e3, 1), "tflops": round(fl / (ms * 1e-3) / 1e12, 1)}
        if nb:
            gbps = nb / (ms * 1e-3) / 1e9
            e.update(hbm_gbps_algorithmic=round(gbps, 1), hbm_frac=round(gbps / HBM_PEAK_GBPS, 3))
        if k[0] != "dcn":
            e["mfma_frac"] = round(fl / (ms * 1e-3) / 1e12 / dec_peak, 3)
        out["_".join(str(x) for x in k)] = e
    return out


def synth_frames(first, count, H, W, device):
    """Deterministic synthetic frames: frame k = U[0,1) from a generator seeded by its global index."""
    out = torch.empty(count, 3, H, W)
    for i in range(count):
        g = torch.Generator().manual_seed(1234 + first + i)
        out[i] = torch.rand(3, H, W, generator=g)
    return out.to(device)


def cpu_baseline(stif, sd, frames_cpu, times, scale, crop=128):
    """The numpy oracle (fp32) on a bounded sample of the same workload: one pair of the
    window, cropped to crop x crop LR pixels (FLOP per output pixel does not depend on the
    frame size), on all host BLAS threads."""
    from oracle import stif_oracle as O
    try:
        from threadpoolctl import threadpool_info
        threads = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    except Exception:
        threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    x = np.ascontiguousarray(frames_cpu[0:2, :, :crop, :crop].numpy()[None])
    t0 = time.perf_counter()
    O.forward(x, times, sd, dtype=np.float32)
    dt = time.perf_counter() - t0
    H, W = x.shape[-2:]
    mpix = len(times) * H * scale * W * scale / 1e6
    return {"value": mpix / dt, "unit": "Mpix/s", "cores": threads, "kind": "port",
            "sample": f"1 pair (frames 0-1) of the same window cropped to {H}x{W} -> {H * scale}x{W * scale}, "
                      f"t={times}, numpy fp32 restatement (oracle/stif_oracle.py), {dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c1", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic", default=os.path.join(REPO, "profiles", "pmc_r01.json"),
                    help="PMC summary (tools/pmc_summary.py) giving the dominant kernel's HBM bytes/dispatch")
    ap.add_argument("--mfma", default="f16x3", choices=["f32", "f16x3"],
                    help="Winograd conv operand mode (model.LunaTokis mfma=)")
    ap.add_argument("--kernel-report", action="store_true", help="time every conv launch kind (stderr)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if dist:
        import torch.distributed as td
        torch.cuda.set_device(local)
        td.init_process_group("nccl")
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    import stif_pkg
    stif = stif_pkg.load()
    nframes, H, W, scale, times = CONFIGS[args.config]
    pairs = nframes - 1
    sd = stif.weights.make_state_dict(seed=0)
    model = stif.LunaTokis(64, 6, 8, 5, 40, device=device, mfma=args.mfma)
    model.load_state_dict(sd, strict=True)
    frames_cpu = synth_frames(rank * pairs, nframes, H, W, "cpu")
    frames = frames_cpu.to(device)
    tq = [torch.tensor([[t]], device=device) for t in times]

    def step():
        model.gen_feat_window(frames)
        return model.decoding(tq)

    with torch.no_grad():
        # warm-up; the last warm-up step times every launch to find the dominant kernel
        probe = KernelTimer(None)
        for i in range(max(1, args.warmup)):
            stif.ops.TRACE = probe if i == max(1, args.warmup) - 1 else None
            step()
        stif.ops.TRACE = None
        torch.cuda.synchronize()
        dom = probe.dominant()
        hot = hot_path_kernels(probe, args.mfma)
        timer = KernelTimer(dom)
        stif.ops.TRACE = timer
        if dist:
            td.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        if dist:
            td.barrier()
        elapsed = time.perf_counter() - t0
        stif.ops.TRACE = None
    if dist:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        td.all_reduce(t, op=td.ReduceOp.MAX)
        elapsed = float(t.item())
    n_launch, avg_ms, avg_flops, avg_bytes = timer.summary()
    if args.kernel_report and rank == 0:
        with torch.no_grad():
            rep = KernelTimer(None)
            stif.ops.TRACE = rep
            step()
            torch.cuda.synchronize()
            stif.ops.TRACE = None
        print("conv launch report (one extra step, not timed):", file=sys.stderr)
        rep.report()

    out_pix = pairs * len(times) * (H * scale) * (W * scale)
    value = world * out_pix * args.steps / elapsed / 1e6
    if rank == 0:
        achieved = avg_flops / (avg_ms * 1e-3) / 1e12 if avg_ms else 0.0
        kname, kdesc, peak = kernel_desc(dom, args.mfma)
        traffic = None
        # HBM bytes per dispatch of the same kernel from the committed PMC passes over this bench
        # (tools/pmc_summary.py); they were measured at C1, so only a C1 line carries them
        if args.config == "c1" and os.path.exists(args.traffic):
            try:
                pmc = json.load(open(args.traffic))["per_kernel"]
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
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "mfma_operands": ("f16x3: Winograd convs, the DCN core and the SIREN decoder layers run fp32 products as 3 fp16 MFMA products "
                              "on split operands (x = h + l, ~22-bit operands, fp32 accumulation; accuracy "
                              "equal to the fp32-MFMA path, DESIGN.md section 3)") if args.mfma == "f16x3" else
                             "f32: every contraction on fp32 MFMA",
            "data": "synthetic (U[0,1) frames, seeded; deterministic generated weights: checkpoint not in tree)",
            "config": {"workload": f"{nframes}x3x{H}x{W} window ({pairs} pairs), {scale}x spatial, t={times}",
                       "frames_per_gpu": nframes, "lr_hw": [H, W], "scale": scale, "times": times,
                       "parallelism": f"pair-sharded x{world} (1-frame halo, no collective)"},
            "roofline": {"bound": "mfma", "kernel": f"{kname} ({kdesc})", "kind": list(dom),
                         "achieved": round(achieved, 3), "peak": round(peak, 2), "unit": "TFLOP/s",
                         "frac": round(achieved / peak, 4), "traffic": traffic,
                         "launches": n_launch, "avg_launch_us": round(avg_ms * 1e3, 2),
                         "flops_per_launch": avg_flops,
                         "algorithmic_bytes_per_launch": round(avg_bytes),
                         "hbm_gbps_algorithmic": round(avg_bytes / (avg_ms * 1e-3) / 1e9, 1) if avg_ms else None},
        }
        res["hot_path_kernels"] = hot
        if not args.no_cpu_baseline and world == 1:
            res["cpu_baseline"] = cpu_baseline(stif, sd, frames_cpu, times, scale)
        print(json.dumps(res), flush=True)
    if dist:
        td.destroy_process_group()


if __name__ == "__main__":
    main()
