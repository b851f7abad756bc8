"""Numerics of Winograd F(2x2,3x3) vs F(4x4,3x3) on split-fp16 (f16x3) operands, emulated on the CPU
(is F(4x4) usable under the engine's rtol 1e-4 bar and the f16x3 range?).

One 64 -> 64 3x3 conv with a recon_trunk weight (weights.make_state_dict(0)) on N(0, 1) activations:
  reference: direct conv in float64;
  F(m x m, 3x3): V = B^T d B in fp32, U = G g G^T in float64 (host-packed), each split x * 2^s = h + l
  (h = fp16(x 2^s), l = fp16(x 2^s - h)), products h_a h_b + h_a l_b + l_a h_b (exact in fp32) summed
  in fp32 in K blocks of 16 (the MFMA's accumulation), output transform A^T M A in fp32.
Prints the max error relative to max|ref| and the largest |V| / max|d| (the split range: fp16 max 65504
after the 2^4 activation scale).

usage: python tools/experiments/wino43_numerics.py [H] [W]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import stif_pkg  # noqa: E402

F23 = dict(BT=np.array([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], np.float64),
           G=np.array([[1, 0, 0], [.5, .5, .5], [.5, -.5, .5], [0, 0, 1]], np.float64),
           AT=np.array([[1, 1, 1, 0], [0, 1, -1, -1]], np.float64), m=2)
F43 = dict(BT=np.array([[4, 0, -5, 0, 1, 0], [0, -4, -4, 1, 1, 0], [0, 4, -4, -1, 1, 0],
                        [0, -2, -1, 2, 1, 0], [0, 2, -1, -2, 1, 0], [0, 4, 0, -5, 0, 1]], np.float64),
           G=np.array([[1 / 4, 0, 0], [-1 / 6, -1 / 6, -1 / 6], [-1 / 6, 1 / 6, -1 / 6],
                       [1 / 24, 1 / 12, 1 / 6], [1 / 24, -1 / 12, 1 / 6], [0, 0, 1]], np.float64),
           AT=np.array([[1, 1, 1, 1, 1, 0], [0, 1, -1, 2, -2, 0], [0, 1, 1, 4, 4, 0], [0, 1, -1, 8, -8, 1]],
                       np.float64), m=4)


def split(x, s):
    h = (x * 2.0 ** s).astype(np.float16)
    l = (x * 2.0 ** s - h.astype(np.float64)).astype(np.float16)
    return h.astype(np.float32), l.astype(np.float32)


def direct(d, w):
    C, H, W = d.shape
    p = np.pad(d, ((0, 0), (1, 1), (1, 1)))
    out = np.zeros((w.shape[0], H, W))
    for ky in range(3):
        for kx in range(3):
            out += np.einsum("oc,chw->ohw", w[:, :, ky, kx], p[:, ky:ky + H, kx:kx + W])
    return out


def winograd(d, w, T):
    BT, G, AT, m = T["BT"], T["G"], T["AT"], T["m"]
    a = m + 2
    C, H, W = d.shape
    p = np.pad(d, ((0, 0), (1, 1 + a), (1, 1 + a))).astype(np.float32)
    ty, tx = H // m, W // m
    # transformed weights U[xi][o][c] (float64 -> split x 2^10)
    U = np.einsum("ik,ockl,jl->ijoc", G, w, G)
    Uh, Ul = split(U, 10)
    out = np.zeros((w.shape[0], H, W), np.float32)
    vmax = 0.0
    for y in range(ty):
        for x in range(tx):
            dt = p[:, y * m:y * m + a, x * m:x * m + a]
            V = np.einsum("ik,ckl,jl->ijc", BT.astype(np.float32), dt, BT.astype(np.float32)).astype(np.float32)
            vmax = max(vmax, float(np.abs(V).max()))
            Vh, Vl = split(V.astype(np.float64), 4)
            M = np.zeros((a, a, w.shape[0]), np.float32)
            for k0 in range(0, C, 16):   # fp32 accumulation in MFMA K blocks
                sl = slice(k0, k0 + 16)
                blk = (np.einsum("ijoc,ijc->ijo", Uh[:, :, :, sl], Vh[:, :, sl]) +
                       np.einsum("ijoc,ijc->ijo", Ul[:, :, :, sl], Vh[:, :, sl]) +
                       np.einsum("ijoc,ijc->ijo", Uh[:, :, :, sl], Vl[:, :, sl])).astype(np.float32)
                M = (M + blk).astype(np.float32)
            M = (M * np.float32(2.0 ** -14)).astype(np.float32)
            Y = np.einsum("ki,ijo,lj->okl", AT.astype(np.float32), M, AT.astype(np.float32)).astype(np.float32)
            out[:, y * m:(y + 1) * m, x * m:(x + 1) * m] = Y
    return out, vmax


def main():
    H = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    W = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    sd = stif_pkg.load().weights.make_state_dict(seed=0)
    w = sd["recon_trunk.0.conv1.weight"].astype(np.float64)
    d = np.random.default_rng(0).standard_normal((64, H, W))
    ref = direct(d, w)
    for name, T in (("F(2x2,3x3)", F23), ("F(4x4,3x3)", F43)):
        out, vmax = winograd(d, w, T)
        err = float(np.abs(out - ref).max() / np.abs(ref).max())
        print(f"{name}: max error {err:.2e} of max|ref|, max|V| / max|d| = {vmax / np.abs(d).max():.1f}")


if __name__ == "__main__":
    main()
