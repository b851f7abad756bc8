"""Host-side logic without a GPU: C-ABI exports, weight packing layouts, state-dict
contract, decoder coordinate tables."""
import json
import os
import re

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_state_dict_spec_matches_reference(stif):
    ref = json.load(open(os.path.join(REPO, "tests", "golden", "state_dict_spec.json")))
    spec = stif.weights.state_dict_spec()
    assert [k for k, _ in ref] == list(spec.keys())
    assert all(tuple(s) == spec[k] for k, s in ref)
    assert len(spec) == 442
    assert sum(int(np.prod(s)) for s in spec.values()) == 11312698


def test_weights_deterministic(stif):
    a = stif.weights.make_weight("pcd_align.L1_dcnpack_1.conv_offset_mask.weight", (216, 64, 3, 3), 0)
    b = stif.weights.make_weight("pcd_align.L1_dcnpack_1.conv_offset_mask.weight", (216, 64, 3, 3), 0)
    assert np.array_equal(a, b) and np.abs(a).max() > 0


def test_library_exports_every_header_symbol(stif):
    hdr = open(os.path.join(REPO, "include", "stif.h")).read()
    names = set(re.findall(r"^\s*(?:int|size_t|const char\*)\s+(stif_\w+)\s*\(", hdr, re.M))
    assert len(names) >= 15
    lib = stif._lib.lib()
    for n in sorted(names):
        assert hasattr(lib, n), n
    assert set(stif._lib.EXPORTS) >= names


def _device_code_objects(path):
    """The gfx950 code objects of a HIP shared library: its .hip_fatbin holds one clang offload bundle per
    translation unit (magic, entry count, then per entry offset / size / target-triple, little-endian u64)."""
    import struct
    data = open(path, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    out, pos = [], data.find(magic)
    while pos >= 0:
        n = struct.unpack_from("<Q", data, pos + 24)[0]
        q = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, q)
            triple = data[q + 24:q + 24 + tlen].decode()
            q += 24 + tlen
            if "amdgcn" in triple and "gfx950" in triple:
                out.append((triple, data[pos + off:pos + off + size]))
        pos = data.find(magic, pos + 24)
    return out


def test_device_code_has_no_packed_fp32(stif, tmp_path):
    """No kernel may use packed fp32 VALU (v_pk_fma/mul/add_f32): beside MFMAs it is slower than two scalar ops, and in
    the tap-pipelined DCN_sep schedule its results depended on the co-resident workgroup (DESIGN.md section 3d,
    profiles/r06_tappipe_dump_bisect.log).  Makefile: NOPK_SRC lists every .hip object."""
    import shutil
    import subprocess
    objdump = "/opt/rocm/lib/llvm/bin/llvm-objdump"
    if not os.path.exists(objdump) or shutil.which("/opt/rocm/lib/llvm/bin/llvm-objdump") is None:
        pytest.skip("llvm-objdump not available")
    lib = stif._lib.LIB_PATH
    cos = _device_code_objects(lib)
    csrc = os.path.join(REPO, "stif-continuous-video-representation_amd", "csrc")
    kernels = [f for f in os.listdir(csrc) if f.endswith(".hip") and "__global__" in open(os.path.join(csrc, f)).read()]
    assert len(cos) >= len(kernels), (len(cos), kernels)
    total = 0
    for i, (triple, co) in enumerate(cos):
        f = tmp_path / f"co{i}.elf"
        f.write_bytes(co)
        asm = subprocess.run([objdump, "-d", "--mcpu=gfx950", str(f)], capture_output=True, text=True, check=True).stdout
        n_ins = len(re.findall(r"^\s+v_\w+", asm, re.M))
        total += n_ins
        assert not re.search(r"\bv_pk_(fma|mul|add)_f32\b", asm), f"packed fp32 in code object {i} ({triple})"
    assert total > 10000   # the disassembly really covered the kernels


def _unpack_conv(wd, cout_pad, cin, ks, nt):
    """inverse of the [slice][chunk][tap][nt][lane][4] packing -> [cout_pad][cin][ks][ks]"""
    ns = cout_pad // (32 * nt)
    a = wd.reshape(ns, cin // 8, ks * ks, nt, 2, 32, 4)      # lane = h*32 + j
    a = a.transpose(0, 3, 5, 1, 4, 6, 2)                      # [s][nt][j][chunk][h][e][tap]
    return a.reshape(cout_pad, cin, ks, ks)


@pytest.mark.parametrize("mode", ["plain", "offmask", "lstm", "plain1x1"])
def test_pack_conv_layout(stif, mode):
    L = stif._lib
    rng = np.random.default_rng(0)
    cout, cin, ks, m, nt = {"plain": (64, 128, 3, L.PACK_PLAIN, 2), "offmask": (216, 64, 3, L.PACK_OFFMASK, 7),
                            "lstm": (256, 128, 3, L.PACK_LSTM, 4), "plain1x1": (256, 200, 1, L.PACK_PLAIN, 2)}[mode]
    w = rng.standard_normal((cout, cin, ks, ks)).astype(np.float32)
    b = rng.standard_normal(cout).astype(np.float32)
    lib = L.lib()
    wd = np.empty(lib.stif_conv_weight_floats(cout, cin, ks, m), np.float32)
    bd = np.empty(lib.stif_conv_bias_floats(cout, m), np.float32)
    assert lib.stif_pack_conv_weight(w.ctypes.data, b.ctypes.data, cout, cin, ks, m, wd.ctypes.data, bd.ctypes.data) == 0
    cp = bd.size
    assert cp % (32 * nt) == 0 and cp >= cout
    up = _unpack_conv(wd, cp, cin, ks, nt)
    if mode == "offmask":
        perm = []
        for g in range(8):
            for k in range(9):
                perm += [g * 18 + 2 * k, g * 18 + 2 * k + 1, 144 + g * 9 + k]
        perm = np.array(perm)
    elif mode == "lstm":
        perm = np.array([gate * 64 + s * 32 + j for s in range(2) for gate in range(4) for j in range(32)])
    else:
        perm = np.arange(cout)
    assert np.array_equal(up[:cout], w[perm])
    assert np.array_equal(bd[:cout], b[perm])
    assert not up[cout:].any() and not bd[cout:].any()


def test_pack_rejects_bad_shapes(stif):
    L = stif._lib
    lib = L.lib()
    w = np.zeros((64, 3, 3, 3), np.float32)
    out = np.zeros(64 * 3 * 9 * 4, np.float32)
    rc = lib.stif_pack_conv_weight(w.ctypes.data, None, 64, 3, 3, 0, out.ctypes.data, None)
    assert rc == 1 and b"bad arguments" in lib.stif_last_error()


def test_pack_dec_mlp_tile_layout(stif, sd):
    """One tile of the decoder MLP packing: element [v][lane][e] = W[ot*32+(lane&31)][kt*32+F(4v+e, lane>>5)]."""
    L = stif._lib
    lib = L.lib()
    arrs = {}
    for p, n in (("feat_imnet.", 3), ("flow_imnet.", 3), ("encode_imnet.", 4)):
        a = []
        for i in range(n):
            a += [sd[f"{p}net.{i}.linear.weight"], sd[f"{p}net.{i}.linear.bias"]]
        a += [sd[f"{p}net.{n}.weight"], sd[f"{p}net.{n}.bias"]]
        arrs[p] = [np.ascontiguousarray(x) for x in a]
    ptr = lambda a: (L._P * len(a))(*[x.ctypes.data for x in a])
    mlp = np.empty(lib.stif_dec_mlp_floats(), np.float32)
    assert lib.stif_pack_dec_mlp(ptr(arrs["feat_imnet."]), ptr(arrs["flow_imnet."]), ptr(arrs["encode_imnet."]),
                                 mlp.ctypes.data) == 0
    # encode layer 3 (256x256) lives after: find it through the documented feat W1 tile at offset 192
    W1 = arrs["feat_imnet."][2]
    tile = mlp[192:192 + 1024].reshape(4, 64, 4)
    for ot, kt in ((0, 0),):
        for v in range(4):
            for lane in range(64):
                for e in range(4):
                    q = 4 * v + e
                    f = (q & 3) + 8 * (q >> 2) + 4 * (lane >> 5)
                    # sine layers carry omega_0 = 30 (SIREN.py:44-51), scaled in double
                    assert tile[v, lane, e] == np.float32(30.0 * np.float64(W1[ot * 32 + (lane & 31), kt * 32 + f]))
    assert np.array_equal(mlp[0:64], (30.0 * arrs["feat_imnet."][0][:, 198].astype(np.float64)).astype(np.float32))


def test_pack_dec_mlp_q16_tiles(stif, sd):
    """The f16x3 decoder packing's 16x16x32 copies of encode_imnet's tiles (dec_layout.h Q_*, read by k_dec2q):
    tile (ot, kt) as [s][plane][lane][8 halves], lane l holding W[32 ot + 16 s + (l & 15)][32 kt + 16 (e >> 2)
    + 4 (l >> 4) + (e & 3)] x 2^10 split into fp16 h + l; sine layers in revolutions (omega_0 / 2 pi)."""
    L = stif._lib
    lib = L.lib()
    arrs = {}
    for p, n in (("feat_imnet.", 3), ("flow_imnet.", 3), ("encode_imnet.", 4)):
        a = []
        for i in range(n):
            a += [sd[f"{p}net.{i}.linear.weight"], sd[f"{p}net.{i}.linear.bias"]]
        a += [sd[f"{p}net.{n}.weight"], sd[f"{p}net.{n}.bias"]]
        arrs[p] = [np.ascontiguousarray(x) for x in a]
    ptr = lambda a: (L._P * len(a))(*[x.ctypes.data for x in a])
    mlp = np.empty(lib.stif_dec_mlp_floats(), np.float32)
    L.check(lib.stif_pack_dec_mlp_ex(ptr(arrs["feat_imnet."]), ptr(arrs["flow_imnet."]), ptr(arrs["encode_imnet."]),
                                     mlp.ctypes.data, L.CONV_F16X3), "pack")
    T = 1024
    q_end = mlp.size
    q_w3 = q_end - 64 * T
    q_w2 = q_w3 - 16 * T
    q_w0 = q_w2 - 4 * T - 8 * T
    rev = 30.0 / (2 * np.pi)
    lanes = np.arange(64)
    for base, W, kts, (ot, kt) in ((q_w3, arrs["encode_imnet."][6], 8, (3, 5)), (q_w2, arrs["encode_imnet."][4], 2, (6, 1)),
                                   (q_w0, arrs["encode_imnet."][0], 4, (1, 3))):
        t = mlp[base + (ot * kts + kt) * T:base + (ot * kts + kt + 1) * T].view(np.float16).astype(np.float64)
        t = t.reshape(2, 2, 64, 8)
        val = (t[:, 0] + t[:, 1]) / 1024.0                       # [s][lane][e]
        for s_ in range(2):
            for e in range(8):
                rows = 32 * ot + 16 * s_ + (lanes & 15)
                cols = 32 * kt + 16 * (e >> 2) + 4 * (lanes >> 4) + (e & 3)
                want = rev * W[rows, cols].astype(np.float64)
                assert np.abs(val[s_, :, e] - want).max() <= 2e-6 * np.abs(want).max() + 1e-12


def test_decoder_tables_match_reference_nearest(stif, golden):
    g = golden["ops"]
    for (h, w, hh, ww) in [(16, 20, 40, 50), (24, 32, 60, 80), (135, 240, 337, 600), (32, 32, 128, 128),
                           (5, 7, 13, 17), (16, 20, 64, 80)]:
        t = stif.coords.dec_tables(h, w, hh, ww)
        assert np.array_equal(t["near_y"], g[f"nearest_{h}x{w}_{hh}x{ww}_row"])
        assert np.array_equal(t["near_x"], g[f"nearest_{h}x{w}_{hh}x{ww}_col"])


def test_decoder_tables_bilinear_weights(stif):
    t = stif.coords.dec_tables(16, 20, 64, 80)
    # inside the map the two weights of an axis sum to 1; at the borders one is dropped (zeros padding)
    s = t["w0_y"] + t["w1_y"]
    assert np.allclose(s[4:-4], 1.0)
    assert t["w0_y"][0] == 0.0 and t["w1_y"][-1] == 0.0


def test_load_state_dict_contract(stif, sd):
    m = stif.LunaTokis(64, 6, 8, 5, 40, device="cpu")
    bad = dict(sd)
    bad.pop("fusion.bias")
    with pytest.raises(RuntimeError, match="Missing key"):
        m.load_state_dict(bad)
    extra = {"module." + k: v for k, v in sd.items()}
    extra["module.junk"] = np.zeros(1, np.float32)
    with pytest.raises(RuntimeError, match="Unexpected key"):
        m.load_state_dict(extra)
    wrong = dict(sd)
    wrong["fusion.bias"] = np.zeros(3, np.float32)
    with pytest.raises(RuntimeError, match="size mismatch"):
        m.load_state_dict(wrong)
    m.load_state_dict({"module." + k: v for k, v in sd.items()}, strict=True)
    back = m.state_dict()
    assert list(back.keys()) == list(sd.keys())
    assert np.array_equal(back["recon_trunk.39.conv2.weight"].numpy(), sd["recon_trunk.39.conv2.weight"])


def test_pack_wino_layout(stif):
    """STIF_PACK_WINO: [slice][chunk][i][j][nt][lane][4] of U = G g G^T (F(2x2,3x3))."""
    L = stif._lib
    lib = L.lib()
    rng = np.random.default_rng(1)
    cout, cin = 96, 16          # 96 -> padded to 128 (2 slices)
    w = rng.standard_normal((cout, cin, 3, 3)).astype(np.float32)
    b = rng.standard_normal(cout).astype(np.float32)
    wd = np.empty(lib.stif_conv_weight_floats(cout, cin, 3, L.PACK_WINO), np.float32)
    bd = np.empty(lib.stif_conv_bias_floats(cout, L.PACK_WINO), np.float32)
    assert wd.size == 128 * cin * 16 and bd.size == 128
    assert lib.stif_pack_conv_weight(w.ctypes.data, b.ctypes.data, cout, cin, 3, L.PACK_WINO,
                                     wd.ctypes.data, bd.ctypes.data) == 0
    G = np.array([[1, 0, 0], [.5, .5, .5], [.5, -.5, .5], [0, 0, 1]])
    U = np.einsum("ap,oipq,bq->oiab", G, w.astype(np.float64), G)          # [co][ci][4][4]
    Up = np.zeros((128, cin, 4, 4))
    Up[:cout] = U
    a = wd.reshape(2, cin // 8, 4, 4, 2, 2, 32, 4)        # [s][c][i][j][nt][h][l32][e]
    got = a.transpose(0, 4, 6, 1, 5, 7, 2, 3).reshape(128, cin, 4, 4)
    assert np.allclose(got, Up, rtol=1e-6, atol=1e-7)
    assert np.array_equal(bd[:cout], b) and not bd[cout:].any()


def test_ensemble_tables(stif):
    """local-ensemble tables: rel_coord from the unshifted query, HR remap within range, weights
    summing to 1 (the areas of the four shifted queries tile the LR cell)."""
    C = stif.coords
    t0 = C.dec_tables(16, 20, 64, 80)
    t = C.dec_tables(16, 20, 64, 80, (-1, 1))
    assert (t["hr_y"] >= 0).all() and (t["hr_y"] < 64).all() and (t["hr_x"] < 80).all()
    assert np.array_equal(t0["hr_y"], np.arange(64)) and np.array_equal(t0["hr_x"], np.arange(80))
    assert not np.array_equal(t["near_y"], t0["near_y"])
    w = C.ensemble_weights(16, 20, 64, 80)
    assert np.allclose(sum(w), 1.0, atol=1e-5)


def test_resize_tables_match_reference(stif):
    """video.resize_tables = calculate_weights_indices (data/util.py:248-300), fixture from the reference"""
    h = np.load(os.path.join(REPO, "tests", "golden", "harness.npz"))
    w, i0, s0 = stif.video.resize_tables(37, 19, 0.5)
    assert np.array_equal(w, h["w_37_19"]) and np.array_equal(i0, h["i_37_19"][:, 0]) and s0 == h["sym_37_19"][0]


def test_pack_wino_f16x3_layout(stif):
    """STIF_PACK_WINO | STIF_PACK_F16X3: [slice][pair][i][j][nt][plane][lane][8] fp16 halves,
    element e of lane l = input channel 16 q + 8 (e >> 2) + 4 (l >> 5) + (e & 3); h + l = U * 2^10
    to ~2^-22 relative (fp32-class operands)."""
    L = stif._lib
    lib = L.lib()
    rng = np.random.default_rng(2)
    cout, cin = 96, 32
    mode = L.PACK_WINO | L.PACK_F16X3
    w = (rng.standard_normal((cout, cin, 3, 3)) * 0.05).astype(np.float32)
    b = rng.standard_normal(cout).astype(np.float32)
    wd = np.empty(lib.stif_conv_weight_floats(cout, cin, 3, mode), np.float32)
    bd = np.empty(lib.stif_conv_bias_floats(cout, mode), np.float32)
    assert wd.size == 128 * cin * 16
    assert lib.stif_pack_conv_weight(w.ctypes.data, b.ctypes.data, cout, cin, 3, mode,
                                     wd.ctypes.data, bd.ctypes.data) == 0
    G = np.array([[1, 0, 0], [.5, .5, .5], [.5, -.5, .5], [0, 0, 1]])
    U = np.zeros((128, cin, 4, 4))
    U[:cout] = np.einsum("ap,oipq,bq->oiab", G, w.astype(np.float64), G)
    hv = wd.view(np.float16).astype(np.float64).reshape(2, cin // 16, 4, 4, 2, 2, 2, 32, 2, 4)
    # axes: [s][q][i][j][nt][plane][hf][l32][eh][e4]; channel 16 q + 8 eh + 4 hf + e4
    full = hv[:, :, :, :, :, 0] + hv[:, :, :, :, :, 1]           # h + l
    got = full.transpose(0, 4, 6, 1, 7, 5, 8, 2, 3).reshape(128, cin, 4, 4) / 1024.0
    assert np.abs(got - U).max() <= 2.0 ** -21 * np.abs(U).max()
    hi = hv[:, :, :, :, :, 0].transpose(0, 4, 6, 1, 7, 5, 8, 2, 3).reshape(128, cin, 4, 4)
    assert np.array_equal(hi, (U * 1024).astype(np.float16).astype(np.float64))   # h = rne16(U 2^10)
    assert np.array_equal(bd[:cout], b)
    with pytest.raises(Exception):
        L.check(lib.stif_pack_conv_weight(w.ctypes.data, b.ctypes.data, cout, cin, 3, L.PACK_OFFMASK | L.PACK_F16X3,
                                          wd.ctypes.data, bd.ctypes.data), "pack")


def test_pack_dcnsep_layout(stif):
    """STIF_PACK_DCNSEP | F16X3 (the fused DCN_sep's offset/mask conv, include/stif.h): 7 M-tiles; row i of
    M-tile m is accumulator register r = (i & 3) + 4 (i >> 3) of lane half h = (i >> 2) & 1, whose slot
    s = 16 m + r < 108 holds component s % 3 of tap (s % 27) / 3 of group 2 (s / 27) + h -- the groups that
    lane half samples; the f16 h + l planes carry the weight to ~22 bits; the bias follows the rows.
    STIF_PACK_DCNPAIR | F16X3 (its DCN weight): [pair][tap][nt][plane][lane][8], input channel
    8 (2 pair + (lane >> 5)) + e."""
    L = stif._lib
    lib = L.lib()
    rng = np.random.default_rng(0)
    w = (rng.standard_normal((216, 64, 3, 3)) * 0.1).astype(np.float32)
    b = rng.standard_normal(216).astype(np.float32)
    mode = L.PACK_DCNSEP | L.PACK_F16X3
    wd = np.empty(lib.stif_conv_weight_floats(216, 64, 3, mode), np.float32)
    bd = np.empty(lib.stif_conv_bias_floats(216, mode), np.float32)
    L.check(lib.stif_pack_conv_weight(w.ctypes.data, b.ctypes.data, 216, 64, 3, mode, wd.ctypes.data,
                                      bd.ctypes.data), "pack")
    h = wd.view(np.float16).reshape(36, 7, 2, 64, 8).astype(np.float64)
    val = (h[:, :, 0] + h[:, :, 1]) / 1024.0                    # [k][M-tile][lane][e]
    seen = set()
    for m in range(7):
        for i in range(32):
            hh, r = (i >> 2) & 1, (i & 3) + 4 * (i >> 3)
            s_ = 16 * m + r
            if s_ >= 108:
                assert bd[m * 32 + i] == 0 and not val[:, m, i].any() and not val[:, m, i + 32].any()
                continue
            g, tap, comp = 2 * (s_ // 27) + hh, (s_ % 27) // 3, s_ % 3
            src = (g * 18 + 2 * tap + comp) if comp < 2 else 144 + g * 9 + tap
            seen.add(src)
            assert bd[m * 32 + i] == b[src]
            for k in range(36):
                c, t = divmod(k, 9)
                for lane in (i, i + 32):
                    ci = 16 * c + 8 * (lane >> 5) + np.arange(8)
                    assert np.abs(val[k, m, lane] - w[src, ci, t // 3, t % 3]).max() <= 2e-7 * np.abs(w).max()
    assert seen == set(range(216))
    # the DCN weight for the fused kernel: two deformable groups per K step
    wc = (rng.standard_normal((64, 64, 3, 3)) * 0.1).astype(np.float32)
    mode2 = L.PACK_DCNPAIR | L.PACK_F16X3
    wd2 = np.empty(lib.stif_conv_weight_floats(64, 64, 3, mode2), np.float32)
    bd2 = np.empty(lib.stif_conv_bias_floats(64, mode2), np.float32)
    L.check(lib.stif_pack_conv_weight(wc.ctypes.data, b.ctypes.data, 64, 64, 3, mode2, wd2.ctypes.data,
                                      bd2.ctypes.data), "pack")
    h2 = wd2.view(np.float16).reshape(4, 9, 2, 2, 64, 8).astype(np.float64)
    v2 = (h2[:, :, :, 0] + h2[:, :, :, 1]) / 1024.0             # [pair][tap][nt][lane][e]
    for pa in range(4):
        for t in range(9):
            for nt in range(2):
                for lane in (0, 5, 31, 32, 47, 63):
                    ci = 8 * (2 * pa + (lane >> 5)) + np.arange(8)
                    assert np.abs(v2[pa, t, nt, lane] - wc[nt * 32 + (lane & 31), ci, t // 3, t % 3]).max() <= 2e-7 * np.abs(wc).max()
    assert (bd2 == b[:64]).all()
    # both modes exist for split-fp16 operands only
    for md in (L.PACK_DCNSEP, L.PACK_DCNPAIR):
        with pytest.raises(L.StifError):
            L.check(lib.stif_pack_conv_weight(w.ctypes.data, b.ctypes.data, 216 if md == L.PACK_DCNSEP else 64, 64, 3,
                                              md, wd.ctypes.data, bd.ctypes.data), "pack")
