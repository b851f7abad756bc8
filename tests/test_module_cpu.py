"""Host-side (no GPU) coverage of the model API as an nn.Module and of the f16x3 weight-range guard
at packing time (the packers run on the CPU)."""
import numpy as np
import pytest
import torch


@pytest.fixture(scope="module")
def cpu_model(stif, sd):
    m = stif.LunaTokis(64, 6, 8, 5, 40, device="cpu")
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    return m


def test_parameters_are_the_reference_state_dict(cpu_model, sd):
    """442 keys in the reference's registration order, 11,312,698 parameters,
    values as loaded; packed kernel copies are non-persistent (not in state_dict)."""
    msd = cpu_model.state_dict()
    assert list(msd.keys()) == list(sd.keys())
    assert sum(p.numel() for p in cpu_model.parameters()) == 11312698
    for k in ("conv_first.weight", "pcd_align.L1_dcnpack_2.conv_offset_mask.bias", "encode_imnet.net.4.weight"):
        assert np.array_equal(msd[k].numpy(), sd[k])
    assert all(not p.requires_grad for p in cpu_model.parameters())
    assert len(list(cpu_model.buffers())) > 300          # packed layers ride along with .to()/replicate


def test_load_state_dict_contract(stif, sd):
    m = stif.LunaTokis(64, 6, 8, 5, 40, device="cpu")
    m.load_state_dict({"module." + k: torch.from_numpy(v) for k, v in sd.items()})   # base_model.py:93-98
    bad = dict(sd)
    del bad["fusion.bias"]
    with pytest.raises(RuntimeError, match="Missing key"):
        m.load_state_dict(bad)
    bad = dict(sd)
    bad["fusion.bias"] = np.zeros(3, np.float32)
    with pytest.raises(RuntimeError, match="size mismatch"):
        m.load_state_dict(bad)
    r = m.load_state_dict({"fusion.bias": sd["fusion.bias"]}, strict=False)
    assert len(r.missing_keys) == 441


def test_module_behaviour(stif, cpu_model):
    assert cpu_model.eval() is cpu_model and not cpu_model.training
    with pytest.raises(NotImplementedError):
        cpu_model.train()
    with pytest.raises(NotImplementedError):
        cpu_model.to(torch.float16)
    with pytest.raises(NotImplementedError):
        cpu_model.half()
    dp = torch.nn.DataParallel(cpu_model)             # VideoSR_base_model.py:31-32 (no GPU: plain call)
    assert dp.module is cpu_model
    with pytest.raises(stif._lib.StifError, match="GPU only"):
        cpu_model(torch.zeros(1, 2, 3, 8, 8), [0.5])


def test_f16x3_weight_range_fallback_at_pack(stif):
    L, ops = stif._lib, stif.ops
    rng = np.random.default_rng(0)
    w = rng.standard_normal((64, 64, 3, 3)).astype(np.float32) * 0.05
    b = np.zeros(64, np.float32)
    assert ops.pack_conv(w, b, L.PACK_WINO | L.PACK_F16X3, "cpu").mode == L.PACK_WINO | L.PACK_F16X3
    big = w.copy()
    big[3, 5, 0, 0] = 70.0                            # U[0][0] = g[0][0] >= 64: not representable split
    assert ops.pack_conv(big, b, L.PACK_WINO | L.PACK_F16X3, "cpu").mode == L.PACK_WINO
    with pytest.raises(L.StifError, match="f16x3 range") as e:
        ops.pack_conv(big, b, L.PACK_WINO | L.PACK_F16X3, "cpu", range_fallback=False)
    assert e.value.code == L.E_RANGE
    assert ops.pack_conv(big, b, L.PACK_PLAIN | L.PACK_F16X3, "cpu").mode == L.PACK_PLAIN   # DCN core


def test_model_packs_out_of_range_layers_in_fp32(stif, sd):
    L = stif._lib
    sd2 = dict(sd)
    sd2["recon_trunk.7.conv2.weight"] = sd["recon_trunk.7.conv2.weight"] * 3000.0
    # x 30 / (2 pi) (the f16x3 packing's sine scale, in revolutions): > 64
    sd2["encode_imnet.net.3.linear.weight"] = sd["encode_imnet.net.3.linear.weight"] * 10000.0
    m = stif.LunaTokis(64, 6, 8, 5, 40, device="cpu")
    m.load_state_dict(sd2)
    lay = m._build_layers(m._pk, m._meta)
    assert lay["recon_trunk.7.conv2"].mode == L.PACK_WINO
    assert lay["recon_trunk.7.conv1"].mode == L.PACK_WINO | L.PACK_F16X3
    assert m._dec_flags == 0 and m._meta["dec.mlp"][1] == 0


def test_const_cache_is_device_scoped_and_bounded(stif, cpu_model):
    """_const (the weight-only constant maps): entries are grouped by (device, shape), at most
    const_shapes groups per device are kept (least recently used evicted), a replica sharing the dict
    on another device never receives this device's tensors, and .to() drops the groups of the device
    the module left (advisor r5)."""
    import copy
    m = cpu_model
    m._consts.clear()
    calls = []

    def mk(tag):
        calls.append(tag)
        return torch.full((1,), float(len(calls)))

    a = m._const(("k", 1), (2, 8, 8), lambda: mk("a"))
    assert m._const(("k", 1), (2, 8, 8), lambda: mk("x")) is a and calls == ["a"]
    m._const(("k", 1), (2, 16, 16), lambda: mk("b"))
    m._const(("k", 1), (2, 8, 8), lambda: mk("y"))          # hit: (2, 8, 8) becomes most recent
    m._const(("k", 1), (2, 32, 32), lambda: mk("c"))        # third shape: evicts (2, 16, 16)
    assert calls == ["a", "b", "c"] and list(m._consts) == [("cpu", 2, 8, 8), ("cpu", 2, 32, 32)]
    assert m._zeros(2, 8, 8, 64).shape == (2, 8, 8, 64) and ("zeros", 2, 8, 8, 64) in m._consts[("cpu", 2, 8, 8)]
    # a replica whose device differs (DataParallel shares __dict__ entries shallowly): its own group
    class OnMeta(type(m)):
        device = property(lambda self: torch.device("meta"))

    rep = copy.copy(m)
    rep.__class__ = OnMeta
    assert rep._consts is m._consts
    r = rep._const(("k", 1), (2, 8, 8), lambda: mk("rep"))
    assert r is not a and calls[-1] == "rep" and ("meta", 2, 8, 8) in m._consts
    m.to("cpu")                                                # leaving "meta"-device entries behind
    assert all(g[0] == "cpu" for g in m._consts)
    with pytest.raises(ValueError):
        stif.LunaTokis(64, 6, 8, 5, 40, device="cpu", const_shapes=0)
