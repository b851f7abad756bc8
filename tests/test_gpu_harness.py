"""Video-harness data formats on the GPU (custom_video_test.py:88-110): imresize_np input resize,
uint8 output quantisation, and the folder driver."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_resize_frames_matches_reference(stif):
    h = np.load(os.path.join(GOLD, "harness.npz"))
    for k in ("37x50", "64x90", "21x33"):
        out = stif.video.resize_frames(h["img_" + k][None]).cpu().numpy()[0]          # [3, oh, ow] RGB / 255
        ref = (h["half_" + k].astype(np.float32) / 255.0)[:, :, ::-1].transpose(2, 0, 1)
        assert out.shape == ref.shape
        assert np.abs(out - ref).max() < 1e-6, k


def test_frames_to_u8_truncates_like_numpy(stif):
    x = torch.linspace(-0.2, 1.2, 3 * 7 * 11, device="cuda").view(1, 3, 7, 11)
    x[0, 0, 0, :4] = torch.tensor([0.999, 254.9 / 255, 1.0, 0.5 / 255])
    got = stif.video.frames_to_u8(x).cpu().numpy()[0]
    ref = (x.clamp(0, 1)[0].permute(1, 2, 0).cpu() * 255).numpy().astype(np.uint8)
    assert np.array_equal(got, ref)


def test_run_folder(stif, sd, tmp_path):
    from PIL import Image
    src = tmp_path / "in"
    src.mkdir()
    rng = np.random.default_rng(5)
    for k in range(3):
        Image.fromarray(rng.integers(0, 256, (22, 26, 3), dtype=np.uint8)).save(src / f"{k:03d}.png")
    m = stif.LunaTokis(64, 6, 8, 5, 40)
    m.load_state_dict(sd)
    stif.video.run_folder(m, str(src), str(tmp_path / "out"), times=[0.0, 0.5])
    assert sorted(os.listdir(tmp_path / "out" / "HR")) == [f"{i}.jpg" for i in range(4)]
    assert len(os.listdir(tmp_path / "out" / "bicubic")) == 4 and len(os.listdir(tmp_path / "out" / "LR")) == 2
    im = np.asarray(Image.open(tmp_path / "out" / "HR" / "0.jpg"))
    assert im.shape == (48, 64, 3)      # LR 11x13, zero-padded to 12x16 (custom_video_test.py:44-48), x4
