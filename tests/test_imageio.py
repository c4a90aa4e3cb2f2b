"""N4 image IO (schwarzschild_raytracer_wgpu_amd/imageio.py): texture loading
as image::load_from_memory(..).to_rgba8() does it, frame dumps.  CPU only."""
import numpy as np
import pytest

from schwarzschild_raytracer_wgpu_amd import imageio


def test_png_roundtrip_and_rgba_conversion(tmp_path):
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, size=(37, 53, 4), dtype=np.uint8)
    p = str(tmp_path / "a.png")
    imageio.save_png(p, img.reshape(-1), 53, 37)
    assert np.array_equal(imageio.load_texture(p), img)
    # an RGB file gains alpha 255, like to_rgba8()
    from PIL import Image

    q = str(tmp_path / "b.png")
    Image.fromarray(img[..., :3], "RGB").save(q)
    t = imageio.load_texture(q)
    assert t.shape == (37, 53, 4) and np.all(t[..., 3] == 255) and np.array_equal(t[..., :3], img[..., :3])


def test_ppm_roundtrip(tmp_path):
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, size=(20, 31, 4), dtype=np.uint8)
    img[..., 3] = 255
    p = str(tmp_path / "f.ppm")
    imageio.save_ppm(p, img, 31, 20)
    assert np.array_equal(imageio.load_ppm(p), img)


def test_frame_to_host_accepts_tensors_and_checks_size():
    import torch

    t = torch.arange(4 * 6 * 4, dtype=torch.uint8)
    a = imageio.frame_to_host(t, 6, 4)
    assert a.shape == (4, 6, 4) and a[0, 1, 0] == 4
    with pytest.raises(ValueError):
        imageio.frame_to_host(t, 7, 4)
