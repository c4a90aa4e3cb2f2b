"""GEO_FLAG_MIPS pieces on the CPU: the product header's mip chain and level of
detail (geo_pixel.h mip_down / lod_q8, host build) equal the oracle's
restatement, and the chain is the box filter it specifies (numpy)."""
import ctypes

import numpy as np
import pytest

import oracle as O
from test_host_kernel_math import host  # noqa: F401  (fixture)


def _host_chain(lib, sky):
    h, w = sky.shape[:2]
    out = np.empty(int(O.lib.geo_oracle_mip_chain_texels(w, h)), np.uint32)
    lib.host_mip_chain(ctypes.c_void_p(sky.ctypes.data), ctypes.c_uint32(w), ctypes.c_uint32(h),
                       ctypes.c_void_p(out.ctypes.data))
    return out


def _box(level):
    """numpy restatement: 2 x 2 means, block indices clamped (odd sizes)."""
    h, w = level.shape[:2]
    h2, w2 = max(1, h // 2), max(1, w // 2)
    ys = np.minimum(np.arange(h2)[:, None] * 2 + np.array([0, 1]), h - 1)
    xs = np.minimum(np.arange(w2)[:, None] * 2 + np.array([0, 1]), w - 1)
    a = level.astype(np.int64)
    s = sum(a[ys[:, j]][:, xs[:, i]] for j in range(2) for i in range(2))
    return ((s + 2) >> 2).astype(np.uint8)


@pytest.mark.parametrize("w,h", [(256, 128), (37, 19), (1, 5), (6, 1), (3, 3)])
def test_mip_chain_host_equals_oracle_and_box_filter(host, w, h):  # noqa: F811
    sky = np.random.default_rng(w * 131 + h).integers(0, 256, size=(h, w, 4), dtype=np.uint8)
    levels = O.mip_chain(sky)
    assert np.array_equal(levels[0], sky)
    for l in range(1, 4):
        assert levels[l].shape == (max(1, h >> l), max(1, w >> l), 4)
        assert np.array_equal(levels[l], _box(levels[l - 1])), l
    flat = np.concatenate([lv.reshape(-1, 4) for lv in levels]).view(np.uint32).ravel()
    assert np.array_equal(_host_chain(host, np.ascontiguousarray(sky)), flat)


def test_lod_host_equals_oracle_sweep(host):  # noqa: F811
    """Every 5th float in [1/2, 128], the specials, and the level bounds."""
    bits = np.arange(np.float32(0.5).view(np.uint32), np.float32(128.0).view(np.uint32), 5, dtype=np.uint32)
    x = np.concatenate([bits.view(np.float32), np.array([0.0, -1.0, 1.0, 4.0, 16.0, 64.0, np.inf, np.nan,
                                                           np.nextafter(np.float32(64), 0)], np.float32)])
    x = np.ascontiguousarray(x)
    a = np.empty(x.size, np.uint32)
    b = np.empty(x.size, np.uint32)
    host.host_lod_q8(ctypes.c_void_p(x.ctypes.data), ctypes.c_uint32(x.size), ctypes.c_void_p(a.ctypes.data))
    O.lib.geo_oracle_lod_q8_n(x.ctypes.data, x.size, b.ctypes.data)
    assert np.array_equal(a, b)
    # the specification: 256 * log2(rho2)/2 within one step of the exact value, clamped to [0, 768]
    ok = np.isfinite(x) & (x > 0)
    exact = np.clip(np.floor(128.0 * np.log2(x[ok].astype(np.float64))), 0, 768)
    assert np.abs(a[ok].astype(np.int64) - exact).max() <= 1
    assert a[~np.isfinite(x) & ~np.isinf(x)].max() == 0 and a[np.isinf(x)].min() == 768


def test_oracle_mips_keeps_mask_uv_steps(host):  # noqa: F811
    """The mip path changes colours only: mask, UV and steps are the level-0 render's."""
    from helpers import default_frame, default_scene
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    sky = make_sky("equirect", (256, 128))
    fr, sc = default_frame(66, 38), default_scene(512)
    m = O.render_mips_f32(fr, sc, sky, 66, 38, threads=4)
    l0 = O.render_f32(fr, sc, sky, 66, 38, threads=4)
    for f in ("mask", "uv", "steps"):
        assert np.array_equal(m[f], l0[f]), f
    assert m["steps_total"] == l0["steps_total"]
    assert (m["rgba"] != l0["rgba"]).any()  # minified: coarser levels
    with pytest.raises(ValueError):
        O.render_mips_f32(fr, sc, sky, 66, 38, row0=1, nrows=4)
