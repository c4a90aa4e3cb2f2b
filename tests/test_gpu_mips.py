"""GEO_FLAG_MIPS on the GPU: the trilinear mip-mapped sky (the reference's
Texture::new_with_mipmaps(..., 4) + textureSample, basic_sphere_buffer.rs:
31-36, shader.wgsl:101) equals the oracle's restatement (oracle
render_mips_f32) bit for bit, row blocks and band layouts compose to the full
frame, and odd row offsets are refused.  Colour only: mask, UV and steps are
the level-0 render's."""
import math

import numpy as np
import pytest

import oracle as O
from helpers import default_frame, default_scene

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_mod():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch


@pytest.fixture(scope="module")
def geo():
    import schwarzschild_raytracer_wgpu_amd as g

    return g


def mips(scene, geo):
    scene.flags |= geo._lib.GEO_FLAG_MIPS
    return scene


def render(geo, torch, ctx, frame, scene, w, h, row0=0, nrows=None, target=None):
    nrows = h - row0 if nrows is None else nrows
    dev = torch.device("cuda:0")
    if target is None:
        rgba = torch.empty(nrows * w * 4, dtype=torch.uint8, device=dev)
    else:
        rgba = torch.from_numpy(np.ascontiguousarray(target).reshape(-1)).to(dev)
    mask = torch.empty(nrows * w, dtype=torch.uint8, device=dev)
    uv = torch.empty(nrows * w * 2, dtype=torch.float32, device=dev)
    steps = torch.empty(nrows * w, dtype=torch.int32, device=dev)
    total = torch.zeros(1, dtype=torch.int64, device=dev)
    ctx.render_rows(frame, scene, w, h, row0, nrows, rgba, mask, uv, steps, total)
    torch.cuda.synchronize()
    return dict(rgba=rgba.cpu().numpy().reshape(nrows, w, 4), mask=mask.cpu().numpy().reshape(nrows, w),
                uv=uv.cpu().numpy().reshape(nrows, w, 2),
                steps=steps.cpu().numpy().view(np.uint32).reshape(nrows, w), total=int(total.item()))


def same(hip, ref):
    for f in ("rgba", "mask", "steps"):
        bad = np.argwhere(hip[f] != ref[f])
        assert bad.size == 0, f"{f} differs at {len(bad)} places, first {bad[:4]}"
    assert np.array_equal(hip["uv"].view(np.uint32), ref["uv"].view(np.uint32))
    assert hip["total"] == ref["steps_total"]


def sky_of(kind, size):
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    if kind == "random_alpha":
        return np.random.default_rng(7).integers(0, 256, size=(size[1], size[0], 4), dtype=np.uint8)
    return make_sky(kind, size)


SCENES = [
    # name, w, h, frame kwargs, scene kwargs, sky, sky size
    ("default_64x36", 64, 36, {}, dict(max_steps=512), "equirect", (256, 128)),
    ("odd_333x187", 333, 187, {}, dict(max_steps=512), "equirect", (512, 256)),
    ("big_sky_160x90", 160, 90, {}, dict(max_steps=512), "equirect", (4096, 2048)),
    ("odd_sky_121x67", 121, 67, {}, dict(max_steps=512), "equirect", (37, 19)),
    ("translucent", 120, 68, {}, dict(max_steps=512), "random_alpha", (128, 64)),
    ("inside_photon_sphere", 192, 108, dict(pos=(1.3 * math.cos(0.2), 1.3 * math.sin(0.2), 0.05),
                                            camera=(math.pi + 0.6, 0.3)),
     dict(max_steps=2048, r_obs=math.sqrt(1.3 ** 2 + 0.05 ** 2)), "equirect", (512, 256)),
    ("flat_space", 128, 72, dict(rs=0.0, state=0), dict(rs=0.0, max_steps=512), "equirect", (512, 256)),
    ("single_row", 97, 1, {}, dict(max_steps=512), "equirect", (256, 128)),
]


@pytest.mark.parametrize("name,w,h,fk,sk,skykind,skysize", SCENES, ids=[s[0] for s in SCENES])
def test_mips_match_oracle_bitexact(geo, torch_mod, name, w, h, fk, sk, skykind, skysize):
    sky = sky_of(skykind, skysize)
    frame, scene = default_frame(w, h, **fk), mips(default_scene(**sk), geo)
    ctx = geo.Context(0)
    ctx.set_sky(sky)
    hip = render(geo, torch_mod, ctx, frame, scene, w, h)
    ref = O.render_mips_f32(frame, scene, sky, w, h, threads=8)
    same(hip, ref)
    # colour only: the level-0 render has the same mask, UV and steps
    l0 = O.render_f32(frame, default_scene(**sk), sky, w, h, threads=8)
    assert np.array_equal(hip["mask"], l0["mask"]) and np.array_equal(hip["steps"], l0["steps"])


def test_mips_adaptive_and_fan_modes(geo, torch_mod):
    sky = sky_of("equirect", (512, 256))
    w, h = 96, 54
    frame = default_frame(w, h)
    ctx = geo.Context(0)
    ctx.set_sky(sky)
    scene = mips(default_scene(max_steps=256, mode=geo.GEO_MODE_ADAPTIVE), geo)
    same(render(geo, torch_mod, ctx, frame, scene, w, h), O.render_mips_f32(frame, scene, sky, w, h, threads=8))
    fan = O.solve_ray_fan(50.0, 1.0, 1000, math.pi / 100, 400, float(np.sqrt(2.5 ** 2 + 0.1 ** 2)))
    ctx.set_fan(fan)
    scene = mips(default_scene(mode=geo.GEO_MODE_FAN), geo)
    hip = render(geo, torch_mod, ctx, frame, scene, w, h)
    ref = O.render_mips_f32(frame, scene, sky, w, h, fan=fan, threads=8)
    for f in ("rgba", "mask"):
        assert np.array_equal(hip[f], ref[f]), f


def test_mips_fan_mode_ragged_rows_bands_composite(geo, torch_mod):
    """The mip-mapped fan draw (the reference's sampler on its display
    path): ragged frames, even row blocks, 8-row bands and a composite over a
    target, bit for bit."""
    sky = sky_of("random_alpha", (200, 90))
    fan = O.solve_ray_fan(50.0, 1.0, 1000, math.pi / 100, 400, float(np.sqrt(2.5 ** 2 + 0.1 ** 2)))
    ctx = geo.Context(0)
    ctx.set_sky(sky)
    ctx.set_fan(fan)
    for (w, h) in ((65, 37), (34, 20)):
        frame = default_frame(w, h)
        scene = mips(default_scene(mode=geo.GEO_MODE_FAN), geo)
        ref = O.render_mips_f32(frame, scene, sky, w, h, fan=fan, threads=8)
        same(render(geo, torch_mod, ctx, frame, scene, w, h), ref)
        for r0, n in ((2, h - 2), (h - 1 - ((h - 1) & 1), 1 + ((h - 1) & 1))):
            hip = render(geo, torch_mod, ctx, frame, scene, w, h, row0=r0, nrows=n)
            assert np.array_equal(hip["rgba"], ref["rgba"][r0:r0 + n]), (w, h, r0)
        nb = (h + 7) // 8
        rgba = torch_mod.empty(nb * 8 * w * 4, dtype=torch_mod.uint8, device=torch_mod.device("cuda:0"))
        ctx.render_bands(frame, scene, w, h, 8, 0, 1, nb, rgba)
        torch_mod.cuda.synchronize()
        got = rgba.cpu().numpy().reshape(nb * 8, w, 4)[:h]
        assert np.array_equal(got, ref["rgba"]), (w, h)
        target = np.random.default_rng(w).integers(0, 256, size=(h, w, 4), dtype=np.uint8)
        cs = mips(default_scene(mode=geo.GEO_MODE_FAN), geo)
        cs.flags |= geo._lib.GEO_FLAG_COMPOSITE
        hip = render(geo, torch_mod, ctx, frame, cs, w, h, target=target)
        assert np.array_equal(hip["rgba"], O.render_mips_f32(frame, cs, sky, w, h, fan=fan, threads=8,
                                                             target=target)["rgba"]), (w, h)
    ctx.close()


def test_mips_composite_over_target(geo, torch_mod):
    sky = sky_of("random_alpha", (128, 64))
    w, h = 80, 46
    frame, scene = default_frame(w, h), default_scene(max_steps=512)
    scene.flags |= geo._lib.GEO_FLAG_COMPOSITE | geo._lib.GEO_FLAG_MIPS
    target = np.random.default_rng(11).integers(0, 256, size=(h, w, 4), dtype=np.uint8)
    ctx = geo.Context(0)
    ctx.set_sky(sky)
    hip = render(geo, torch_mod, ctx, frame, scene, w, h, target=target)
    ref = O.render_mips_f32(frame, scene, sky, w, h, threads=8, target=target)
    assert np.array_equal(hip["rgba"], ref["rgba"])


def test_mips_row_blocks_and_bands_compose(geo, torch_mod):
    """Even row offsets (odd row counts included: the last row's quad partner
    is a helper below it) compose to the full frame; bands of 8 rows for 3
    ranks too.  An odd row0 is refused."""
    sky = sky_of("equirect", (512, 256))
    w, h = 150, 101
    frame, scene = default_frame(w, h), mips(default_scene(2048), geo)
    ctx = geo.Context(0)
    ctx.set_sky(sky)
    full = render(geo, torch_mod, ctx, frame, scene, w, h)
    parts = [render(geo, torch_mod, ctx, frame, scene, w, h, r0, n) for r0, n in ((0, 50), (50, 1), (52, 49))]
    got = np.concatenate([parts[0]["rgba"], parts[1]["rgba"], full["rgba"][51:52], parts[2]["rgba"]])
    assert np.array_equal(got, full["rgba"])
    dev = torch_mod.device("cuda:0")
    B, world = 8, 3
    for r in range(world):
        nb = (-(-h // B) - r + world - 1) // world
        if nb <= 0:
            continue
        out = torch_mod.empty(nb * B * w * 4, dtype=torch_mod.uint8, device=dev)
        ctx.render_bands(frame, scene, w, h, B, r, world, nb, out)
        torch_mod.cuda.synchronize()
        o = out.cpu().numpy().reshape(nb * B, w, 4)
        for j in range(nb):
            y0 = (r + j * world) * B
            n = min(B, h - y0)
            assert np.array_equal(o[j * B:j * B + n], full["rgba"][y0:y0 + n]), (r, j)
    from schwarzschild_raytracer_wgpu_amd._lib import GeoError

    with pytest.raises(GeoError):
        render(geo, torch_mod, ctx, frame, scene, w, h, 1, 10)


def test_basic_sphere_buffer_mipmaps(geo, torch_mod):
    """BasicSphereBuffer(..., mipmaps=True) draws the GEO_FLAG_MIPS frame (the
    reference's sampler) through the host mirror."""
    sky = sky_of("equirect", (512, 256))
    w, h = 128, 72
    frame = default_frame(w, h)
    r = float(np.sqrt(2.5 ** 2 + 0.1 ** 2))
    sphere = geo.BasicSphereBuffer(0, 50.0, 1.0, sky, mipmaps=True)
    sphere.update_ray_fan(r)
    rgba = torch_mod.empty(h * w * 4, dtype=torch_mod.uint8, device=torch_mod.device("cuda:0"))
    sphere.draw(frame, geo.RenderTarget(w, h, rgba))
    torch_mod.cuda.synchronize()
    ref = O.render_mips_f32(frame, sphere.scene(), sky, w, h, threads=8)
    assert np.array_equal(rgba.cpu().numpy().reshape(h, w, 4), ref["rgba"])
    assert sphere.scene().max_steps == 1000 and sphere.scene().flags == geo._lib.GEO_FLAG_MIPS


def test_mips_4k_config_rows(geo, torch_mod):
    """Config 3's 4K frame with the mip-mapped sampler (its 4096 x 2048 sky):
    row blocks across the frame equal the oracle's mip restatement."""
    from schwarzschild_raytracer_wgpu_amd.scenes import CONFIGS, make_sky

    cfg = CONFIGS["cfg3_4k"]
    w, h = cfg.width, cfg.height
    obs = geo.Observer(cfg.rs, cfg.fov, w, h)
    obs.set_position(*cfg.position)
    obs.set_camera(*cfg.camera)
    frame = obs.calc_transformation_pipeline()
    scene = mips(geo.make_scene(cfg.rs, cfg.sphere_r, obs.get_radial_position(), cfg.step, cfg.max_steps), geo)
    sky = make_sky(cfg.sky, cfg.sky_size)
    ctx = geo.Context(0)
    ctx.set_sky(sky)
    full = render(geo, torch_mod, ctx, frame, scene, w, h)
    for r0 in (0, 540, 1080, 1618, 2150):
        ref = O.render_mips_f32(frame, scene, sky, w, h, row0=r0, nrows=10, threads=16)
        for f in ("rgba", "mask", "steps"):
            assert np.array_equal(full[f][r0:r0 + 10], ref[f]), (f, r0)
