"""GEO_FLAG_RING_F64 (geo.h, geo_band.h; DESIGN.md §2, "The capture band in
f64"): the pixels next to the capture orbit take their traveled angle from
an f64 path inside the render kernel.

Against the oracle (render_f32 with the flag: its f32 mirror, and the band
by its own f64 restatement, oracle band_lambda): every output bit for bit,
the band included (the band is decided on the f32 ray by the same f32
operations; its f64 arithmetic is IEEE + - * / sqrt fma on both sides).
Against the f64 literal (the reference's algorithm): the band's mask and
steps exactly, on whole config frames every pixel inside north_star's bar.
"""
import math
import os

import numpy as np
import pytest

import f64_bar as B
import oracle as O
from fuzz_scenes import random_scene
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


def _render(geo, torch, ctx, frame, scene, w, h):
    dev = torch.device("cuda:0")
    rgba = torch.empty(h * w * 4, dtype=torch.uint8, device=dev)
    mask = torch.empty(h * w, dtype=torch.uint8, device=dev)
    uv = torch.empty(h * w * 2, dtype=torch.float32, device=dev)
    steps = torch.empty(h * w, dtype=torch.int32, device=dev)
    tot = torch.zeros(1, dtype=torch.int64, device=dev)
    ctx.render_rows(frame, scene, w, h, 0, h, rgba, mask, uv, steps, tot)
    torch.cuda.synchronize()
    return dict(rgba=rgba.cpu().numpy().reshape(h, w, 4), mask=mask.cpu().numpy().reshape(h, w),
                uv=uv.cpu().numpy().reshape(h, w, 2), steps=steps.cpu().numpy().view(np.uint32).reshape(h, w),
                total=int(tot.item()))


def _ring(geo, scene):
    s = geo.GeoScene.from_buffer_copy(bytes(scene))
    s.flags |= geo._lib.GEO_FLAG_RING_F64
    return s


def _compare(hip, ref):
    for f in ("mask", "steps", "rgba"):
        assert np.array_equal(hip[f], ref[f]), f"{f} differs"
    assert np.array_equal(hip["uv"].view(np.uint32), ref["uv"].view(np.uint32)), "uv differs"
    assert hip["total"] == ref["steps_total"]


def test_ring_default_pose_against_the_oracle(geo, torch_mod):
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    w, h = 480, 270
    sky = make_sky("equirect", (512, 256))
    ctx = geo.Context(0)
    ctx.set_sky(sky)
    for cam in [(math.pi, 0.0), (math.pi + 0.3, 0.2), (math.pi - 0.5, -0.4)]:
        frame = default_frame(w, h, camera=cam)
        scene = _ring(geo, default_scene(2048))
        hip = _render(geo, torch_mod, ctx, frame, scene, w, h)
        ref = O.render_f32(frame, scene, sky, w, h, threads=8)
        band = O.ring_band(frame, scene, w, h).astype(bool)
        assert band.sum() > 100  # the frame crosses the orbit's band
        _compare(hip, ref)
        # the band against the f64 literal: the same mask and steps, the UV far inside the bar
        lit = O.render_f64(frame, default_scene(2048), w, h, threads=8)
        assert np.array_equal(hip["mask"][band], lit["mask"][band])
        assert np.array_equal(hip["steps"][band], lit["steps"][band])
        print("ring default pose", cam, int(band.sum()), "band pixels")
    ctx.close()


def test_ring_adaptive_against_the_oracle(geo, torch_mod):
    """In the adaptive mode the band's lanes take the same f64 fixed-step path
    (config 5's band fix: its f32 error there is the tolerance's)."""
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    w, h = 320, 180
    sky = make_sky("equirect", (256, 128))
    ctx = geo.Context(0)
    ctx.set_sky(sky)
    for pos, cam in [((2.5, 0.0, 0.1), (math.pi, 0.0)), ((1.2, 0.5, 0.0), (math.pi + 0.6, 0.3))]:
        frame = default_frame(w, h, camera=cam, pos=pos)
        r = math.sqrt(sum(c * c for c in pos))
        scene = _ring(geo, geo.make_scene(1.0, 50.0, r, math.pi / 100, 2048, geo.GEO_MODE_ADAPTIVE, tol=1e-6))
        hip = _render(geo, torch_mod, ctx, frame, scene, w, h)
        ref = O.render_f32(frame, scene, sky, w, h, threads=8)
        assert O.ring_band(frame, scene, w, h).sum() > 50
        _compare(hip, ref)
    ctx.close()


def test_ring_fuzz_scenes_against_the_oracle(geo, torch_mod):
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    w, h = 96, 54
    sky = make_sky("equirect", (256, 128))
    ctx = geo.Context(0)
    ctx.set_sky(sky)
    seen = 0
    n = int(os.environ.get("GEO_FUZZ_N", 300))
    base = int(os.environ.get("GEO_FUZZ_BASE", 40_000))
    for seed in range(base, base + n):
        frame, scene, desc = random_scene(seed, w, h)
        if scene.mode == geo.GEO_MODE_FAN:
            continue
        scene = _ring(geo, scene)
        hip = _render(geo, torch_mod, ctx, frame, scene, w, h)
        ref = O.render_f32(frame, scene, sky, w, h, threads=8)
        seen += int(O.ring_band(frame, scene, w, h).any())
        _compare(hip, ref)
    print(f"fuzz ring: {n} scenes, {seen} with band pixels, bit for bit")
    assert seen > n // 10
    ctx.close()


def test_ring_band_set_equals_rows(geo, torch_mod):
    """The redraw follows the launch's band mapping: a band set equals the
    same rows of the whole frame."""
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    torch = torch_mod
    w, h = 320, 180
    dev = torch.device("cuda:0")
    ctx = geo.Context(0)
    ctx.set_sky(make_sky("equirect", (256, 128)))
    frame = default_frame(w, h)
    scene = _ring(geo, default_scene(2048))
    full = torch.empty(h * w * 4, dtype=torch.uint8, device=dev)
    ctx.render_rows(frame, scene, w, h, 0, h, full)
    row0, stride, band_rows = 8, 24, 8
    nb = (h - row0 + stride - 1) // stride
    out = torch.empty(nb * band_rows * w * 4, dtype=torch.uint8, device=dev)
    ctx.render_band_set(frame, scene, w, h, band_rows, row0, stride, nb, out)
    torch.cuda.synchronize()
    img = full.view(h, w, 4).cpu().numpy()
    got = out.view(nb * band_rows, w, 4).cpu().numpy()
    rows = [y for j in range(nb) for y in range(row0 + j * stride, row0 + j * stride + band_rows)]
    for k, y in enumerate(rows):
        if y < h:
            assert np.array_equal(got[k], img[y]), y
    ctx.close()


@pytest.mark.parametrize("cfgname", ["cfg2_1080p", "cfg3_4k"])
def test_ring_config_frame_meets_the_bar_everywhere(geo, torch_mod, cfgname):
    """Whole config frames against the f64 literal: with the flag no pixel is
    over the 1e-4 UV bar (the capture band and the sky's poles included) and
    no mask flips; the same frame without it has pixels over the bar next to
    the orbit (profiles/r05p_f64_full_frame.json)."""
    from schwarzschild_raytracer_wgpu_amd.scenes import CONFIGS, make_sky

    torch = torch_mod
    cfg = CONFIGS[cfgname]
    w, h = cfg.width, cfg.height
    obs = geo.Observer(cfg.rs, cfg.fov, w, h)
    obs.set_position(*cfg.position)
    obs.set_camera(*cfg.camera)
    obs.set_energy(cfg.energy)
    frame = obs.calc_transformation_pipeline()
    r = obs.get_radial_position()
    scene = geo.make_scene(cfg.rs, cfg.sphere_r, r, cfg.step, cfg.max_steps, geo.GEO_MODE_DIRECT)
    ctx = geo.Context(0)
    ctx.set_sky(make_sky("equirect", (512, 256)))
    dev = torch.device("cuda:0")
    rgba = torch.empty(h * w * 4, dtype=torch.uint8, device=dev)
    mask = torch.empty(h * w, dtype=torch.uint8, device=dev)
    uv = torch.empty(h * w * 2, dtype=torch.float32, device=dev)
    ctx.render_rows(frame, _ring(geo, scene), w, h, 0, h, rgba, mask, uv)
    torch.cuda.synchronize()
    m = mask.view(h, w).cpu().numpy()
    u = uv.view(h, w, 2).cpu().numpy()
    ref = O.render_f64(frame, scene, w, h, threads=16)
    sky = (m == 0) & (ref["mask"] == 0)
    e = B.uv_err(u, ref["uv"])
    over = int((sky & (e > B.UV_BAR)).sum())
    flips = int((m != ref["mask"]).sum())
    print(f"{cfgname} ring: uv max {e[sky].max():.3e}, over the bar {over}, mask flips {flips}")
    assert flips == 0
    assert over == 0
    ctx.close()


def test_ring_config5_meets_the_bar_against_the_fine_reference(geo, torch_mod):
    """Config 5 (8K, adaptive RK5(4), observer inside the photon sphere) with
    the flag, against the adaptive mode's own f64 check (fixed RK4 at
    step/32) on every 54th row, with no model band: no mask flip, and every
    sky pixel within the 1e-4 UV bar except at the poles (|latitude| > 89
    deg, where U's sensitivity to the direction, 1/(2 pi cos lat), is over 9x
    the equator's).  Without the flag the same rows have pixels over the bar
    next to the orbit (the adaptive tolerance's error there)."""
    from schwarzschild_raytracer_wgpu_amd.scenes import CONFIGS, make_sky

    torch = torch_mod
    cfg = CONFIGS["cfg5_8k_adaptive"]
    w, h = cfg.width, cfg.height
    obs = geo.Observer(cfg.rs, cfg.fov, w, h)
    obs.set_position(*cfg.position)
    obs.set_camera(*cfg.camera)
    obs.set_energy(cfg.energy)
    frame = obs.calc_transformation_pipeline()
    r = obs.get_radial_position()
    scene = geo.make_scene(cfg.rs, cfg.sphere_r, r, cfg.step, cfg.max_steps, geo.GEO_MODE_ADAPTIVE, tol=cfg.tol)
    ctx = geo.Context(0)
    ctx.set_sky(make_sky("equirect", (512, 256)))
    dev = torch.device("cuda:0")
    row_step = 54
    row0 = row_step // 2
    nrows = (h - row0 + row_step - 1) // row_step
    fine = B.f64_rows(frame, scene, w, h, row0, nrows, row_step)
    lat = np.pi * (0.5 - fine["uv"][..., 1].astype(np.float64))
    pole = np.abs(lat) > np.radians(89.0)
    res = {}
    for name, sc in (("plain", scene), ("ring", _ring(geo, scene))):
        rgba = torch.empty(h * w * 4, dtype=torch.uint8, device=dev)
        mask = torch.empty(h * w, dtype=torch.uint8, device=dev)
        uv = torch.empty(h * w * 2, dtype=torch.float32, device=dev)
        ctx.render_rows(frame, sc, w, h, 0, h, rgba, mask, uv)
        torch.cuda.synchronize()
        m = mask.view(h, w)[row0::row_step].cpu().numpy()
        u = uv.view(h, w, 2)[row0::row_step].cpu().numpy()
        sky = (m == 0) & (fine["mask"] == 0)
        e = B.uv_err(u, fine["uv"])
        res[name] = {"flips": int((m != fine["mask"]).sum()), "over": int((sky & ~pole & (e > B.UV_BAR)).sum()),
                     "uv_max_off_pole": float(e[sky & ~pole].max()), "pole_pixels": int((sky & pole).sum())}
    print("config 5 vs f64 step/32:", res)
    assert res["ring"]["flips"] == 0
    assert res["ring"]["over"] == 0
    assert res["plain"]["over"] > 0 or res["plain"]["flips"] > 0  # the band's adaptive error, fixed by the flag
    ctx.close()


def test_ring_rejects_what_it_does_not_draw(geo, torch_mod):
    import ctypes

    from schwarzschild_raytracer_wgpu_amd import _lib
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    torch = torch_mod
    w, h = 64, 32
    ctx = geo.Context(0)
    ctx.set_sky(make_sky("equirect", (64, 32)))
    frame = default_frame(w, h)
    out = torch.empty(2 * h * w * 4, dtype=torch.uint8, device=torch.device("cuda:0"))
    stream = torch.cuda.current_stream().cuda_stream

    def rows(scene):
        return _lib.lib.geo_render_rows(ctx._h, ctypes.byref(frame), ctypes.byref(scene), w, h, 0, h,
                                        out.data_ptr(), None, None, None, None, stream)

    ok = _ring(geo, default_scene(64))
    assert rows(ok) == _lib.GEO_OK
    s = _ring(geo, geo.make_scene(1.0, 50.0, 2.5, math.pi / 100, 64, geo.GEO_MODE_FAN))
    ctx.solve_ray_fan(50.0, 1.0, 1000, math.pi / 100, 400, 2.5, host=False)
    assert rows(s) == _lib.GEO_EINVAL
    assert rows(_ring(geo, geo.make_scene(1.0, 50.0, 2.5, math.pi / 100, 64, geo.GEO_MODE_ADAPTIVE))) == _lib.GEO_OK
    for flag in (_lib.GEO_FLAG_COMPOSITE, _lib.GEO_FLAG_MIPS):
        s = _ring(geo, default_scene(64))
        s.flags |= flag
        assert rows(s) == _lib.GEO_EINVAL, flag
    fa = (geo.GeoFrame * 2)(frame, frame)  # a batch draws the band too (test_ring_batched_launches_...)
    assert _lib.lib.geo_render_band_set_frames(ctx._h, fa, 2, ctypes.byref(ok), w, h, 8, 0, 8, 4, out.data_ptr(),
                                               h * w * 4, None, stream) == _lib.GEO_OK
    # no capture orbit (flat space, inside the horizon): the flag draws the f32 frame
    for s in (geo.make_scene(0.0, 50.0, 2.5, math.pi / 100, 64, geo.GEO_MODE_DIRECT),
              geo.make_scene(1.0, 50.0, 0.7, math.pi / 100, 64, geo.GEO_MODE_DIRECT)):
        assert O.ring_band(frame, _ring(geo, s), w, h).sum() == 0
        assert rows(_ring(geo, s)) == _lib.GEO_OK
    torch.cuda.synchronize()
    ctx.close()


def test_ring_across_streams_and_sizes(geo, torch_mod):
    """Ring frames on two streams in turn and of growing sizes, each equal to
    the same frame drawn alone by another context (the mode keeps no state
    between renders: its constants ride in the launch's arguments)."""
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    torch = torch_mod
    dev = torch.device("cuda:0")
    ctx = geo.Context(0)
    ctx.set_sky(make_sky("equirect", (256, 128)))
    scene = _ring(geo, default_scene(2048))
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    sizes = [(160, 90), (320, 180), (480, 270)]
    cams = [(math.pi + 0.1 * i, 0.05 * i) for i in range(6)]
    refs = {}
    ref_ctx = geo.Context(0)
    ref_ctx.set_sky(make_sky("equirect", (256, 128)))
    for w, h in sizes:
        for i, cam in enumerate(cams):
            out = torch.empty(h * w * 4, dtype=torch.uint8, device=dev)
            ref_ctx.render_rows(default_frame(w, h, camera=cam), scene, w, h, 0, h, out)
            refs[(w, h, i)] = out
    torch.cuda.synchronize()
    outs = {}
    for w, h in sizes:
        for i, cam in enumerate(cams):
            st = s1 if i % 2 == 0 else s2
            out = torch.empty(h * w * 4, dtype=torch.uint8, device=dev)
            with torch.cuda.stream(st):
                ctx.render_rows(default_frame(w, h, camera=cam), scene, w, h, 0, h, out, stream=st.cuda_stream)
            outs[(w, h, i)] = (out, st)
    torch.cuda.synchronize()
    for k, (out, _) in outs.items():
        assert torch.equal(out, refs[k]), k
    ctx.close()
    ref_ctx.close()


@pytest.mark.parametrize("mode", ["direct", "adaptive"])
def test_ring_batched_launches_equal_one_frame_launches(geo, torch_mod, mode):
    """GEO_FLAG_RING_F64 in batched launches (the multi-GPU pipeline's
    geo_render_band_set_frames / _batch): each frame's band factor rides in
    the batch and a wave with band lanes derives its frame's f64 constants
    (geo::band_consts_into, the host's operations) in its LDS slot.  Every
    frame of the batch equals its one-frame ring render byte for byte: three
    cameras in one launch, and a moving observer's frames (one radius each,
    one inside the photon sphere) through geo_render_band_set_batch; band
    layouts with a partial last band."""
    import ctypes

    from schwarzschild_raytracer_wgpu_amd import _lib
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    torch = torch_mod
    dev = torch.device("cuda:0")
    W, H, BR = 320, 180, 8
    ctx = geo.Context(0)
    ctx.set_sky(make_sky("equirect", (256, 128)))
    md = geo.GEO_MODE_ADAPTIVE if mode == "adaptive" else geo.GEO_MODE_DIRECT
    stream = torch.cuda.current_stream().cuda_stream

    def frame_at(pos, cam):
        obs = geo.Observer(1.0, math.pi / 2, W, H)
        obs.set_position(*pos)
        obs.set_camera(*cam)
        return obs.calc_transformation_pipeline(), obs.get_radial_position()

    def one(frame, scene, row0, stride, nb):
        o = torch.zeros(nb * BR * W * 4, dtype=torch.uint8, device=dev)
        ctx.render_band_set(frame, scene, W, H, BR, row0, stride, nb, o)
        return o

    for row0, stride, nb in ((0, 8, 23), (8, 24, 8), (16, 32, 6)):
        fb = nb * BR * W * 4
        # three cameras, one scene, one launch
        poses = [frame_at((2.5, 0.0, 0.1), (math.pi + d, 0.0)) for d in (0.0, 0.02, -0.03)]
        scene = _ring(geo, geo.make_scene(1.0, 50.0, poses[0][1], math.pi / 100, 512, md,
                                          tol=1e-6 if md == geo.GEO_MODE_ADAPTIVE else 0.0))
        out = torch.zeros(3 * fb, dtype=torch.uint8, device=dev)
        fa = (geo.GeoFrame * 3)(*[p[0] for p in poses])
        assert _lib.lib.geo_render_band_set_frames(ctx._h, fa, 3, ctypes.byref(scene), W, H, BR, row0, stride, nb,
                                                   out.data_ptr(), fb, None, stream) == _lib.GEO_OK
        for i, (fr, _) in enumerate(poses):
            assert torch.equal(out[i * fb:(i + 1) * fb], one(fr, scene, row0, stride, nb)), (row0, i)
        # a moving observer: one radius per frame (outside and inside the photon sphere)
        poses = [frame_at((r, 0.0, 0.1), (math.pi, 0.0)) for r in (2.5, 1.3, 4.0)]
        scenes = [_ring(geo, geo.make_scene(1.0, 50.0, rr, math.pi / 100, 512, md,
                                            tol=1e-6 if md == geo.GEO_MODE_ADAPTIVE else 0.0)) for _, rr in poses]
        sa = (geo.GeoScene * 3)(*scenes)
        fa = (geo.GeoFrame * 3)(*[p[0] for p in poses])
        out = torch.zeros(3 * fb, dtype=torch.uint8, device=dev)
        assert _lib.lib.geo_render_band_set_batch(ctx._h, fa, sa, 3, W, H, BR, row0, stride, nb, out.data_ptr(), fb,
                                                  None, stream) == _lib.GEO_OK
        for i, (fr, _) in enumerate(poses):
            ref = one(fr, scenes[i], row0, stride, nb)
            assert torch.equal(out[i * fb:(i + 1) * fb], ref), (row0, i)
        # the band is in these frames: the ring frames differ from plain ones
        plain = geo.GeoScene.from_buffer_copy(bytes(scenes[0]))
        plain.flags &= ~_lib.GEO_FLAG_RING_F64
        uv_r = torch.empty(nb * BR * W * 2, dtype=torch.float32, device=dev)
        uv_p = torch.empty(nb * BR * W * 2, dtype=torch.float32, device=dev)
        tmp = torch.empty(nb * BR * W * 4, dtype=torch.uint8, device=dev)
        ctx.render_band_set(poses[0][0], scenes[0], W, H, BR, row0, stride, nb, tmp, out_uv=uv_r)
        ctx.render_band_set(poses[0][0], plain, W, H, BR, row0, stride, nb, tmp, out_uv=uv_p)
        torch.cuda.synchronize()
        assert int((uv_r != uv_p).sum().item()) > 0
