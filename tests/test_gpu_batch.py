"""geo_render_band_set_frames: a batch of frames of one scene in one launch
(the frame in blockIdx.z, its uniform from the launch's frame batch) draws,
frame by frame, the bytes geo_render_band_set draws for that frame alone,
and counts the same steps ("What a launch costs whatever its
size"; dist.ShardedFrame renders a rank's batch this way)."""
import math

import pytest

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


def _frames(geo, w, h, n, r=(2.5, 0.0, 0.1)):
    """n uniforms of an observer at one radius, camera turning frame by frame."""
    out = []
    for i in range(n):
        obs = geo.Observer(1.0, math.pi / 2, w, h)
        obs.set_position(*r)
        obs.set_camera(math.pi + 0.07 * i, 0.05 * (i % 3) - 0.05)
        out.append(obs.calc_transformation_pipeline())
    return out, obs.get_radial_position()


@pytest.mark.parametrize("mode_name", ["direct", "adaptive", "fan"])
@pytest.mark.parametrize("w,h,band_rows,row0,row_stride", [
    (100, 56, 8, 0, 8),        # contiguous rows, ragged tiles
    (160, 96, 8, 8, 24),       # a peer's interleaved 8-row bands (N = 3)
    (128, 120, 16, 0, 40),     # rank 0's lead bands (lead 2, N = 4)
])
def test_batch_equals_single_frames(geo, torch_mod, mode_name, w, h, band_rows, row0, row_stride):
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    mode = {"direct": geo.GEO_MODE_DIRECT, "adaptive": geo.GEO_MODE_ADAPTIVE, "fan": geo.GEO_MODE_FAN}[mode_name]
    dev = torch_mod.device("cuda:0")
    ctx = geo.Context(0)
    ctx.set_sky(make_sky("equirect", (256, 128)))
    nbands = (h - row0 + row_stride - 1) // row_stride
    packed = nbands * band_rows * w * 4
    for n in (1, 3, geo._lib.GEO_MAX_BATCH_FRAMES):
        frames, r = _frames(geo, w, h, n)
        if mode == geo.GEO_MODE_FAN:
            ctx.solve_ray_fan(50.0, 1.0, 1000, math.pi / 100, 400, r, host=False)
        scene = geo.make_scene(1.0, 50.0, r, math.pi / 100, 2048, mode,
                               tol=1e-6 if mode == geo.GEO_MODE_ADAPTIVE else 0.0)
        stride = packed + 4 * 37  # a gap between frames, left untouched
        out = torch_mod.full((n * stride,), 7, dtype=torch_mod.uint8, device=dev)
        tot = torch_mod.zeros(1, dtype=torch_mod.int64, device=dev)
        ctx.render_band_set_frames(frames, scene, w, h, band_rows, row0, row_stride, nbands, out,
                                   frame_stride=stride, steps_total=tot)
        ref_tot = torch_mod.zeros(1, dtype=torch_mod.int64, device=dev)
        for f in range(n):
            ref = torch_mod.full((packed,), 7, dtype=torch_mod.uint8, device=dev)
            ctx.render_band_set(frames[f], scene, w, h, band_rows, row0, row_stride, nbands, ref,
                                steps_total=ref_tot)
            got = out[f * stride:(f + 1) * stride]
            assert torch_mod.equal(got[:packed], ref), (mode_name, n, f)
            assert bool((got[packed:] == 7).all()), (mode_name, n, f)  # the gap
        torch_mod.cuda.synchronize()
        if mode != geo.GEO_MODE_FAN:
            assert int(tot.item()) == int(ref_tot.item()) > 0
        if n > 1:
            assert len({bytes(out[f * stride:f * stride + packed].cpu().numpy()) for f in range(n)}) == n
    ctx.close()


def test_batch_rejects_what_it_does_not_draw(geo, torch_mod):
    """Colour only: no mip-mapped sampler; frame strides must hold a frame and
    keep 4-byte alignment; 1 .. GEO_MAX_BATCH_FRAMES frames."""
    import ctypes

    from schwarzschild_raytracer_wgpu_amd import _lib
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    dev = torch_mod.device("cuda:0")
    ctx = geo.Context(0)
    ctx.set_sky(make_sky("equirect", (64, 32)))
    frames, r = _frames(geo, 64, 32, 2)
    arr = (geo.GeoFrame * 2)(*frames)
    out = torch_mod.empty(2 * 64 * 32 * 4 + 64, dtype=torch_mod.uint8, device=dev)
    fb = 64 * 32 * 4

    def call(scene, stride, n=2):
        return _lib.lib.geo_render_band_set_frames(ctx._h, arr, n, ctypes.byref(scene), 64, 32, 8, 0, 8, 4,
                                                   out.data_ptr(), stride, None,
                                                   torch_mod.cuda.current_stream().cuda_stream)

    plain = geo.make_scene(1.0, 50.0, r, math.pi / 100, 64, geo.GEO_MODE_DIRECT)
    mips = geo.make_scene(1.0, 50.0, r, math.pi / 100, 64, geo.GEO_MODE_DIRECT, flags=_lib.GEO_FLAG_MIPS)
    assert call(plain, fb) == _lib.GEO_OK
    assert call(plain, fb, n=1) == _lib.GEO_OK
    assert call(mips, fb) == _lib.GEO_EINVAL
    assert call(mips, fb, n=1) == _lib.GEO_OK  # one frame: the single-frame kernel, any sampler
    assert call(plain, fb - 4) == _lib.GEO_EINVAL
    assert call(plain, fb + 2) == _lib.GEO_EINVAL
    torch_mod.cuda.synchronize()
    ctx.close()


def _moving(geo, w, h, n, kind):
    """n uniforms and scenes of a moving observer (the reference's present
    loop: Observer::update_position then calc_transformation_pipeline per
    frame, observer.rs:105-125, renderer.rs:208-264): 'orbit' =
    start_orbit(1.8) from (2.5, 0, 0.1), 'fall' = start_orbit(0) (the Fall
    button, lib.rs:180), dt = 1/20 s per frame (large steps: the radius moves
    visibly within a batch)."""
    obs = geo.Observer(1.0, math.pi / 2, w, h)
    obs.set_position(2.5, 0.0, 0.1)
    assert obs.start_orbit(1.8 if kind == "orbit" else 0.0)
    frames, scenes = [], []
    for _ in range(n):
        obs.update_position((0.0, 0.0, 0.0), 0.05)
        frames.append(obs.calc_transformation_pipeline())
        scenes.append(geo.make_scene(1.0, 50.0, obs.get_radial_position(), math.pi / 100, 1024, geo.GEO_MODE_DIRECT))
    return frames, scenes


@pytest.mark.parametrize("kind", ["orbit", "fall"])
@pytest.mark.parametrize("mode_name", ["direct", "adaptive"])
def test_batch_of_a_moving_observer(geo, torch_mod, kind, mode_name):
    """geo_render_band_set_batch: frames whose scenes differ in r_obs (each
    frame's own radius) in one launch == each frame rendered alone with its
    own scene, bytes and step totals."""
    from schwarzschild_raytracer_wgpu_amd import _lib
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    w, h, band_rows, row0, row_stride = 160, 96, 8, 8, 24
    dev = torch_mod.device("cuda:0")
    ctx = geo.Context(0)
    ctx.set_sky(make_sky("equirect", (256, 128)))
    n = _lib.GEO_MAX_BATCH_FRAMES
    frames, scenes = _moving(geo, w, h, n, kind)
    if mode_name == "adaptive":
        scenes = [geo.make_scene(s.rs, s.sphere_r, s.r_obs, s.step, s.max_steps, geo.GEO_MODE_ADAPTIVE)
                  for s in scenes]
    assert len({s.r_obs for s in scenes}) == n  # every frame its own radius
    nbands = (h - row0 + row_stride - 1) // row_stride
    packed = nbands * band_rows * w * 4
    out = torch_mod.full((n * packed,), 7, dtype=torch_mod.uint8, device=dev)
    tot = torch_mod.zeros(1, dtype=torch_mod.int64, device=dev)
    fa, sa = (geo.GeoFrame * n)(*frames), (geo.GeoScene * n)(*scenes)
    _lib.check("geo_render_band_set_batch", _lib.lib.geo_render_band_set_batch(
        ctx._h, fa, sa, n, w, h, band_rows, row0, row_stride, nbands, out.data_ptr(), packed, tot.data_ptr(),
        torch_mod.cuda.current_stream().cuda_stream))
    ref_tot = torch_mod.zeros(1, dtype=torch_mod.int64, device=dev)
    for f in range(n):
        ref = torch_mod.full((packed,), 7, dtype=torch_mod.uint8, device=dev)
        ctx.render_band_set(frames[f], scenes[f], w, h, band_rows, row0, row_stride, nbands, ref, steps_total=ref_tot)
        assert torch_mod.equal(out[f * packed:(f + 1) * packed], ref), (kind, f)
    torch_mod.cuda.synchronize()
    assert int(tot.item()) == int(ref_tot.item()) > 0
    ctx.close()


def test_batch_scenes_must_agree_but_for_the_radius(geo, torch_mod):
    import ctypes

    from schwarzschild_raytracer_wgpu_amd import _lib
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    dev = torch_mod.device("cuda:0")
    ctx = geo.Context(0)
    ctx.set_sky(make_sky("equirect", (64, 32)))
    frames, r = _frames(geo, 64, 32, 2)
    fa = (geo.GeoFrame * 2)(*frames)
    out = torch_mod.empty(2 * 64 * 32 * 4, dtype=torch_mod.uint8, device=dev)

    def call(s0, s1):
        sa = (geo.GeoScene * 2)(s0, s1)
        return _lib.lib.geo_render_band_set_batch(ctx._h, fa, sa, 2, 64, 32, 8, 0, 8, 4, out.data_ptr(),
                                                  64 * 32 * 4, None, torch_mod.cuda.current_stream().cuda_stream)

    def sc(r_obs=r, budget=64, mode=geo.GEO_MODE_DIRECT, step=math.pi / 100):
        return geo.make_scene(1.0, 50.0, r_obs, step, budget, mode)

    assert call(sc(), sc(r * 1.01)) == _lib.GEO_OK
    assert call(sc(), sc(budget=65)) == _lib.GEO_EINVAL             # another budget
    assert call(sc(), sc(step=math.pi / 99)) == _lib.GEO_EINVAL     # another step
    assert call(sc(), sc(mode=geo.GEO_MODE_ADAPTIVE)) == _lib.GEO_EINVAL
    assert call(sc(), sc(r_obs=0.9)) == _lib.GEO_EINVAL             # inside the horizon: another kind
    assert call(sc(), sc(r_obs=-1.0)) == _lib.GEO_EINVAL
    assert call(sc(r_obs=0.8), sc(r_obs=0.9)) == _lib.GEO_OK        # both inside
    ctx.solve_ray_fan(50.0, 1.0, 1000, math.pi / 100, 400, r, host=False)
    assert call(sc(mode=geo.GEO_MODE_FAN), sc(mode=geo.GEO_MODE_FAN)) == _lib.GEO_OK
    assert call(sc(mode=geo.GEO_MODE_FAN), sc(r * 1.01, mode=geo.GEO_MODE_FAN)) == _lib.GEO_EINVAL  # one fan
    torch_mod.cuda.synchronize()
    ctx.close()
