"""The workgroup dispatch order (geo_set_dispatch, geo_set_tile_order) changes
when tiles run, never what they draw.  An explicit random permutation of the
tile grid, and the learned longest-first order (re-learned every render or
every few, on one stream or alternating between two), render the same frames
byte for byte as row-major order, step counts included (direct, fan and
adaptive mode, ragged frames); a render of another grid ignores an explicit
order; invalid orders and settings are rejected."""
import numpy as np
import pytest
import torch

from helpers import default_frame, default_scene
from schwarzschild_raytracer_wgpu_amd import Context, GeoError, make_scene
from schwarzschild_raytracer_wgpu_amd._lib import (GEO_DISPATCH_LONGEST_FIRST, GEO_DISPATCH_ROW_MAJOR, GEO_MODE_ADAPTIVE,
                                                   GEO_MODE_FAN)
from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

pytestmark = pytest.mark.gpu


def _grid(w, h, fan=False):
    return (w + 31) // 32, (h + (16 if fan else 8) - 1) // (16 if fan else 8)


@pytest.mark.parametrize("mode", ["direct", "fan", "adaptive"])
def test_any_order_same_frame(dev, mode):
    w, h = 200, 117  # ragged in both tile dimensions
    frame = default_frame(w, h)
    base = default_scene(2048)
    scene = base
    if mode == "adaptive":
        scene = make_scene(base.rs, base.sphere_r, base.r_obs, base.step, base.max_steps, GEO_MODE_ADAPTIVE)
    if mode == "fan":
        scene = make_scene(base.rs, base.sphere_r, base.r_obs, base.step, base.max_steps, GEO_MODE_FAN)
    ctx = Context(0)
    ctx.set_sky(make_sky("equirect", (256, 128)))
    if mode == "fan":
        ctx.solve_ray_fan(50.0, 1.0, 2048, base.step, 400, base.r_obs)
    outs = []
    tx, ty = _grid(w, h, mode == "fan")
    rng = np.random.default_rng(11)
    packed = (np.arange(ty)[:, None] << 16 | np.arange(tx)[None, :]).astype(np.uint32).ravel()
    for order in (None, rng.permutation(packed), packed[::-1].copy()):
        ctx.set_tile_order(tx, ty, order)
        rgba = torch.zeros(h * w * 4, dtype=torch.uint8, device=dev)
        steps = torch.zeros(h * w, dtype=torch.int32, device=dev)
        tot = torch.zeros(1, dtype=torch.int64, device=dev)
        ctx.render_rows(frame, scene, w, h, 0, h, rgba, out_steps=steps, steps_total=tot)
        torch.cuda.synchronize()
        outs.append((rgba.cpu(), steps.cpu(), int(tot.item())))
    for o in outs[1:]:
        assert torch.equal(o[0], outs[0][0]) and torch.equal(o[1], outs[0][1]) and o[2] == outs[0][2]
    # a render of another grid (fewer rows) ignores the order: still the same rows
    ctx.set_tile_order(tx, ty, rng.permutation(packed))
    part = torch.zeros(64 * w * 4, dtype=torch.uint8, device=dev)
    ctx.render_rows(frame, scene, w, h, 16, 64, part)
    torch.cuda.synchronize()
    assert torch.equal(part.cpu(), outs[0][0][16 * w * 4:80 * w * 4])
    ctx.close()


def test_invalid_orders_rejected(dev):
    ctx = Context(0)
    tx, ty = 3, 2
    packed = (np.arange(ty)[:, None] << 16 | np.arange(tx)[None, :]).astype(np.uint32).ravel()
    bad_dup = packed.copy()
    bad_dup[1] = bad_dup[0]
    bad_range = packed.copy()
    bad_range[0] = (5 << 16) | 0
    for bad in (bad_dup, bad_range):
        with pytest.raises(GeoError):
            ctx.set_tile_order(tx, ty, bad)
    with pytest.raises(ValueError):
        ctx.set_tile_order(tx, ty, packed[:-1])
    ctx.set_tile_order(tx, ty, packed)
    ctx.set_tile_order(tx, ty, None)
    ctx.close()


@pytest.mark.parametrize("mode", ["direct", "adaptive"])
@pytest.mark.parametrize("period", [1, 3])
def test_learned_order_same_frames(dev, mode, period):
    w, h = 200, 117
    frame = default_frame(w, h)
    base = default_scene(2048)
    scene = base if mode == "direct" else make_scene(base.rs, base.sphere_r, base.r_obs, base.step, base.max_steps,
                                                      GEO_MODE_ADAPTIVE)
    ctx = Context(0)
    ctx.set_sky(make_sky("equirect", (256, 128)))

    def render(stream=None):
        rgba = torch.zeros(h * w * 4, dtype=torch.uint8, device=dev)
        steps = torch.zeros(h * w, dtype=torch.int32, device=dev)
        tot = torch.zeros(1, dtype=torch.int64, device=dev)
        ctx.render_rows(frame, scene, w, h, 0, h, rgba, out_steps=steps, steps_total=tot, stream=stream)
        return rgba, steps, tot

    ctx.set_dispatch(GEO_DISPATCH_ROW_MAJOR)
    ref = render()
    torch.cuda.synchronize()
    ctx.set_dispatch(GEO_DISPATCH_LONGEST_FIRST, period)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = []
    for i in range(8):  # learn, use, re-learn; alternating streams after the first four
        st = None if i < 4 else (s1 if i % 2 else s2)
        with torch.cuda.stream(st or torch.cuda.current_stream()):
            outs.append(render(st))
    # a band render in between (another grid) and back
    band = torch.zeros(64 * w * 4, dtype=torch.uint8, device=dev)
    ctx.render_rows(frame, scene, w, h, 16, 64, band)
    outs.append(render())
    torch.cuda.synchronize()
    for o in outs:
        assert torch.equal(o[0], ref[0]) and torch.equal(o[1], ref[1]) and torch.equal(o[2], ref[2])
    assert torch.equal(band, ref[0][16 * w * 4:80 * w * 4])
    ctx.close()


def test_dispatch_settings_rejected(dev):
    ctx = Context(0)
    for mode, period in [(7, 16), (GEO_DISPATCH_LONGEST_FIRST, 0), (GEO_DISPATCH_LONGEST_FIRST, (1 << 20) + 1)]:
        with pytest.raises(GeoError):
            ctx.set_dispatch(mode, period)
    ctx.set_dispatch(GEO_DISPATCH_LONGEST_FIRST, 1 << 20)
    ctx.close()


def test_time_next_render(dev):
    """geo_time_next_render: the pair times the next render's kernel only; the
    render is unchanged and the context's own ordering event still fires."""
    from schwarzschild_raytracer_wgpu_amd.timing import HipEvent

    w, h = 256, 144
    frame = default_frame(w, h)
    scene = default_scene(2048)
    ctx = Context(0)
    ctx.set_sky(make_sky("equirect", (256, 128)))
    ref = torch.zeros(h * w * 4, dtype=torch.uint8, device=dev)
    ctx.render_rows(frame, scene, w, h, 0, h, ref)
    a, b = HipEvent(), HipEvent()
    out = torch.zeros_like(ref)
    ctx.time_next_render(a, b)
    ctx.render_rows(frame, scene, w, h, 0, h, out)
    ms = a.elapsed_time(b)
    assert torch.equal(out, ref) and 0.0 < ms < 50.0
    ctx.set_sky(make_sky("equirect", (128, 64)))  # waits on the context's event: must not hang
    ctx.close()


@pytest.mark.parametrize("period", [1, 3, 16])
def test_learning_period_counts(dev, period):
    """GEO_DISPATCH_LONGEST_FIRST records every period-th render of a grid
    (renders 1, period + 1, ...) and the next render adopts the order built
    from it; with a sync after each render every rebuild completes in time."""
    w, h = 200, 117
    frame = default_frame(w, h)
    scene = default_scene(256)
    ctx = Context(0)
    ctx.set_sky(make_sky("equirect", (256, 128)))
    ctx.set_dispatch(GEO_DISPATCH_LONGEST_FIRST, period)
    rec0, ad0 = ctx.dispatch_stats()
    n = 2 * period + 2
    out = torch.zeros(h * w * 4, dtype=torch.uint8, device=dev)
    for _ in range(n):
        ctx.render_rows(frame, scene, w, h, 0, h, out)
        torch.cuda.synchronize()
    rec, ad = ctx.dispatch_stats()
    assert rec - rec0 == len([i for i in range(n) if i % period == 0])
    assert ad - ad0 == len([i for i in range(n - 1) if i % period == 0])
    ctx.close()


def test_refused_render_drops_the_timing_pair(dev):
    """geo_time_next_render's pair belongs to the next render call: a call
    refused before launching records neither event, and the render after it
    does not record them either."""
    from schwarzschild_raytracer_wgpu_amd import _lib
    from schwarzschild_raytracer_wgpu_amd.timing import HipEvent

    w, h = 64, 32
    frame = default_frame(w, h)
    scene = default_scene(256)
    ctx = Context(0)
    ctx.set_sky(make_sky("equirect", (128, 64)))
    out = torch.zeros(h * w * 4, dtype=torch.uint8, device=dev)
    a, b = HipEvent(), HipEvent()
    for bad in ("args", "state"):
        ctx.time_next_render(a, b)
        if bad == "args":  # rows past the frame: refused by the entry point
            st = _lib.lib.geo_render_rows(ctx._h, frame, scene, w, h, h - 1, 2, out.data_ptr(), None, None, None,
                                          None, None)
        else:  # fan mode without a fan: refused inside
            fs = make_scene(1.0, 50.0, scene.r_obs, scene.step, 256, GEO_MODE_FAN)
            st = _lib.lib.geo_render_rows(ctx._h, frame, fs, w, h, 0, h, out.data_ptr(), None, None, None, None, None)
        assert st < 0
        ctx.render_rows(frame, scene, w, h, 0, h, out)
        torch.cuda.synchronize()
        with pytest.raises(RuntimeError):
            a.elapsed_time(b)  # never recorded
    ctx.close()
