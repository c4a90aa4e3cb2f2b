"""HIP kernel parity (through the C-ABI) against the CPU oracle.

Bar (BASELINE.json north_star): hit-classification mask identical pixel for
pixel, sky UV within 1e-4 relative.  The kernel and the oracle's f32 mirror
evaluate the same fixed operation sequence, so we require MORE: mask, UV,
steps and RGBA bit-identical.  UV_TOL is the stated tolerance, checked too.
"""
import ctypes
import math
import os

import numpy as np
import pytest

import f64_bar as B
import oracle as O
from helpers import R_OBS, default_frame, default_scene, wrap_du

pytestmark = pytest.mark.gpu

UV_TOL = 1e-4  # relative, north_star
GOLD = os.path.join(os.path.dirname(__file__), "golden")


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


def render(g, torch, ctx, frame, scene, w, h, row0=0, nrows=None):
    nrows = h - row0 if nrows is None else nrows
    dev = torch.device("cuda:0")
    rgba = torch.empty(nrows * w * 4, dtype=torch.uint8, device=dev)
    mask = torch.empty(nrows * w, dtype=torch.uint8, device=dev)
    uv = torch.empty(nrows * w * 2, dtype=torch.float32, device=dev)
    steps = torch.empty(nrows * w, dtype=torch.int32, device=dev)
    total = torch.zeros(1, dtype=torch.int64, device=dev)
    ctx.render_rows(frame, scene, w, h, row0, nrows, rgba, mask, uv, steps, total)
    torch.cuda.synchronize()
    return dict(rgba=rgba.cpu().numpy().reshape(nrows, w, 4), mask=mask.cpu().numpy().reshape(nrows, w),
                uv=uv.cpu().numpy().reshape(nrows, w, 2),
                steps=steps.cpu().numpy().view(np.uint32).reshape(nrows, w), total=int(total.item()))


def assert_same(hip, ref, fields=("mask", "uv", "steps", "rgba")):
    for f in fields:
        a, b = hip[f], ref[f]
        if f == "uv":
            assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), (
                f"uv differs at {np.argwhere(a.view(np.uint32) != b.view(np.uint32))[:5]}")
        else:
            bad = np.argwhere(a != b)
            assert bad.size == 0, f"{f} differs at {len(bad)} places, first {bad[:5]}"
    # the stated tolerance, for the record
    d = wrap_du(hip["uv"], ref["uv"])
    assert float(d.max()) <= UV_TOL


def make_ctx(g, sky):
    ctx = g.Context(0)
    ctx.set_sky(sky)
    return ctx


def test_golden_fixture_bitexact(geo, torch_mod):
    z = np.load(os.path.join(GOLD, "pixels_64x36.npz"))
    frame = geo.GeoFrame.from_buffer_copy(z["frame"].tobytes())
    ctx = make_ctx(geo, z["sky"])
    hip = render(geo, torch_mod, ctx, frame, default_scene(2048), 64, 36)
    assert_same(hip, dict(rgba=z["f32_rgba"], mask=z["f32_mask"], uv=z["f32_uv"], steps=z["f32_steps"]))
    assert hip["total"] == int(z["f32_steps"].sum())
    # against the f64 literal restatement: north_star's bar on every pixel of
    # this frame (mask identical; UV within 1e-4 of the [0, 1] range, U
    # wrap-aware; tests/f64_bar.py), no band exclusion needed here
    assert np.array_equal(hip["mask"], z["f64_mask"])
    nb = (z["f64_mask"] == 0) & (hip["mask"] == 0)
    assert B.uv_err(hip["uv"], z["f64_uv"])[nb].max() <= B.UV_BAR


SCENES = [
    # name, w, h, frame kwargs, scene kwargs, sky
    ("cfg1_256_flat", 256, 256, {}, dict(max_steps=128), "flat"),
    ("odd_333x187", 333, 187, {}, dict(max_steps=512), "equirect"),
    ("unmoving", 160, 90, dict(state=0), dict(max_steps=512), "equirect"),
    ("offaxis_inside_photon_sphere", 192, 108, dict(pos=(1.3 * math.cos(0.2), 1.3 * math.sin(0.2), 0.05),
                                                      camera=(math.pi + 0.6, 0.3)),
     dict(max_steps=2048, r_obs=math.sqrt(1.3 ** 2 + 0.05 ** 2)), "equirect"),
    ("inside_horizon", 128, 128, dict(pos=(0.8, 0.0, 0.05)), dict(max_steps=512, r_obs=math.sqrt(0.64 + 0.0025)),
     "equirect"),
    ("flat_space", 128, 72, dict(rs=0.0, state=0), dict(rs=0.0, max_steps=512), "equirect"),
    ("far_ref_scale", 200, 120, dict(pos=(25.0, 0.0, 1.0), rs=10.0),
     dict(rs=10.0, sphere_r=500.0, r_obs=math.sqrt(626.0), max_steps=1000), "equirect"),
    ("single_row", 97, 1, {}, dict(max_steps=512), "equirect"),
    ("single_col", 1, 77, {}, dict(max_steps=512), "equirect"),
    ("translucent_sky", 120, 68, {}, dict(max_steps=512), "random_alpha"),
    # both sides of the one-test-per-group loop's limit (sphere beyond / inside the photon sphere)
    ("sphere_just_beyond_photon_sphere", 160, 90, dict(pos=(1.2, 0.3, 0.05), camera=(math.pi + 0.4, 0.2)),
     dict(sphere_r=1.51, r_obs=math.sqrt(1.44 + 0.09 + 0.0025)), "equirect"),
    ("sphere_inside_photon_sphere", 160, 90, dict(pos=(1.2, 0.0, 0.05), camera=(math.pi + 1.0, 0.0)),
     dict(sphere_r=1.4, r_obs=math.sqrt(1.44 + 0.0025)), "equirect"),
]


@pytest.mark.parametrize("name,w,h,fk,sk,skykind", SCENES, ids=[s[0] for s in SCENES])
def test_direct_mode_matches_oracle_bitexact(geo, torch_mod, name, w, h, fk, sk, skykind):
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    if skykind == "random_alpha":
        sky = np.random.default_rng(3).integers(0, 256, size=(128, 256, 4), dtype=np.uint8)
    else:
        sky = make_sky(skykind, (1, 1) if skykind == "flat" else (512, 256))
    frame = default_frame(w, h, **fk)
    scene = default_scene(**sk)
    ctx = make_ctx(geo, sky)
    hip = render(geo, torch_mod, ctx, frame, scene, w, h)
    ref = O.render_f32(frame, scene, sky, w, h, threads=8)
    assert_same(hip, ref)
    assert hip["total"] == int(ref["steps"].sum()) == ref["steps_total"]


def test_row_blocks_compose_full_frame(geo, torch_mod):
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    w, h = 320, 181
    sky = make_sky("equirect", (256, 128))
    frame, scene = default_frame(w, h), default_scene(2048)
    ctx = make_ctx(geo, sky)
    full = render(geo, torch_mod, ctx, frame, scene, w, h)
    parts = [render(geo, torch_mod, ctx, frame, scene, w, h, r0, n) for r0, n in ((0, 50), (50, 1), (51, 100),
                                                                                   (151, 30))]
    for f in ("rgba", "mask", "uv", "steps"):
        assert np.array_equal(np.concatenate([p[f] for p in parts]), full[f])
    assert sum(p["total"] for p in parts) == full["total"]


def test_tallest_frame_takes_several_launches(geo, torch_mod):
    """A narrow frame of the C-ABI's maximum height, 2^20 rows: 131072 tile
    rows, more than grid.y's 65535, so the render goes out as three launches
    (ADVICE r02).  Sampled rows from every launch equal the oracle, a row
    block across a launch boundary equals its own render, and the step total
    covers every launch."""
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    w, h = 4, 1 << 20
    sky = make_sky("equirect", (256, 128))
    frame, scene = default_frame(w, h), default_scene(64)
    ctx = make_ctx(geo, sky)
    full = render(geo, torch_mod, ctx, frame, scene, w, h)
    assert full["total"] == int(full["steps"].astype(np.int64).sum()) > 0
    row0, step = 3, 4099
    ref = O.render_f32(frame, scene, sky, w, h, row0=row0, nrows=(h - row0 + step - 1) // step, row_step=step,
                       threads=8)
    for f in ("rgba", "mask", "uv", "steps"):
        a = full[f][row0::step]
        assert np.array_equal(a.view(np.uint32) if f == "uv" else a, ref[f].view(np.uint32) if f == "uv" else ref[f]), f
    b0 = 65535 * 8 - 20  # the first launch's last tile rows and the second's first
    part = render(geo, torch_mod, ctx, frame, scene, w, h, b0, 40)
    for f in ("rgba", "mask", "uv", "steps"):
        assert np.array_equal(part[f], full[f][b0:b0 + 40]), f
    last = render(geo, torch_mod, ctx, frame, scene, w, h, h - 9, 9)
    assert np.array_equal(last["rgba"], full["rgba"][h - 9:])


def test_sky_swap_waits_for_renders_on_other_streams(geo, torch_mod):
    """geo_set_sky waits for the context's renders in flight on every stream
    it has rendered on (per-stream events, no device-wide wait),
    including streams evicted from the context's 8 tracked slots: renders
    queued before the swap sample the old sky, renders after it the new one."""
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    torch = torch_mod
    w, h = 1920, 1080
    frame, scene = default_frame(w, h), default_scene(2048)
    sky_a = make_sky("equirect", (512, 256))
    sky_b = np.ascontiguousarray(255 - sky_a)
    sky_b[..., 3] = 255
    want = {}
    for name, sky in (("a", sky_a), ("b", sky_b)):
        ref_ctx = make_ctx(geo, sky)
        want[name] = render(geo, torch, ref_ctx, frame, scene, w, h)["rgba"]
        ref_ctx.close()
    assert not np.array_equal(want["a"], want["b"])
    dev = torch.device("cuda:0")
    ctx = make_ctx(geo, sky_a)
    streams = [torch.cuda.Stream() for _ in range(11)]  # > 8 tracked slots
    before = [torch.empty(h * w * 4, dtype=torch.uint8, device=dev) for _ in streams]
    for st, buf in zip(streams, before):
        ctx.render_rows(frame, scene, w, h, 0, h, buf, stream=st)
    ctx.set_sky(sky_b)  # same size: overwritten in place
    after = torch.empty(h * w * 4, dtype=torch.uint8, device=dev)
    ctx.render_rows(frame, scene, w, h, 0, h, after, stream=streams[0])
    torch.cuda.synchronize()
    for buf in before:
        assert np.array_equal(buf.cpu().numpy().reshape(h, w, 4), want["a"])
    assert np.array_equal(after.cpu().numpy().reshape(h, w, 4), want["b"])


def test_render_bands_interleaved(geo, torch_mod):
    """geo_render_bands for 3 ranks x 8-row bands == the full frame's rows."""
    from schwarzschild_raytracer_wgpu_amd.dist import BandLayout
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    w, h, B, world = 120, 101, 8, 3
    sky = make_sky("equirect", (256, 128))
    frame, scene = default_frame(w, h), default_scene(2048)
    ctx = make_ctx(geo, sky)
    full = render(geo, torch_mod, ctx, frame, scene, w, h)
    dev = torch_mod.device("cuda:0")
    tot = 0
    for r in range(world):
        L = BandLayout(h, B, world, r)
        n = L.nb_mine * B * w
        rgba = torch_mod.zeros(n * 4, dtype=torch_mod.uint8, device=dev)
        steps = torch_mod.zeros(n, dtype=torch_mod.int32, device=dev)
        ctr = torch_mod.zeros(1, dtype=torch_mod.int64, device=dev)
        ctx.render_bands(frame, scene, w, h, B, r, world, L.nb_mine, rgba, out_steps=steps, steps_total=ctr)
        torch_mod.cuda.synchronize()
        rgba = rgba.cpu().numpy().reshape(-1, w, 4)
        steps = steps.cpu().numpy().view(np.uint32).reshape(-1, w)
        for i, fr in enumerate(L.local_to_frame_rows()):
            if fr >= 0:
                assert np.array_equal(rgba[i], full["rgba"][fr]) and np.array_equal(steps[i], full["steps"][fr])
        tot += int(ctr.item())
    assert tot == full["total"]
    with pytest.raises(geo.GeoError):  # band_rows must be a multiple of 8
        ctx.render_bands(frame, scene, w, h, 12, 0, 1, 2, torch_mod.zeros(24 * w * 4, dtype=torch_mod.uint8,
                                                                         device=dev))


def test_step_totals_per_call_across_streams(geo, torch_mod):
    """Each render's steps_total gets exactly its own rows' steps, also when
    renders with their own totals overlap on different streams (more calls in
    flight than the context has per-call counter sets), and a DEFER
    accumulation on a third stream is not disturbed by them."""
    from schwarzschild_raytracer_wgpu_amd import _lib
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    torch = torch_mod
    w, h = 256, 192
    frame, scene = default_frame(w, h), default_scene(2048)
    ctx = make_ctx(geo, make_sky("equirect", (256, 128)))
    full = render(geo, torch, ctx, frame, scene, w, h)
    dev = torch.device("cuda:0")
    want = [int(full["steps"][r0:r0 + 16].astype(np.int64).sum()) for r0 in range(0, h, 16)]
    streams = [torch.cuda.Stream(dev) for _ in range(3)]
    defer = geo.make_scene(scene.rs, scene.sphere_r, scene.r_obs, scene.step, scene.max_steps,
                           flags=_lib.GEO_FLAG_DEFER_STEPS)
    for _ in range(3):
        totals = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in want]
        outs = [torch.empty(16 * w * 4, dtype=torch.uint8, device=dev) for _ in want]
        dout = torch.empty(h * w * 4, dtype=torch.uint8, device=dev)
        acc = torch.zeros(1, dtype=torch.int64, device=dev)
        torch.cuda.synchronize()  # the zero fills ran on the current stream
        ctx.render_rows(frame, defer, w, h, 0, h, dout, stream=streams[2])
        for i, r0 in enumerate(range(0, h, 16)):
            ctx.render_rows(frame, scene, w, h, r0, 16, outs[i], steps_total=totals[i], stream=streams[i % 2])
        ctx.steps_flush(acc, stream=streams[2])
        torch.cuda.synchronize()
        assert [int(t.item()) for t in totals] == want
        assert int(acc.item()) == full["total"]


def test_fan_kernel_matches_oracle(geo, torch_mod):
    ctx = geo.Context(0)
    for args in [(500.0, 10.0, 1000, math.pi / 100, 400, math.sqrt(626.0)),
                 (100.0, 10.0, 100, math.pi / 100, 20, 25.0),
                 (50.0, 1.0, 1000, math.pi / 100, 400, R_OBS),
                 (50.0, 1.0, 1000, math.pi / 100, 400, 0.7),  # inside the horizon
                 (50.0, 0.0, 1000, math.pi / 100, 64, 3.0)]:  # flat space
        gpu = ctx.solve_ray_fan(*args)
        ref = O.solve_ray_fan(*args)
        # f64 on both sides; device cos/sin may differ from glibc by an f64 ulp,
        # which survives the f32 rounding at most as one f32 ulp.
        d = np.abs(gpu.astype(np.float64) - ref)
        assert np.all(d <= np.spacing(np.abs(ref)).astype(np.float64)), (args, d.max())
        assert np.mean(gpu == ref) > 0.99


@pytest.mark.parametrize("max_iter", [0, 1, 2, 3, 5, 7, 37, 250, 1001, 1003])
def test_fan_kernel_budget_edges(geo, torch_mod, max_iter):
    """The fan kernel takes its steps in groups of 4 with a per-step tail for
    the budget's remainder: budgets on and off the group size end each node
    where the literal loop does (NO_VALUE on exhaustion, a crossing on the
    last allowed step still counts)."""
    ctx = geo.Context(0)
    for sphere_r, rs, r in [(50.0, 1.0, R_OBS), (500.0, 10.0, 25.0), (50.0, 0.0, 3.0)]:
        args = (sphere_r, rs, max_iter, math.pi / 100, 400, r)
        gpu = ctx.solve_ray_fan(*args)
        ref = O.solve_ray_fan(*args)
        d = np.abs(gpu.astype(np.float64) - ref)
        assert np.all(d <= np.spacing(np.abs(ref)).astype(np.float64)), (args, d.max())
        assert np.mean(gpu == ref) > 0.99, args


def test_fan_solved_on_side_stream_matches_one_stream(geo, torch_mod):
    """The context double-buffers its fan and orders it with events: a loop
    whose per-frame fans are solved on a side stream (with no waits of its
    own; each solve overlaps the previous frame's draw) draws the same frames
    as the loop on one stream, and a frame equals the oracle's render with
    that frame's fan."""
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    w, h = 320, 180
    dev = torch_mod.device("cuda:0")
    sky = make_sky("equirect", (512, 256))

    def loop(side):
        obs = geo.Observer(1.0, math.pi / 2, w, h)
        obs.set_position(2.5, 0.0, 0.1)
        sphere = geo.BasicSphereBuffer(0, 50.0, 1.0, sky, mode=geo.GEO_MODE_FAN)
        tgt = geo.RenderTarget(w, h, torch_mod.empty(w * h * 4, dtype=torch_mod.uint8, device=dev))
        frames, radii = [], []
        for i in range(12):
            obs.set_position(2.5 + 0.25 * i, 0.0, 0.1)  # a new radius per frame: every fan differs
            r = obs.get_radial_position()
            sphere.update_ray_fan(r, stream=side)
            sphere.draw(obs.calc_transformation_pipeline(), tgt)
            frames.append(tgt.rgba.clone())
            radii.append(r)
        torch_mod.cuda.synchronize()
        return [f.cpu().numpy() for f in frames], radii, obs

    one, radii, _ = loop(None)
    two, radii2, obs = loop(torch_mod.cuda.Stream(dev))
    assert radii == radii2
    for a, b in zip(one, two):
        assert np.array_equal(a, b)
    assert len({a.tobytes() for a in one}) == len(one)  # the frames differ: each one needs its own fan
    # the last frame against the oracle with that frame's fan
    fan = O.solve_ray_fan(50.0, 1.0, 1000, math.pi / 100, 400, radii[-1])
    scene = geo.make_scene(1.0, 50.0, radii[-1], math.pi / 100, 1000, geo.GEO_MODE_FAN)
    ref = O.render_f32(obs.calc_transformation_pipeline(), scene, sky, w, h, fan=fan, threads=8)
    got = two[-1].reshape(h, w, 4)
    assert np.mean(np.all(got == ref["rgba"], axis=-1)) > 0.999  # GPU fan within 1 f32 ulp of the oracle's


def test_fan_stream_switches_match_one_stream(geo, torch_mod):
    """The fan buffers' readers on the solve's own stream are tracked by
    render slot (no per-draw event), readers on other streams by a chained
    event: solves and draws that switch streams from frame to frame, with a
    synchronous host upload (geo_set_fan) among them, draw the frames of the
    same sequence run on one stream with a sync after every frame.  1080p
    draws, so a solve issued early into a buffer still being read would
    change the frame."""
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    w, h = 1920, 1080
    dev = torch_mod.device("cuda:0")
    sky = make_sky("equirect", (512, 256))
    radii = [2.5 + 0.2 * i for i in range(14)]
    # (solve stream, draw stream) per frame; "set": the fan uploaded from the host
    plan = [("A", "A"), ("A", "A"), ("B", "A"), ("B", "A"), ("B", "B"), ("A", "B"), ("A", "A"), ("C", "B"),
            ("set", "A"), ("B", "C"), ("A", "C"), ("A", "A"), ("set", "B"), ("C", "A")]
    host_fans = {i: O.solve_ray_fan(50.0, 1.0, 1000, math.pi / 100, 400, radii[i])
                 for i, (s, _) in enumerate(plan) if s == "set"}

    def run(streams, sync_each):
        ctx = geo.Context(0)
        ctx.set_sky(sky)
        tgts = [torch_mod.empty(w * h * 4, dtype=torch_mod.uint8, device=dev) for _ in plan]
        obs = geo.Observer(1.0, math.pi / 2, w, h)
        torch_mod.cuda.synchronize()
        for i, (s, d) in enumerate(plan):
            obs.set_position(radii[i], 0.0, 0.1)
            r = obs.get_radial_position()
            if s == "set":
                ctx.set_fan(host_fans[i])
            else:
                ctx.solve_ray_fan(50.0, 1.0, 1000, math.pi / 100, 400, r, stream=streams[s], host=False)
            scene = geo.make_scene(1.0, 50.0, r, math.pi / 100, 1000, geo.GEO_MODE_FAN)
            ctx.render_rows(obs.calc_transformation_pipeline(), scene, w, h, 0, h, tgts[i], stream=streams[d])
            if sync_each:
                torch_mod.cuda.synchronize()
        torch_mod.cuda.synchronize()
        out = [t.cpu().numpy() for t in tgts]
        ctx.close()
        return out

    cur = torch_mod.cuda.current_stream(dev)
    ref = run({"A": cur, "B": cur, "C": cur}, True)
    got = run({"A": cur, "B": torch_mod.cuda.Stream(dev), "C": torch_mod.cuda.Stream(dev)}, False)
    assert len({f.tobytes() for f in ref}) == len(ref)  # every frame needs its own fan
    for i, (a, b) in enumerate(zip(ref, got)):
        assert np.array_equal(a, b), (i, plan[i])


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_stream_plans_match_one_stream(geo, torch_mod, seed):
    """Seeded random plans over ten streams (more than the context's eight
    render slots, so slots are evicted mid-plan): fan solves, host fan
    uploads, fan-mode draws (some of them two or three per fan), and
    direct-mode draws with per-call step counts (the learned tile order is
    rebuilt across streams), each on a random stream with no host sync;
    every output equals the same plan run on one stream with a sync after
    every call."""
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    rng = np.random.default_rng(seed)
    w, h = 1920, 1080
    dw, dh = 480, 272
    dev = torch_mod.device("cuda:0")
    sky = make_sky("equirect", (512, 256))
    plan = []  # (op, stream index, radius)
    for _ in range(36):
        u = rng.random()
        op = "solve" if u < 0.3 else "set" if u < 0.38 else "draw" if u < 0.8 else "direct"
        plan.append((op, int(rng.integers(0, 10)), float(2.3 + 1.5 * rng.random())))
    plan.insert(0, ("solve", 0, 2.5))
    host_fans = {i: O.solve_ray_fan(50.0, 1.0, 1000, math.pi / 100, 400, r) for i, (op, _, r) in enumerate(plan)
                 if op == "set"}

    def run(streams, sync_each):
        ctx = geo.Context(0)
        ctx.set_sky(sky)
        obs = geo.Observer(1.0, math.pi / 2, w, h)
        dobs = geo.Observer(1.0, math.pi / 2, dw, dh)
        outs = []
        torch_mod.cuda.synchronize()
        fan_r = None
        for i, (op, k, r) in enumerate(plan):
            s = streams[k]
            if op == "solve":
                obs.set_position(r, 0.0, 0.1)
                fan_r = obs.get_radial_position()
                ctx.solve_ray_fan(50.0, 1.0, 1000, math.pi / 100, 400, fan_r, stream=s, host=False)
            elif op == "set":
                ctx.set_fan(host_fans[i])
                obs.set_position(r, 0.0, 0.1)
                fan_r = obs.get_radial_position()
            elif op == "draw":
                obs.set_position(fan_r * 0.999, 0.0, 0.1)  # the pose moves, the fan stays
                scene = geo.make_scene(1.0, 50.0, fan_r, math.pi / 100, 1000, geo.GEO_MODE_FAN)
                t = torch_mod.empty(w * h * 4, dtype=torch_mod.uint8, device=dev)
                ctx.render_rows(obs.calc_transformation_pipeline(), scene, w, h, 0, h, t, stream=s)
                outs.append(t)
            else:
                dobs.set_position(r, 0.0, 0.1)
                scene = geo.make_scene(1.0, 50.0, dobs.get_radial_position(), math.pi / 100, 512,
                                       geo.GEO_MODE_DIRECT)
                t = torch_mod.empty(dw * dh * 4, dtype=torch_mod.uint8, device=dev)
                st = torch_mod.zeros(1, dtype=torch_mod.int64, device=dev)
                s.wait_stream(torch_mod.cuda.current_stream(dev))  # the zero fill ran on the current stream
                ctx.render_rows(dobs.calc_transformation_pipeline(), scene, dw, dh, 0, dh, t, stream=s,
                                steps_total=st)
                outs += [t, st]
            if sync_each:
                torch_mod.cuda.synchronize()
        torch_mod.cuda.synchronize()
        res = [t.cpu().numpy() for t in outs]
        ctx.close()
        return res

    cur = torch_mod.cuda.current_stream(dev)
    ref = run([cur] * 10, True)
    got = run([cur] + [torch_mod.cuda.Stream(dev) for _ in range(9)], False)
    assert len(ref) == len(got)
    for i, (a, b) in enumerate(zip(ref, got)):
        assert np.array_equal(a, b), i


def test_fan_plain_draw_bitexact(geo, torch_mod):
    """The fan-mode draw with no output but the colour (a lane draws two
    pixels, 8 rows apart, loads of both in flight): bit for bit the oracle's
    f32 mirror with the same (host) fan, on ragged frames (partial 32 x 16
    tiles), row blocks from any row, 8-row bands, an opaque and a
    translucent sky; and equal to the same draw with every output requested
    (the per-pixel epilogue)."""
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    dev = torch_mod.device("cuda:0")
    fan = O.solve_ray_fan(50.0, 1.0, 1000, math.pi / 100, 400, R_OBS)
    scene = geo.make_scene(1.0, 50.0, R_OBS, math.pi / 100, 1000, geo.GEO_MODE_FAN)
    skies = (make_sky("equirect", (256, 128)),
             np.random.default_rng(21).integers(0, 256, size=(64, 128, 4), dtype=np.uint8))
    for sky in skies:
        ctx = geo.Context(0)
        ctx.set_sky(sky)
        ctx.set_fan(fan)
        for (w, h) in ((100, 57), (64, 36), (33, 17)):
            frame = default_frame(w, h)
            ref = O.render_f32(frame, scene, sky, w, h, fan=fan, threads=8)
            for row0, nrows in ((0, h), (3, h - 3), (h - 5, 5)):
                rgba = torch_mod.empty(nrows * w * 4, dtype=torch_mod.uint8, device=dev)
                ctx.render_rows(frame, scene, w, h, row0, nrows, rgba)
                torch_mod.cuda.synchronize()
                got = rgba.cpu().numpy().reshape(nrows, w, 4)
                assert np.array_equal(got, ref["rgba"][row0:row0 + nrows]), (w, h, row0)
            full = render(geo, torch_mod, ctx, frame, scene, w, h)  # every output: the per-pixel path
            assert_same(full, ref, fields=("mask", "uv", "rgba"))
            # 8-row bands 1, 3, 5, ... packed
            nb = (h // 8 - 1) // 2 + 1 if h >= 16 else 1
            band0 = 1 if h >= 16 else 0
            rgba = torch_mod.empty(nb * 8 * w * 4, dtype=torch_mod.uint8, device=dev)
            ctx.render_bands(frame, scene, w, h, 8, band0, 2, nb, rgba)
            torch_mod.cuda.synchronize()
            got = rgba.cpu().numpy().reshape(nb * 8, w, 4)
            for j in range(nb):
                r0 = (band0 + 2 * j) * 8
                n = max(0, min(8, h - r0))
                assert np.array_equal(got[8 * j:8 * j + n], ref["rgba"][r0:r0 + n]), (w, h, j)
        ctx.close()


def test_sphere_buffer_fan_mode_matches_oracle(geo, torch_mod):
    """Reference-exact mode: BasicSphereBuffer.update_ray_fan + draw = fan lerp
    (shader.wgsl:77-84) with the GPU-solved fan."""
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    w, h = 256, 144
    sky = make_sky("equirect", (512, 256))
    ctx = geo.Context(0)
    buf = geo.BasicSphereBuffer(ctx, 50.0, 1.0, sky, mode=geo.GEO_MODE_FAN)
    buf.update_ray_fan(R_OBS)  # stream-ordered, device only
    fan = buf.ray_tracer.solve_ray_fan(R_OBS).copy()  # the same fan, copied to the host for the oracle
    frame = default_frame(w, h)
    dev = torch_mod.device("cuda:0")
    tgt = geo.RenderTarget(w, h, torch_mod.empty(w * h * 4, dtype=torch_mod.uint8, device=dev),
                           torch_mod.empty(w * h, dtype=torch_mod.uint8, device=dev),
                           torch_mod.empty(w * h * 2, dtype=torch_mod.float32, device=dev))
    buf.draw(frame, tgt)
    torch_mod.cuda.synchronize()
    ref = O.render_f32(frame, buf.scene(), sky, w, h, fan=fan, threads=8)
    hip = dict(rgba=tgt.rgba.cpu().numpy().reshape(h, w, 4), mask=tgt.mask.cpu().numpy().reshape(h, w),
               uv=tgt.uv.cpu().numpy().reshape(h, w, 2))
    assert_same(hip, ref, fields=("mask", "uv", "rgba"))
    # fan mode vs f64 literal shader with the same fan: UV tolerance, mask equal off the lerp edge
    r64 = O.render_f64(frame, buf.scene(), w, h, fan=fan)
    agree = np.mean(hip["mask"] == r64["mask"])
    assert agree > 0.999


def test_1080p_rows_bitexact(geo, torch_mod):
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    w, h = 1920, 1080
    sky = make_sky("equirect", (4096, 2048))
    frame, scene = default_frame(w, h), default_scene(512)
    ctx = make_ctx(geo, sky)
    hip = render(geo, torch_mod, ctx, frame, scene, w, h)
    step = 9
    ref = O.render_f32(frame, scene, sky, w, h, row0=4, nrows=h // step, row_step=step, threads=16)
    sub = {k: hip[k][4::step][: h // step] for k in ("rgba", "mask", "uv", "steps")}
    assert_same(sub, ref)


def test_4k_2048_properties(geo, torch_mod):
    """Full config-3 frame: size-independent properties + sampled bit-exact rows."""
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    w, h = 3840, 2160
    sky = make_sky("equirect", (4096, 2048))
    frame, scene = default_frame(w, h), default_scene(2048)
    ctx = make_ctx(geo, sky)
    a = render(geo, torch_mod, ctx, frame, scene, w, h)
    b = render(geo, torch_mod, ctx, frame, scene, w, h)
    for f in ("rgba", "mask", "uv", "steps"):
        assert np.array_equal(a[f], b[f])  # deterministic
    assert a["total"] == int(a["steps"].astype(np.uint64).sum())
    assert a["steps"].max() < 2048  # budget never binds at step PI/100
    frac = a["mask"].mean()
    # analytic shadow: half-angle 27 deg after aberration -> pi tan^2(27)/(2*3.56) = 11.5 %
    assert 0.105 < frac < 0.125
    assert np.all(a["rgba"][a["mask"] == 1] == np.array([0, 0, 0, 255], np.uint8))
    ref = O.render_f32(frame, scene, sky, w, h, row0=13, nrows=h // 97, row_step=97, threads=16)
    sub = {k: a[k][13::97][: h // 97] for k in ("rgba", "mask", "uv", "steps")}
    assert_same(sub, ref)


def test_adaptive_golden_fixture_bitexact(geo, torch_mod):
    z = np.load(os.path.join(GOLD, "adaptive_64x36.npz"))
    frame = geo.GeoFrame.from_buffer_copy(z["frame"].tobytes())
    ctx = make_ctx(geo, z["sky"])
    scene = geo.make_scene(1.0, 50.0, 1.3, math.pi / 100, 2048, geo.GEO_MODE_ADAPTIVE, tol=1e-6)
    hip = render(geo, torch_mod, ctx, frame, scene, 64, 36)
    assert_same(hip, dict(rgba=z["f32_rgba"], mask=z["f32_mask"], uv=z["f32_uv"], steps=z["f32_steps"]))
    assert np.array_equal(hip["mask"], z["f64_mask"])


ADAPTIVE_SCENES = [
    # name, w, h, frame kwargs, (r_obs, max_steps, tol, rs)
    ("cfg5_small", 384, 216, dict(pos=(1.2, 0.5, 0.0), camera=(math.pi + 0.6, 0.3)), (1.3, 2048, 1e-6, 1.0)),
    ("default_scene", 320, 180, {}, (R_OBS, 2048, 0.0, 1.0)),
    ("tight_tol", 160, 90, {}, (R_OBS, 2048, 1e-9, 1.0)),
    ("budget_7", 160, 90, {}, (R_OBS, 7, 1e-6, 1.0)),
    ("inside_horizon", 128, 128, dict(pos=(0.8, 0.0, 0.05)), (math.sqrt(0.64 + 0.0025), 2048, 1e-6, 1.0)),
    ("flat_space", 128, 72, dict(rs=0.0, state=0), (R_OBS, 2048, 1e-6, 0.0)),
]


@pytest.mark.parametrize("name,w,h,fk,sp", ADAPTIVE_SCENES, ids=[s[0] for s in ADAPTIVE_SCENES])
def test_adaptive_mode_matches_oracle_bitexact(geo, torch_mod, name, w, h, fk, sp):
    """GEO_MODE_ADAPTIVE (config 5): the kernel's RK5(4) loop == the oracle's literal adaptive loop."""
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    r_obs, ms, tol, rs = sp
    sky = make_sky("equirect", (512, 256))
    frame = default_frame(w, h, **{"rs": rs, **fk})
    scene = geo.make_scene(rs, 50.0, r_obs, math.pi / 100, ms, geo.GEO_MODE_ADAPTIVE, tol=tol)
    ctx = make_ctx(geo, sky)
    hip = render(geo, torch_mod, ctx, frame, scene, w, h)
    ref = O.render_f32(frame, scene, sky, w, h, threads=8)
    assert_same(hip, ref)
    assert hip["total"] == ref["steps_total"]


def test_cfg5_8k_adaptive_properties(geo, torch_mod):
    """Full config-5 frame (7680x4320, adaptive): deterministic, step counter
    == sum of per-pixel attempts, sampled rows bit-exact against the oracle,
    and the frame agrees with the fixed-step RK4 frame on the BH mask almost
    everywhere (the two integrators differ only at the photon-ring edge)."""
    from schwarzschild_raytracer_wgpu_amd.scenes import CONFIGS, make_sky

    cfg = CONFIGS["cfg5_8k_adaptive"]
    w, h = cfg.width, cfg.height
    sky = make_sky("equirect", (4096, 2048))
    frame = default_frame(w, h, pos=cfg.position, camera=cfg.camera)
    scene = geo.make_scene(1.0, 50.0, 1.3, math.pi / 100, cfg.max_steps, geo.GEO_MODE_ADAPTIVE, tol=cfg.tol)
    ctx = make_ctx(geo, sky)
    a = render(geo, torch_mod, ctx, frame, scene, w, h)
    assert a["total"] == int(a["steps"].astype(np.uint64).sum())
    assert a["steps"].max() < cfg.max_steps
    ref = O.render_f32(frame, scene, sky, w, h, row0=21, nrows=h // 211, row_step=211, threads=16)
    sub = {k: a[k][21::211][: h // 211] for k in ("rgba", "mask", "uv", "steps")}
    assert_same(sub, ref)
    fixed = render(geo, torch_mod, ctx, frame, default_scene(2048, r_obs=1.3), w, h)
    assert np.mean(fixed["mask"] == a["mask"]) > 0.999
    both = (a["mask"] == 0) & (fixed["mask"] == 0)
    assert np.percentile(wrap_du(a["uv"], fixed["uv"])[both], 99) < 1e-4
    # ~5x fewer attempts than fixed steps
    assert a["total"] < 0.3 * fixed["total"]


def test_invalid_arguments(geo, torch_mod):
    from schwarzschild_raytracer_wgpu_amd import _lib

    ctx = geo.Context(0)
    frame, scene = default_frame(8, 8), default_scene(16)
    dev = torch_mod.device("cuda:0")
    out = torch_mod.empty(8 * 8 * 4, dtype=torch_mod.uint8, device=dev)
    # render before set_sky
    st = _lib.lib.geo_render_rows(ctx._h, ctypes.byref(frame), ctypes.byref(scene), 8, 8, 0, 8, out.data_ptr(),
                                  None, None, None, None, None)
    assert st == _lib.GEO_ESTATE
    # a sky whose padded device copy would reach 2^31 bytes, or wider than 2^20
    dummy = np.zeros(4, np.uint8)
    for w, h in ((1 << 20) + 1, 1), (1, (1 << 20) + 1), (32766, 16384):
        assert _lib.lib.geo_set_sky(ctx._h, dummy.ctypes.data, w, h) == _lib.GEO_EINVAL
    ctx.set_sky(np.zeros((1, 1, 4), np.uint8))
    # rows out of range
    st = _lib.lib.geo_render_rows(ctx._h, ctypes.byref(frame), ctypes.byref(scene), 8, 8, 4, 5, out.data_ptr(),
                                  None, None, None, None, None)
    assert st == _lib.GEO_EINVAL
    # fan mode without a fan
    sc2 = default_scene(16, mode=geo.GEO_MODE_FAN)
    st = _lib.lib.geo_render_rows(ctx._h, ctypes.byref(frame), ctypes.byref(sc2), 8, 8, 0, 8, out.data_ptr(),
                                  None, None, None, None, None)
    assert st == _lib.GEO_ESTATE
    with pytest.raises(geo.GeoError):
        ctx.set_fan(np.zeros(1, np.float32))
    # tol: only in the adaptive mode, and finite >= 0 there
    for sc in (geo.make_scene(1.0, 50.0, 2.5, math.pi / 100, 16, geo.GEO_MODE_DIRECT, tol=1e-6),
               geo.make_scene(1.0, 50.0, 2.5, math.pi / 100, 16, geo.GEO_MODE_ADAPTIVE, tol=-1e-6),
               geo.make_scene(1.0, 50.0, 2.5, math.pi / 100, 16, geo.GEO_MODE_ADAPTIVE, tol=float("nan")),
               geo.make_scene(1.0, 50.0, 2.5, math.pi / 100, 16, geo.GEO_MODE_ADAPTIVE, tol=float("inf")),
               geo.make_scene(1.0, 50.0, 2.5, math.pi / 100, 16, 3)):
        st = _lib.lib.geo_render_rows(ctx._h, ctypes.byref(frame), ctypes.byref(sc), 8, 8, 0, 8, out.data_ptr(),
                                      None, None, None, None, None)
        assert st == _lib.GEO_EINVAL
    # empty frames / row ranges and the step budget limit (a wave's step sum must fit u32)
    for args in ((0, 8, 0, 8), (8, 0, 0, 8), (8, 8, 0, 0)):
        st = _lib.lib.geo_render_rows(ctx._h, ctypes.byref(frame), ctypes.byref(scene), *args, out.data_ptr(),
                                      None, None, None, None, None)
        assert st == _lib.GEO_EINVAL, args
    big = default_scene((1 << 24) + 1)
    st = _lib.lib.geo_render_rows(ctx._h, ctypes.byref(frame), ctypes.byref(big), 8, 8, 0, 8, out.data_ptr(),
                                  None, None, None, None, None)
    assert st == _lib.GEO_EINVAL
    with pytest.raises(geo.GeoError):
        geo.Context(99)


def test_output_buffers_checked_by_bytes_and_type(geo, torch_mod):
    """The Python wrappers refuse outputs that would be overrun: the right
    element count in a narrower dtype (u8 steps, f16 UV, i32 total), the
    wrong type, too few bytes or host memory.  Nothing is launched."""
    torch = torch_mod
    ctx = geo.Context(0)
    ctx.set_sky(np.zeros((1, 1, 4), np.uint8))
    frame, scene = default_frame(8, 8), default_scene(16)
    dev = torch.device("cuda:0")
    n = 64
    rgba = torch.zeros(n * 4, dtype=torch.uint8, device=dev)
    bad = [dict(out_steps=torch.zeros(n, dtype=torch.uint8, device=dev)),
           dict(out_uv=torch.zeros(2 * n, dtype=torch.float16, device=dev)),
           dict(out_uv=torch.zeros(n, dtype=torch.float64, device=dev)),
           dict(steps_total=torch.zeros(1, dtype=torch.int32, device=dev)),
           dict(out_mask=torch.zeros(n - 1, dtype=torch.uint8, device=dev)),
           dict(out_steps=torch.zeros(n, dtype=torch.int32))]
    for kw in bad:
        with pytest.raises(ValueError):
            ctx.render_rows(frame, scene, 8, 8, 0, 8, rgba, **kw)
        with pytest.raises(ValueError):
            ctx.render_bands(frame, scene, 8, 8, 8, 0, 1, 1, rgba, **kw)
        with pytest.raises(ValueError):
            ctx.render_band_set(frame, scene, 8, 8, 8, 0, 8, 1, rgba, **kw)
    with pytest.raises(ValueError):  # 4 B per pixel: an RGBA8 buffer of n elements is too short
        ctx.render_rows(frame, scene, 8, 8, 0, 8, torch.zeros(n, dtype=torch.uint8, device=dev))
    # the RGBA8 target may be any dtype of enough bytes (an int32 view of the frame)
    ok = torch.zeros(n, dtype=torch.int32, device=dev)
    ctx.render_rows(frame, scene, 8, 8, 0, 8, ok, out_steps=torch.zeros(n, dtype=torch.int32, device=dev),
                    steps_total=torch.zeros(1, dtype=torch.int64, device=dev))
    torch.cuda.synchronize()


def test_maximum_step_budget_bitexact(geo, torch_mod):
    """The largest budget the ABI accepts (2^24 steps): every ray still stops on its own
    (crossing, escape or horizon), so the frame equals the oracle's and the 2048-step frame's."""
    w, h = 64, 36
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    sky = make_sky("equirect", (128, 64))
    frame = default_frame(w, h)
    ctx = make_ctx(geo, sky)
    hip = render(geo, torch_mod, ctx, frame, default_scene(1 << 24), w, h)
    ref = O.render_f32(frame, default_scene(1 << 24), sky, w, h, threads=8)
    assert_same(hip, ref)
    hip2k = render(geo, torch_mod, ctx, frame, default_scene(2048), w, h)
    assert np.array_equal(hip["rgba"], hip2k["rgba"]) and np.array_equal(hip["steps"], hip2k["steps"])


def test_three_sphere_composite_bitexact(geo, torch_mod):
    """The reference's three-sphere frame (lib.rs:62-89) drawn pass by pass with
    GEO_FLAG_COMPOSITE into one device target: equal to the oracle's passes."""
    from test_host_kernel_math import three_spheres

    w, h = 320, 180
    frame, passes = three_spheres(w, h)
    ctx = geo.Context(0)
    dev = torch_mod.device("cuda:0")
    rgba = torch_mod.empty(w * h * 4, dtype=torch_mod.uint8, device=dev)
    ref = None
    for scene, sky in passes:
        ctx.set_sky(sky)
        ctx.render_rows(frame, scene, w, h, 0, h, rgba)
        torch_mod.cuda.synchronize()
        ref = O.render_f32(frame, scene, sky, w, h, threads=8, target=None if ref is None else ref["rgba"])
        assert np.array_equal(rgba.cpu().numpy().reshape(h, w, 4), ref["rgba"])


def test_renderer_three_spheres_and_points(geo, torch_mod):
    """Renderer.render over three BasicSphereBuffers (each with its own
    context) + an accretion-disk PointCloud == the oracle's passes + raster."""
    from test_host_kernel_math import three_spheres

    w, h = 256, 144
    frame, passes = three_spheres(w, h)
    obs = geo.Observer(1.0, math.pi / 2, w, h)
    obs.set_position(2.5, 0.0, 0.1)
    spheres = [geo.BasicSphereBuffer(0, sc.sphere_r, 1.0, sky, max_iter=2048) for sc, sky in passes]
    for sp in spheres:
        sp.update_ray_fan(obs.get_radial_position())
    dev = torch_mod.device("cuda:0")
    tgt = geo.RenderTarget(w, h, torch_mod.empty(w * h * 4, dtype=torch_mod.uint8, device=dev))
    from test_points import accretion_disk

    disk = geo.PointCloud(spheres[0].ctx, accretion_disk(1000, seed=2), 1.0, obs.get_position(), True, False)
    fr = geo.Renderer(obs).render(spheres, tgt, point_clouds=[disk])
    torch_mod.cuda.synchronize()
    assert bytes(fr) == bytes(frame)
    ref = None
    for sc, sky in passes:
        ref = O.render_f32(frame, sc, sky, w, h, threads=8, target=None if ref is None else ref["rgba"])
    img, _ = O.draw_points(frame, disk.get_vertices(False), w, h, rgba=ref["rgba"])
    img, _ = O.draw_points(frame, disk.get_vertices(True), w, h, rgba=img)
    assert np.array_equal(tgt.rgba.cpu().numpy().reshape(h, w, 4), img)


def test_points_update_on_side_stream_matches_one_stream(geo, torch_mod):
    """The frame loop with PointCloud.update on a side stream (overlapping the
    sky draw; geo_points_draw orders itself after the update and the next
    update after the draw) == the same loop on one stream, frame by frame,
    with orbits and respawns running."""
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    w, h = 640, 360
    dev = torch_mod.device("cuda:0")
    sky = make_sky("equirect", (1024, 512))

    def loop(side):
        obs = geo.Observer(1.0, math.pi / 2, w, h)
        obs.set_position(2.5, 0.0, 0.1)
        sphere = geo.BasicSphereBuffer(0, 50.0, 1.0, sky, max_iter=2048)
        disk = geo.PointCloud.new_accretion_disk(sphere.ctx, 1.0, obs.get_position(), True, seed=3, n=5000)
        tgt = geo.RenderTarget(w, h, torch_mod.empty(w * h * 4, dtype=torch_mod.uint8, device=dev))
        frames = []
        for _ in range(8):
            obs.update_position((0.0, 0.0, 0.0), 1 / 60)
            sphere.update_ray_fan(obs.get_radial_position())
            disk.update(obs.get_position(), 0.25, stream=side)  # long steps: particles fall and respawn
            geo.Renderer(obs).render([sphere], tgt, point_clouds=[disk])
            frames.append(tgt.rgba.clone())
        torch_mod.cuda.synchronize()
        return [f.cpu().numpy() for f in frames], disk.get_vertices(False), disk.get_vertices(True)

    one = loop(None)
    two = loop(torch_mod.cuda.Stream(dev))
    for a, b in zip(one[0], two[0]):
        assert np.array_equal(a, b)
    assert np.array_equal(one[1], two[1]) and np.array_equal(one[2], two[2])
    red = [int((f.reshape(h, w, 4)[..., :3] == np.array([255, 0, 0], np.uint8)).all(-1).sum()) for f in one[0]]
    assert min(red) > 100  # the disk is drawn in every frame


def test_points_updates_and_draws_across_streams(geo, torch_mod):
    """Back-to-back updates on alternating streams with no draw between them,
    and several draws on different streams before the next update: every
    update waits for the previous update and for all draws before it (the
    chained `drawn` event), so the vertices and frames equal the one-stream
    sequence.  Long dt: particles fall and respawn."""
    torch = torch_mod
    w, h = 320, 180
    dev = torch.device("cuda:0")

    def run(streams):
        ctx = geo.Context(0)
        obs = geo.Observer(1.0, math.pi / 2, w, h)
        obs.set_position(2.5, 0.0, 0.1)
        disk = geo.PointCloud.new_accretion_disk(ctx, 1.0, obs.get_position(), True, seed=11, n=20000)
        tgts = [geo.RenderTarget(w, h, torch.zeros(w * h * 4, dtype=torch.uint8, device=dev)) for _ in range(3)]
        frames = []
        for k in range(6):
            for j in range(3):  # three updates, no draw between them
                obs.update_position((0.0, 0.0, 0.0), 1 / 60)
                disk.update(obs.get_position(), 0.3, stream=streams[(k + j) % len(streams)])
            frame = obs.calc_transformation_pipeline()
            for j, t in enumerate(tgts):  # three draws, on different streams
                t.rgba.zero_()
                torch.cuda.synchronize()
                disk.draw(frame, t, stream=streams[(k + j + 1) % len(streams)])
            obs.update_position((0.0, 0.0, 0.0), 1 / 60)
            disk.update(obs.get_position(), 0.3, stream=streams[k % len(streams)])  # must wait for all 3 draws
            torch.cuda.synchronize()
            frames.append([t.rgba.cpu().numpy() for t in tgts])
        return frames, disk.get_vertices(False), disk.get_vertices(True)

    one = run([None])
    many = run([torch.cuda.Stream(dev), torch.cuda.Stream(dev), None])
    for fa, fb in zip(one[0], many[0]):
        for a, b in zip(fa, fb):
            assert np.array_equal(a, b)
    assert np.array_equal(one[1], many[1]) and np.array_equal(one[2], many[2])


@pytest.mark.parametrize("rotation,nframes", [(3.2, 120), (2.0, 200)])
def test_orbit_replay_render_bitexact(geo, torch_mod, rotation, nframes):
    """N2 scenario replay: an orbiting observer (non-identity movement_to_central,
    observer.rs:215-242) after n frames; the rendered frame == the oracle's."""
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    w, h = 320, 180
    obs = geo.Observer(1.0, math.pi / 2, w, h)
    obs.set_position(2.5, 0.0, 0.1)
    obs.set_camera(math.pi + 0.3, 0.1)
    assert obs.start_orbit(rotation)
    for _ in range(nframes):
        obs.update_position((0.0, 0.0, 0.0), 1 / 60)
    frame = obs.calc_transformation_pipeline()
    m1 = np.array(frame.movement_to_central[:])
    assert not np.allclose(m1, np.eye(4).reshape(-1))
    scene = default_scene(2048, r_obs=obs.get_radial_position())
    sky = make_sky("equirect", (512, 256))
    ctx = make_ctx(geo, sky)
    hip = render(geo, torch_mod, ctx, frame, scene, w, h)
    ref = O.render_f32(frame, scene, sky, w, h, threads=8)
    assert_same(hip, ref)


@pytest.mark.parametrize("world,W,H,B,K", [(3, 40, 37, 8, 2), (8, 64, 2160 // 8, 8, 3), (2, 33, 20, 16, 1)])
def test_assemble_bands_matches_host_assembly(geo, torch_mod, world, W, H, B, K):
    """geo_assemble_bands == the host (torch) reassembly of dist.assemble, for
    every frame of a K-frame batch (16-B and 4-B copy paths)."""
    from schwarzschild_raytracer_wgpu_amd.dist import BandLayout, assemble

    ctx = geo.Context(0)
    L = BandLayout(H, B, world, 0)
    row_bytes = W * 4
    sl = L.nb_max * B * row_bytes
    rng = np.random.default_rng(world * 100 + K)
    src = rng.integers(0, 256, size=world * K * sl, dtype=np.uint8)
    dev = torch_mod.device("cuda:0")
    frame_bytes = L.nb_total * B * row_bytes
    out = torch_mod.zeros(K * H * row_bytes, dtype=torch_mod.uint8, device=dev)
    ctx.assemble_bands(torch_mod.from_numpy(src).to(dev), K * sl, sl, world, B, W, H, K, out)
    got = out.cpu().numpy()
    gl = list(torch_mod.from_numpy(src).chunk(world))
    for f in range(K):
        full = torch_mod.zeros(frame_bytes, dtype=torch_mod.uint8)
        assemble(full, gl, L, row_bytes, frame=f, frame_stride=sl)
        assert np.array_equal(got[f * H * row_bytes:(f + 1) * H * row_bytes], full[:H * row_bytes].numpy()), f
    if W % 4 == 0:
        # RGB24 transport: pack, reassemble with alpha restored == the RGBA path on opaque pixels
        src[3::4] = 255
        dsrc = torch_mod.from_numpy(src).to(dev)
        packed = torch_mod.empty(src.size // 4 * 3, dtype=torch_mod.uint8, device=dev)
        ctx.pack_rgb(dsrc, src.size // 4, packed)
        out3 = torch_mod.zeros_like(out)
        ctx.assemble_bands(packed, K * sl // 4 * 3, sl // 4 * 3, world, B, W, H, K, out3, src_bpp=3)
        out4 = torch_mod.zeros_like(out)
        ctx.assemble_bands(dsrc, K * sl, sl, world, B, W, H, K, out4)
        assert torch_mod.equal(out3, out4)
