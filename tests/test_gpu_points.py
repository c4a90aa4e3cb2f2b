"""HIP point path (geo_rays_* / geo_points_* / geo_draw_points) against the
CPU oracle (oracle/geo_oracle_points.c, kernel-polynomial variant): the
RayConnector and vs_main are bit-exact; orbits are f64 with the device math
library, compared with a tolerance.  Also runs the reference's own
RayConnector tests (SR/simulation/tests.rs:15-79, 5e-4 rad) through the C-ABI.
"""
import math

import numpy as np
import pytest

import oracle as O
from helpers import default_frame
from test_points import TOL, accretion_disk, glam_angle_between

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


@pytest.fixture(scope="module")
def ctx(geo, torch_mod):
    return geo.Context(0)


def host(t, torch_mod):
    torch_mod.cuda.synchronize()
    return t.cpu().numpy()


def test_ray_connector_euclidian_hip(geo, ctx, torch_mod):
    """tests.rs:15-38 through the C-ABI: 100 connectors, each reset against its
    own observer on the r = 19 circle (per-point other ends)."""
    n = 100
    pos = np.tile(np.array([20.0, 0.0, 0.1], np.float32), (n, 1))
    ang = np.arange(n, dtype=np.float32) / np.float32(n) * np.float32(math.pi)
    obs = np.stack([np.float32(19) * np.cos(ang), np.float32(19) * np.sin(ang), np.zeros(n, np.float32)], 1)
    rays = geo.RayConnectors(ctx, 0.0, pos)
    out = host(rays.reset_ray(obs), torch_mod)
    ref = O.Rays(0.0, pos, libm=False).update(obs, reset=True)
    assert np.array_equal(out.view(np.uint32), ref.view(np.uint32))
    for i in range(n):
        assert abs(glam_angle_between(pos[i] - obs[i], -obs[i]) - out[i, 3]) < TOL


def test_ray_connector_tracing_hip(geo, ctx, torch_mod):
    """tests.rs:42-79 through the C-ABI, frame by frame bit-exact with the oracle."""
    pos = np.array([[20.0, 0.0, 0.1]], np.float32)
    hip1 = geo.RayConnectors(ctx, 5.0, pos, sides=geo.GEO_RAYS_NEAR | geo.GEO_RAYS_FAR)
    hip5 = geo.RayConnectors(ctx, 5.0, pos, sides=geo.GEO_RAYS_NEAR | geo.GEO_RAYS_FAR)
    ref1 = O.Rays(5.0, pos, sides=3, libm=False)
    ref5 = O.Rays(5.0, pos, sides=3, libm=False)
    for i in range(60):
        a = np.float32(np.float32(i) / np.float32(60) * np.float32(2 * math.pi))
        obs = np.array([np.float32(7) * np.cos(a), np.float32(7) * np.sin(a), 0.0], np.float32)
        o1 = host(hip1.update_ray(obs, 1), torch_mod)
        o5 = host(hip5.update_ray(obs, 5), torch_mod)
        assert np.array_equal(o1.view(np.uint32), ref1.update(obs, 1).view(np.uint32)), i
        assert np.array_equal(o5.view(np.uint32), ref5.update(obs, 5).view(np.uint32)), i
        assert np.all(np.abs(o5[:, 3] - o1[:, 3]) < TOL), i


def test_rays_batch_moving_observer_bitexact(geo, ctx, torch_mod):
    """20k connectors (near + far of 10k disk points), 12 frames of an observer
    spiralling in from r = 25 to r = 1.2 (inside the photon sphere, then the
    horizon crossing at r < 1 is skipped): vertices bit-exact every frame,
    covering resets, jumps, small angles and the inside-horizon branch."""
    pos = accretion_disk(10000, seed=11)
    hip = geo.RayConnectors(ctx, 1.0, pos, sides=3)
    ref = O.Rays(1.0, pos, sides=3, libm=False)
    for f in range(12):
        r = 25.0 * (1.2 / 25.0) ** (f / 11)
        obs = np.array([r * math.cos(0.4 * f), r * math.sin(0.4 * f), 0.3], np.float32)
        o = host(hip.update_ray(obs, 1), torch_mod)
        e = ref.update(obs, 1)
        bad = np.argwhere(o.view(np.uint32) != e.view(np.uint32))
        assert bad.size == 0, (f, bad[:5])


def test_point_cloud_no_orbits_bitexact(geo, ctx, torch_mod):
    model = accretion_disk(3000, seed=2)
    obs = np.array([[25.0, 0.0, 1.0], [24.0, 2.0, 1.0], [20.0, 5.0, 0.5], [12.0, 9.0, 0.2]], np.float32)
    pc = geo.PointCloud(ctx, model, 1.0, obs[0], True, False)
    for f in range(1, 4):
        pc.update(obs[f], 1 / 60)
    near, far, pos = O.points_run(1.0, model, obs, np.full(3, 1 / 60), farside=True, orbits=False, libm=False)
    assert np.array_equal(pc.get_vertices(False).view(np.uint32), near.view(np.uint32))
    assert np.array_equal(pc.get_vertices(True).view(np.uint32), far.view(np.uint32))


def test_point_cloud_orbits_track_oracle(geo, ctx, torch_mod):
    """Accretion disk with f64 orbits (device libm vs glibc: ulp-level
    differences) over 60 frames: positions within 1e-5 relative, angles within
    1e-4 rad; respawns (rs = 15: every particle falls) keep the cloud valid."""
    model = accretion_disk(2000, seed=4)
    obs = np.tile(np.array([25.0, 0.0, 1.0], np.float32), (61, 1))
    pc = geo.PointCloud(ctx, model, 1.0, obs[0], True, True, seed=99)
    for f in range(60):
        pc.update(obs[f + 1], 1 / 60)
    near, far, pos = O.points_run(1.0, model, obs, np.full(60, 1 / 60), seed=99, libm=False)
    p = pc.positions()
    assert np.max(np.abs(p - pos) / np.linalg.norm(pos, axis=1, keepdims=True)) < 1e-5
    assert np.max(np.abs(pc.get_vertices(False)[:, 3] - near[:, 3])) < 1e-4
    assert np.max(np.abs(pc.get_vertices(True)[:, 3] - far[:, 3])) < 1e-4
    # respawn path
    obs2 = np.tile(np.array([40.0, 0.0, 1.0], np.float32), (201, 1))
    pc2 = geo.PointCloud(ctx, accretion_disk(256, seed=5), 15.0, obs2[0], True, True, seed=3)
    for f in range(200):
        pc2.update(obs2[f + 1], 0.5)
    v = pc2.get_vertices(False)
    assert np.all(np.isfinite(v)) and np.all(np.linalg.norm(v[:, :3], axis=1) > 0)


def test_draw_points_bitexact(geo, ctx, torch_mod):
    """The point pipeline over a rendered sphere frame: pixel positions and the
    overlaid frame equal the oracle's vs_main + raster."""
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    w, h = 640, 360
    frame = default_frame(w, h, pos=(25.0, 0.0, 1.0))
    model = accretion_disk(5000, seed=8)
    pc = geo.PointCloud(ctx, model, 1.0, (25.0, 0.0, 1.0), True, False)
    ctx.set_sky(make_sky("equirect", (512, 256)))
    dev = torch_mod.device("cuda:0")
    tgt = geo.RenderTarget(w, h, torch_mod.empty(w * h * 4, dtype=torch_mod.uint8, device=dev))
    scene = geo.make_scene(1.0, 50.0, math.sqrt(626.0), math.pi / 100, 2048)
    ctx.render_rows(frame, scene, w, h, 0, h, tgt.rgba)
    base = host(tgt.rgba, torch_mod).reshape(h, w, 4).copy()
    xy = torch_mod.empty((5000, 2), dtype=torch_mod.int32, device=dev)
    geo.draw_points(ctx, frame, pc.vertices_ptr(False), 5000, tgt, out_xy=xy)
    xy_h = host(xy, torch_mod)
    geo.draw_points(ctx, frame, pc.vertices_ptr(True), 5000, tgt)
    got = host(tgt.rgba, torch_mod).reshape(h, w, 4)
    ref, ref_xy = O.draw_points(frame, pc.get_vertices(False), w, h, rgba=base.copy())
    ref, _ = O.draw_points(frame, pc.get_vertices(True), w, h, rgba=ref)
    assert np.array_equal(xy_h, ref_xy)
    assert np.array_equal(got, ref)
    assert (xy_h[:, 0] >= 0).sum() > 1000  # the disk is in view


def test_point_cloud_draw_equals_two_mesh_draws(geo, ctx, torch_mod):
    """PointCloud.draw (geo_points_draw: the near mesh, then the far mesh,
    event-ordered after the cloud's update) == two geo_draw_points calls, frame
    and per-vertex pixels (out_xy: near side first)."""
    w, h = 320, 180
    frame = default_frame(w, h, pos=(25.0, 0.0, 1.0))
    pc = geo.PointCloud(ctx, accretion_disk(3000, seed=4), 1.0, (25.0, 0.0, 1.0), True, False)
    pc.update((25.0, 0.0, 1.0), 0.0)
    dev = torch_mod.device("cuda:0")
    a = geo.RenderTarget(w, h, torch_mod.zeros(w * h * 4, dtype=torch_mod.uint8, device=dev))
    b = geo.RenderTarget(w, h, torch_mod.zeros(w * h * 4, dtype=torch_mod.uint8, device=dev))
    xy = torch_mod.empty((2 * 3000, 2), dtype=torch_mod.int32, device=dev)
    pc.draw(frame, a, out_xy=xy)
    xn = torch_mod.empty((3000, 2), dtype=torch_mod.int32, device=dev)
    xf = torch_mod.empty((3000, 2), dtype=torch_mod.int32, device=dev)
    geo.draw_points(ctx, frame, pc.vertices_ptr(False), 3000, b, out_xy=xn)
    geo.draw_points(ctx, frame, pc.vertices_ptr(True), 3000, b, out_xy=xf)
    assert np.array_equal(host(a.rgba, torch_mod), host(b.rgba, torch_mod))
    assert np.array_equal(host(xy, torch_mod), np.concatenate([host(xn, torch_mod), host(xf, torch_mod)]))
    assert (host(xy, torch_mod)[:, 0] >= 0).sum() > 500


def test_point_draws_reject_short_buffers(geo, ctx, torch_mod):
    """The point draws write 4 B per target pixel and 2 int32 per vertex: a
    target, out_xy or vertex buffer too small (or out_xy of another dtype) is
    refused before any launch."""
    w, h = 64, 32
    frame = default_frame(w, h, pos=(25.0, 0.0, 1.0))
    dev = torch_mod.device("cuda:0")
    pc = geo.PointCloud(ctx, accretion_disk(100, seed=1), 1.0, (25.0, 0.0, 1.0), True, False)
    ok = geo.RenderTarget(w, h, torch_mod.zeros(w * h * 4, dtype=torch_mod.uint8, device=dev))
    short = geo.RenderTarget(w, h, torch_mod.zeros(w * h * 4 - 1, dtype=torch_mod.uint8, device=dev))
    with pytest.raises(ValueError):
        pc.draw(frame, short)
    with pytest.raises(ValueError):  # near + far: 200 vertices
        pc.draw(frame, ok, out_xy=torch_mod.empty((199, 2), dtype=torch_mod.int32, device=dev))
    with pytest.raises(ValueError):
        pc.draw(frame, ok, out_xy=torch_mod.empty((200, 2), dtype=torch_mod.float32, device=dev))
    verts = torch_mod.zeros((99, 4), dtype=torch_mod.float32, device=dev)
    with pytest.raises(ValueError):
        geo.draw_points(ctx, frame, verts, 100, ok)
    with pytest.raises(ValueError):  # rows [8, 32): 24 rows
        geo.draw_points(ctx, frame, pc.vertices_ptr(False), 100, geo.RenderTarget(
            w, h, torch_mod.zeros(23 * w * 4, dtype=torch_mod.uint8, device=dev)), row0=8)
    pc.draw(frame, ok, out_xy=torch_mod.empty((200, 2), dtype=torch_mod.int32, device=dev))
    geo.draw_points(ctx, frame, pc.vertices_ptr(False), 100, geo.RenderTarget(
        w, h, torch_mod.zeros(24 * w * 4, dtype=torch_mod.uint8, device=dev)), row0=8)
    torch_mod.cuda.synchronize()


def test_rays_updates_alternating_streams_bitexact(geo, ctx, torch_mod):
    """RayConnectors updates issued on alternating non-blocking streams with no
    host sync between them (each waits for the batch's previous update), with
    a set_positions in the middle (it waits for the update in flight): the
    same vertices as the oracle's sequential run."""
    pos = accretion_disk(20000, seed=5)
    pos2 = accretion_disk(20000, seed=6)
    hip = geo.RayConnectors(ctx, 1.0, pos, sides=3)
    ref = O.Rays(1.0, pos, sides=3, libm=False)
    streams = [torch_mod.cuda.Stream() for _ in range(2)]
    for f in range(8):
        r = 25.0 * (2.0 / 25.0) ** (f / 7)
        obs = np.array([r * math.cos(0.3 * f), r * math.sin(0.3 * f), 0.2], np.float32)
        if f == 4:
            hip.set_positions(pos2)
            ref.pos = np.ascontiguousarray(pos2, dtype=np.float32).reshape(-1, 3)  # RayConnector::set_position
        hip.update_ray(obs, 2, stream=streams[f % 2])
        e = ref.update(obs, 2)
    o = host(hip.vertices, torch_mod)
    bad = np.argwhere(o.view(np.uint32) != e.view(np.uint32))
    assert bad.size == 0, bad[:5]
