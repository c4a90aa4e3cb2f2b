"""North_star's comparator, direct: the HIP kernel (geo_render_rows) against the
CPU reference path bench.py times (geo_render_cpu, libgeo_cpu.so), with no
oracle in between, on sampled rows of BASELINE.json's full-size configs.

North_star asks for "pixel-for-pixel on the hit-classification mask and
within 1e-4 relative on the sky-sphere UV"; both paths compute the same f32
sequence (geo_pixel.h), so the test asks for more: RGBA bytes, mask, UV bits
and step counts identical.  Reference: the integrator both sides run is
sphere_ray_tracer.rs:134-191 + shader.wgsl:57-106.
"""
import ctypes
import os

import numpy as np
import pytest

from schwarzschild_raytracer_wgpu_amd.scenes import CONFIGS, make_sky

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cpu_lib():
    lib = ctypes.CDLL(os.path.join(ROOT, "schwarzschild_raytracer_wgpu_amd", "libgeo_cpu.so"))
    vp, u32 = ctypes.c_void_p, ctypes.c_uint32
    lib.geo_render_cpu.restype = ctypes.c_int
    lib.geo_render_cpu.argtypes = [vp, vp, vp, u32, u32, vp, u32, u32, u32, u32, u32, u32, ctypes.c_int, vp, vp, vp,
                                   vp, vp]
    return lib


def _scene(g, cfg, mode_name=None):
    obs = g.Observer(cfg.rs, cfg.fov, cfg.width, cfg.height)
    obs.set_position(*cfg.position)
    obs.set_camera(*cfg.camera)
    obs.set_energy(cfg.energy)
    frame = obs.calc_transformation_pipeline()
    mode_name = mode_name or cfg.mode
    mode = {"direct": g.GEO_MODE_DIRECT, "fan": g.GEO_MODE_FAN, "adaptive": g.GEO_MODE_ADAPTIVE}[mode_name]
    scene = g.make_scene(cfg.rs, cfg.sphere_r, obs.get_radial_position(), cfg.step, cfg.max_steps, mode,
                         tol=cfg.tol if mode == g.GEO_MODE_ADAPTIVE else 0.0)
    return obs, frame, scene, mode


# (config, row step, mode): about 300 k-600 k pixels each
CASES = [("cfg2_1080p", 9, None), ("cfg3_4k", 27, None), ("cfg5_8k_adaptive", 54, None), ("cfg3_4k", 27, "fan")]


@pytest.mark.parametrize("name,k,mode_name", CASES, ids=[f"{c[0]}_{c[2] or 'default'}" for c in CASES])
def test_hip_equals_cpu_path(dev, name, k, mode_name):
    import torch

    import schwarzschild_raytracer_wgpu_amd as g

    cfg = CONFIGS[name]
    W, H = cfg.width, cfg.height
    obs, frame, scene, mode = _scene(g, cfg, mode_name)
    sky = np.ascontiguousarray(make_sky(cfg.sky, cfg.sky_size))
    ctx = g.Context(dev.index or 0)
    ctx.set_sky(sky)
    fan = None
    if mode == g.GEO_MODE_FAN:
        fan = ctx.solve_ray_fan(cfg.sphere_r, cfg.rs, cfg.max_steps, cfg.step, 400, obs.get_radial_position())
    # the GPU: the whole frame, then its every k-th row
    rgba = torch.empty(H * W * 4, dtype=torch.uint8, device=dev)
    mask = torch.empty(H * W, dtype=torch.uint8, device=dev)
    uv = torch.empty(H * W * 2, dtype=torch.float32, device=dev)
    steps = torch.empty(H * W, dtype=torch.int32, device=dev)
    ctx.render_rows(frame, scene, W, H, 0, H, rgba, out_mask=mask, out_uv=uv, out_steps=steps)
    torch.cuda.synchronize()
    gr = rgba.view(H, W, 4)[::k].cpu().numpy()
    gm = mask.view(H, W)[::k].cpu().numpy()
    gu = uv.view(H, W, 2)[::k].cpu().numpy()
    gs = steps.view(H, W)[::k].cpu().numpy().view(np.uint32)
    ctx.close()
    # the CPU path: the same rows
    lib = _cpu_lib()
    n = (H + k - 1) // k
    cr = np.empty((n, W, 4), np.uint8)
    cm = np.empty((n, W), np.uint8)
    cu = np.empty((n, W, 2), np.float32)
    cs = np.empty((n, W), np.uint32)
    total = ctypes.c_ulonglong()
    fan_a = None if fan is None else np.ascontiguousarray(fan, np.float32)
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    rc = lib.geo_render_cpu(ctypes.addressof(frame), ctypes.addressof(scene), sky.ctypes.data, sky.shape[1],
                            sky.shape[0], None if fan_a is None else fan_a.ctypes.data,
                            0 if fan_a is None else fan_a.size, W, H, 0, n, k, threads, cr.ctypes.data,
                            cm.ctypes.data, cu.ctypes.data, cs.ctypes.data, ctypes.addressof(total))
    assert rc == 0
    # north_star's bar first (mask exact, UV within 1e-4, U wrap-aware), then bits
    assert int((cm != gm).sum()) == 0, f"{name}: {int((cm != gm).sum())} mask mismatches"
    du = np.abs(cu[..., 0].astype(np.float64) - gu[..., 0])
    du = np.minimum(du, 1.0 - du)
    dv = np.abs(cu[..., 1].astype(np.float64) - gu[..., 1])
    assert max(du.max(), dv.max()) <= 1e-4
    assert np.array_equal(cu.view(np.uint32), gu.view(np.uint32)), f"{name}: UV bits differ"
    assert np.array_equal(cr, gr), f"{name}: RGBA differs"
    assert np.array_equal(cs, gs), f"{name}: steps differ"
    assert total.value == int(gs.astype(np.int64).sum())
    assert 0.0 < cm.mean() < 0.5  # a real frame: both classes present
