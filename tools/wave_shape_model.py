"""Lane efficiency of a wave shape, from a frame's own per-pixel step counts:
the mean over waves of the slowest lane's steps (what a wave executes)
against the lane mean.  The CPU library (bit-identical to the kernel) traces
24 8-row strips of config 5 (adaptive attempts) and config 3 (RK4 steps, in
groups of 4 as the loop runs them) and groups them into 64x1, 32x2, 16x4 and
8x8 waves.

    python tools/wave_shape_model.py
"""
import ctypes, os, sys, numpy as np, math
ROOT=os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, ROOT)
import schwarzschild_raytracer_wgpu_amd as g
from schwarzschild_raytracer_wgpu_amd.scenes import CONFIGS, make_sky
def run(name, mode):
    cfg = CONFIGS[name]; W,H = cfg.width, cfg.height
    obs = g.Observer(cfg.rs, cfg.fov, W, H); obs.set_position(*cfg.position); obs.set_camera(*cfg.camera); obs.set_energy(cfg.energy)
    frame = obs.calc_transformation_pipeline()
    scene = g.make_scene(cfg.rs, cfg.sphere_r, obs.get_radial_position(), cfg.step, cfg.max_steps, mode, tol=cfg.tol if mode==2 else 0.0)
    lib = ctypes.CDLL(os.path.join(ROOT, "schwarzschild_raytracer_wgpu_amd", "libgeo_cpu.so"))
    vp, u32 = ctypes.c_void_p, ctypes.c_uint32
    lib.geo_render_cpu.argtypes = [vp, vp, vp, u32, u32, vp, u32, u32, u32, u32, u32, u32, ctypes.c_int, vp, vp, vp, vp, vp]
    sky = np.ascontiguousarray(make_sky("equirect", (64, 32)))
    res = {}
    strips=[]
    for y0 in range(0, H, H//24)[:24]:
        y0 -= y0 % 8
        rgba = np.empty((8, W, 4), np.uint8); m = np.empty((8, W), np.uint8); st = np.empty((8, W), np.uint32)
        rc = lib.geo_render_cpu(ctypes.addressof(frame), ctypes.addressof(scene), sky.ctypes.data, 64, 32, None, 0, W, H, y0, 8, 1, 8, rgba.ctypes.data, m.ctypes.data, None, st.ctypes.data, None)
        assert rc == 0
        strips.append(st.astype(np.int64))
    S = np.stack(strips)  # (n, 8, W)
    lane = S.mean()
    for ww in (64, 32, 16, 8):
        hh = 64 // ww
        if hh > 8: continue
        t = S.reshape(S.shape[0], 8 // hh, hh, W // ww, ww).max(axis=(2, 4))
        if mode == 0:  # groups of 4 steps
            t = np.ceil(t / 4) * 4
        print(f"{name} wave {ww}x{hh}: per-wave max {t.mean():.3f}  lane mean {lane:.3f}  efficiency {lane / t.mean():.3f}")
run("cfg5_8k_adaptive", 2)
run("cfg3_4k", 0)
