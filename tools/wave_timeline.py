#!/usr/bin/env python3
"""Where a render launch's time goes, from every wave's own start and end.

A diagnostic build of libgeo (tools/build_variant.py ... -DGEO_WAVE_LOG=1,
tools/ab/libgeo_wavelog.so; the product library is never built this way and
its device code is unchanged by the option) has each wave write, after its
pixels, {start, end} from s_memrealtime (the 100 MHz constant clock every
XCD shares), its HW_ID and XCC_ID, and its tile and largest step count, to
a side buffer (geo_debug_set_wave_log; vector stores of lane 0, never the
render's outputs).  Per launch this prints:

  event     the launch's event-pair duration (geo_time_next_render)
  span      first wave start -> last wave end (the kernel's busy interval)
  outside   event - span: dispatch to the first wave plus the last wave to
            the completion signal
  ramp      first wave start -> the resident waves first reach 90 % of the
            launch's steady level (the median over the middle half)
  drain     the resident waves last at 90 % of it -> last wave end
  ideal     the wave-time sum / the steady level: the span at steady
            occupancy with no ramp or drain
  loss      span - ideal

    python tools/wave_timeline.py [--lib tools/ab/libgeo_wavelog.so] [--frames 8] [--out FILE.json]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

TICK_US = 0.01  # s_memrealtime: 100 MHz


def load(path):
    import torch  # noqa: F401  (the HIP runtime first, as _lib does)

    from schwarzschild_raytracer_wgpu_amd._lib import SIGNATURES

    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    lib.geo_debug_set_wave_log.restype = ctypes.c_int
    lib.geo_debug_set_wave_log.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    return lib


def analyse(log, event_ms):
    import numpy as np

    t0 = log[:, 0].astype(np.int64)
    t1 = log[:, 1].astype(np.int64)
    keep = t1 > 0  # every wave writes its entry
    t0, t1 = t0[keep], t1[keep]
    base = t0.min()
    t0, t1 = t0 - base, t1 - base
    span = int(t1.max())
    # resident waves per tick
    occ = np.zeros(span + 2, np.int64)
    np.add.at(occ, t0, 1)
    np.add.at(occ, t1, -1)
    occ = np.cumsum(occ)[:span + 1]
    mid = occ[span // 4: 3 * span // 4 + 1]
    steady = float(np.median(mid)) if mid.size else float(occ.max())
    hi = np.nonzero(occ >= 0.9 * steady)[0]
    ramp = int(hi[0]) if hi.size else 0
    drain = span - int(hi[-1]) if hi.size else 0
    busy = float((t1 - t0).sum())
    ideal = busy / steady if steady > 0 else float(span)
    xcc = (log[keep, 2] >> 32).astype(np.int64)
    per_xcc_end = [int((t1[xcc == x]).max()) for x in sorted(set(xcc.tolist()))]
    return {
        "waves": int(keep.sum()),
        "event_us": event_ms * 1e3,
        "span_us": span * TICK_US,
        "outside_us": event_ms * 1e3 - span * TICK_US,
        "ramp_us": ramp * TICK_US,
        "drain_us": drain * TICK_US,
        "steady_waves": steady,
        "peak_waves": int(occ.max()),
        "ideal_us": ideal * TICK_US,
        "loss_us": (span - ideal) * TICK_US,
        "last_start_us": int(t0.max()) * TICK_US,
        "wave_us_median": float(np.median(t1 - t0)) * TICK_US,
        "wave_us_max": float((t1 - t0).max()) * TICK_US,
        "xcc_end_spread_us": (max(per_xcc_end) - min(per_xcc_end)) * TICK_US,
        "xccs": len(per_xcc_end),
    }


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--lib", default=os.path.join(ROOT, "tools", "ab", "libgeo_wavelog.so"))
    p.add_argument("--frames", type=int, default=8)
    p.add_argument("--warm", type=int, default=200)
    p.add_argument("--out", default=None)
    p.add_argument("--cases", default="cfg2,cfg3,cfg3_fan,cfg5,share8,share8_batch")
    a = p.parse_args()
    import numpy as np
    import torch

    import schwarzschild_raytracer_wgpu_amd as g
    from schwarzschild_raytracer_wgpu_amd.dist import BandLayout
    from schwarzschild_raytracer_wgpu_amd.scenes import CONFIGS, make_sky
    from schwarzschild_raytracer_wgpu_amd.timing import HipEvent

    lib = load(a.lib)
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    sky = np.ascontiguousarray(make_sky("equirect", (4096, 2048)))
    results = []

    def check(st, what):
        if st != 0:
            raise SystemExit(f"{what}: {st}")

    for case in a.cases.split(","):
        cfgname = {"cfg2": "cfg2_1080p", "cfg5": "cfg5_8k_adaptive"}.get(case.split("_")[0], "cfg3_4k")
        cfg = CONFIGS[cfgname]
        W, H = cfg.width, cfg.height
        mode = {"direct": 0, "fan": 1, "adaptive": 2}["fan" if case.endswith("fan") else cfg.mode]
        obs = g.Observer(cfg.rs, cfg.fov, W, H)
        obs.set_position(*cfg.position)
        obs.set_camera(*cfg.camera)
        obs.set_energy(cfg.energy)
        frame = obs.calc_transformation_pipeline()
        scene = g.make_scene(cfg.rs, cfg.sphere_r, obs.get_radial_position(), cfg.step, cfg.max_steps, mode,
                             tol=cfg.tol if mode == 2 else 0.0)
        for order in ("learned", "natural"):
            h = ctypes.c_void_p()
            check(lib.geo_ctx_create(0, ctypes.byref(h)), "ctx")
            check(lib.geo_set_sky(h, sky.ctypes.data, sky.shape[1], sky.shape[0]), "sky")
            if mode == 1:
                check(lib.geo_solve_ray_fan(h, cfg.sphere_r, cfg.rs, cfg.max_steps, cfg.step, 400,
                                            obs.get_radial_position(), None, stream), "fan")
            if order == "natural":
                check(lib.geo_set_dispatch(h, 0, 16), "dispatch")
            nframes = 8 if case.endswith("batch") else 1
            if case.startswith("share"):
                L = BandLayout(H, 8, 8, 1)
                band = (L.band_height(), L.row0(), L.cycle_rows, L.nbands())
                rows = L.packed_rows()
            else:
                band = None
                rows = H
            out = torch.empty(nframes * rows * W * 4, dtype=torch.uint8, device=dev)
            tiles = math.ceil(W / 32) * math.ceil(rows / (16 if mode == 1 else 8))
            log = torch.zeros(nframes * tiles * 4 * 4, dtype=torch.int64, device=dev)
            frames = (g.GeoFrame * nframes)(*([frame] * nframes))
            scenes = (g.GeoScene * nframes)(*([scene] * nframes))

            def render(ev=None):
                if ev is not None:
                    check(lib.geo_time_next_render(h, ev[0].h, ev[1].h), "time")
                if band is None:
                    check(lib.geo_render_rows(h, frame, scene, W, H, 0, H, out.data_ptr(), None, None, None, None,
                                              stream), "render")
                else:
                    check(lib.geo_render_band_set_batch(h, frames, scenes, nframes, W, H, band[0], band[1], band[2],
                                                        band[3], out.data_ptr(), rows * W * 4, None, stream), "batch")

            for _ in range(a.warm):
                render()
            # the clock falls within ~1 ms of an idle queue and takes ~25 ms of
            # work to come back (bench.py): every logged launch follows >= 30 ms
            # of plain ones, queued behind it with no sync in between
            ev0 = (HipEvent(), HipEvent())
            render(ev0)
            torch.cuda.synchronize()
            pre = max(8, math.ceil(30.0 / max(ev0[0].elapsed_time(ev0[1]), 1e-3)))
            per = []
            for _ in range(a.frames):
                log.zero_()
                ev = (HipEvent(), HipEvent())
                for _ in range(pre):
                    render()
                check(lib.geo_debug_set_wave_log(h, ctypes.c_void_p(log.data_ptr())), "log")
                render(ev)
                check(lib.geo_debug_set_wave_log(h, None), "log off")
                torch.cuda.synchronize()
                per.append(analyse(log.view(-1, 4).cpu().numpy(), ev[0].elapsed_time(ev[1])))
            lib.geo_ctx_destroy(h)
            med = {k: statistics.median(r[k] for r in per) for k in per[0]}
            med.update(case=case, order=order, frames_per_launch=nframes, width=W, rows=rows, mode=mode)
            results.append(med)
            print(f"{case:13s} {order:8s} event {med['event_us']:7.1f} us  span {med['span_us']:7.1f}  outside "
                  f"{med['outside_us']:5.1f}  ramp {med['ramp_us']:5.1f}  drain {med['drain_us']:6.1f}  ideal "
                  f"{med['ideal_us']:7.1f}  loss {med['loss_us']:6.1f}  steady {med['steady_waves']:6.0f} / peak "
                  f"{med['peak_waves']:5.0f}  waves {med['waves']:6.0f}  wave median {med['wave_us_median']:5.1f} "
                  f"max {med['wave_us_max']:5.1f} us  last start {med['last_start_us']:6.1f}", flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
