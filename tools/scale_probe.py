#!/usr/bin/env python3
"""Strong-scaling probe on ONE GPU: the per-rank render of the 4K frame's
interleaved bands for N = 1, 2, 4, 8 (every rank's share timed in turn, the
max reported) against full-frame/N — the compute-only part of the N-GPU run
(tail effects of a smaller grid), without the gather."""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import schwarzschild_raytracer_wgpu_amd as g
    from schwarzschild_raytracer_wgpu_amd.dist import BandLayout
    from schwarzschild_raytracer_wgpu_amd.scenes import CONFIGS, make_sky
    from schwarzschild_raytracer_wgpu_amd.timing import HipEvent

    band_rows = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    cfg = CONFIGS["cfg3_4k"]
    W, H = cfg.width, cfg.height
    obs = g.Observer(cfg.rs, cfg.fov, W, H)
    obs.set_position(*cfg.position)
    frame = obs.calc_transformation_pipeline()
    scene = g.make_scene(cfg.rs, cfg.sphere_r, obs.get_radial_position(), cfg.step, cfg.max_steps)
    ctx = g.Context(0)
    ctx.set_sky(make_sky(cfg.sky, cfg.sky_size))
    buf = torch.empty(W * H * 4, dtype=torch.uint8, device="cuda:0")
    for _ in range(300):
        ctx.render_rows(frame, scene, W, H, 0, H, buf)
    torch.cuda.synchronize()

    def timed(fn, reps=40):
        evs = [(HipEvent(), HipEvent()) for _ in range(reps)]
        for a, b in evs:
            a.record()
            fn()
            b.record()
        torch.cuda.synchronize()
        ms = sorted(a.elapsed_time(b) for a, b in evs)
        return ms[len(ms) // 2]

    full = timed(lambda: ctx.render_rows(frame, scene, W, H, 0, H, buf))
    print(f"band_rows {band_rows}: full frame {full:.4f} ms")
    for n in (2, 4, 8):
        worst = 0.0
        for r in range(n):
            L = BandLayout(H, band_rows, n, r)
            t = timed(lambda: ctx.render_bands(frame, scene, W, H, band_rows, r, n, L.nb_mine, buf))
            worst = max(worst, t)
        print(f"  N={n}: max rank {worst:.4f} ms vs full/N {full / n:.4f} ms -> compute efficiency "
              f"{full / n / worst:.3f}")


if __name__ == "__main__":
    main()


def overlap_probe():
    """Wall time per frame of back-to-back rank-0 shares at N = 8 on 1, 2 or 3
    streams (frame i on stream i % S): does the next frame fill the tail?"""
    import time

    import torch

    import schwarzschild_raytracer_wgpu_amd as g
    from schwarzschild_raytracer_wgpu_amd.dist import BandLayout
    from schwarzschild_raytracer_wgpu_amd.scenes import CONFIGS, make_sky

    cfg = CONFIGS["cfg3_4k"]
    W, H = cfg.width, cfg.height
    obs = g.Observer(cfg.rs, cfg.fov, W, H)
    obs.set_position(*cfg.position)
    frame = obs.calc_transformation_pipeline()
    scene = g.make_scene(cfg.rs, cfg.sphere_r, obs.get_radial_position(), cfg.step, cfg.max_steps)
    ctx = g.Context(0)
    ctx.set_sky(make_sky(cfg.sky, cfg.sky_size))
    for n in (1, 8):
        L = BandLayout(H, 8, n, 0)
        bufs = [torch.empty(L.nb_max * 8 * W * 4, dtype=torch.uint8, device="cuda:0") for _ in range(4)]
        for S in (1, 2, 3):
            streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(S - 1)]
            for rep in range(2):
                frames = 400 if n == 8 else 100
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i in range(frames):
                    ctx.render_bands(frame, scene, W, H, 8, 0, n, L.nb_mine, bufs[i % 4],
                                     stream=streams[i % S].cuda_stream)
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) / frames * 1e3
            print(f"N={n} rank-0 share, {S} stream(s): {dt:.4f} ms/frame")


if __name__ == "__main__" and os.environ.get("OVERLAP"):
    overlap_probe()
