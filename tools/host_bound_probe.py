#!/usr/bin/env python3
"""Is an N-rank present loop host-bound?  On ONE GPU, dist.ShardedFrame for
rank 0 and for a peer of an N-rank group on the config-3 frame, with a
gather stand-in that only orders streams (no copy, no links): the host time
of the step loop against the wall time to drain it.  wall ~ host means the
Python/HIP launch path, not the GPU, sets the per-frame time of that rank.

  python tools/host_bound_probe.py [world] [lead] [K] [S] [frames] [batch 0/1]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import schwarzschild_raytracer_wgpu_amd as g
    from schwarzschild_raytracer_wgpu_amd.dist import ShardedFrame
    from schwarzschild_raytracer_wgpu_amd.scenes import CONFIGS, make_sky

    world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    lead = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    S = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    n = int(sys.argv[5]) if len(sys.argv) > 5 else 400
    batch = bool(int(sys.argv[6])) if len(sys.argv) > 6 else False
    cfg = CONFIGS["cfg3_4k"]
    W, H = cfg.width, cfg.height
    obs = g.Observer(cfg.rs, cfg.fov, W, H)
    obs.set_position(*cfg.position)
    frame = obs.calc_transformation_pipeline()
    scene = g.make_scene(cfg.rs, cfg.sphere_r, obs.get_radial_position(), cfg.step, cfg.max_steps)
    ctx = g.Context(0)
    ctx.set_sky(make_sky(cfg.sky, cfg.sky_size))
    dev = torch.device("cuda:0")
    buf = torch.empty(W * H * 4, dtype=torch.uint8, device=dev)
    for _ in range(300):  # clock spin-up
        ctx.render_rows(frame, scene, W, H, 0, H, buf)
    torch.cuda.synchronize()

    class Work:
        def __init__(self, ev):
            self.ev = ev

        def wait(self):
            torch.cuda.current_stream().wait_event(self.ev)

    class OrderOnly:
        """dist.gather stand-in: the collective's stream waits for the caller's,
        nothing moves."""

        def __init__(self):
            self.stream = torch.cuda.Stream()

        def gather(self, src, gather_list=None, dst=0, async_op=True):
            ready = torch.cuda.Event()
            ready.record(torch.cuda.current_stream())
            self.stream.wait_event(ready)
            done = torch.cuda.Event()
            done.record(self.stream)
            return Work(done)

    for rank in (0, 1):
        sf = ShardedFrame(ctx, frame, scene, W, H, 8, rank, world, dev, dist=OrderOnly(), frames_per_gather=K,
                          render_streams=S, lead=lead, batch_launch=batch)
        for i in range(40):
            sf.step(i)
        sf.drain()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n):
            sf.step(i)
        t_host = time.perf_counter() - t0
        sf.drain()
        torch.cuda.synchronize()
        t_wall = time.perf_counter() - t0
        print(f"world {world} lead {lead} K {K} S {S} batch {int(sf.batch)} rank {rank}: host {t_host / n * 1e6:.1f} us/frame, "
              f"wall {t_wall / n * 1e6:.1f} us/frame, rows {sf.layout.rows_mine()}", flush=True)


if __name__ == "__main__":
    main()
