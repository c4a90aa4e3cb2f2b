#!/usr/bin/env python3
"""Per-frame HOST cost of the multi-GPU frame loop's pieces, measured on one
GPU (single-rank RCCL group): the ctypes render_bands call on a tiny frame,
an async dist.gather of a 4 MB slice, and rank 0's band reassembly.  Tells
whether the N = 8 loop (≈ 31 us of GPU work per frame at 4K) is host-bound."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import math

    import numpy as np
    import torch
    import torch.distributed as dist

    import schwarzschild_raytracer_wgpu_amd as g
    from schwarzschild_raytracer_wgpu_amd.dist import BandLayout, assemble

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    ctx = g.Context(0)
    ctx.set_sky(np.full((2, 2, 4), 255, np.uint8))
    obs = g.Observer(1.0, math.pi / 2, 64, 64)
    obs.set_position(2.5, 0, 0.1)
    frame = obs.calc_transformation_pipeline()
    scene = g.make_scene(1.0, 50.0, obs.get_radial_position(), math.pi / 100, 8)
    buf = torch.empty(64 * 8 * 4, dtype=torch.uint8, device=dev)
    n = 2000
    for _ in range(100):
        ctx.render_bands(frame, scene, 64, 64, 8, 0, 1, 1, buf)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        ctx.render_bands(frame, scene, 64, 64, 8, 0, 1, 1, buf)
    t_render = (time.perf_counter() - t) / n
    torch.cuda.synchronize()
    src = torch.empty(4 << 20, dtype=torch.uint8, device=dev)
    recv = [torch.empty_like(src)]
    for _ in range(50):
        dist.gather(src, gather_list=recv, dst=0, async_op=True).wait()
    torch.cuda.synchronize()
    t = time.perf_counter()
    works = []
    for i in range(n):
        works.append(dist.gather(src, gather_list=recv, dst=0, async_op=True))
        if len(works) > 2:
            works.pop(0).wait()
    t_gather = (time.perf_counter() - t) / n
    torch.cuda.synchronize()
    L = BandLayout(2160, 8, 8, 0)
    full = torch.empty(L.nb_total * 8 * 3840 * 4, dtype=torch.uint8, device=dev)
    recv8 = [torch.empty(L.nb_max * 8 * 3840 * 4, dtype=torch.uint8, device=dev) for _ in range(8)]
    t = time.perf_counter()
    for _ in range(200):
        assemble(full, recv8, BandLayout(2160, 8, 8, 0), 3840 * 4)
    t_asm = (time.perf_counter() - t) / 200
    torch.cuda.synchronize()
    sl = L.nb_max * 8 * 3840 * 4
    packed = torch.empty(8 * 4 * sl, dtype=torch.uint8, device=dev)
    frames = torch.empty(4 * 2160 * 3840 * 4, dtype=torch.uint8, device=dev)
    from schwarzschild_raytracer_wgpu_amd.timing import HipEvent

    e0, e1 = HipEvent(), HipEvent()
    t = time.perf_counter()
    e0.record()
    for _ in range(200):
        ctx.assemble_bands(packed, 4 * sl, sl, 8, 8, 3840, 2160, 4, frames)
    e1.record()
    t_gasm = (time.perf_counter() - t) / 200
    gpu_us = e0.elapsed_time(e1) * 1e3 / 200
    torch.cuda.synchronize()
    print(f"host us/frame: render_bands {t_render * 1e6:.1f}, gather(async) {t_gather * 1e6:.1f}, "
          f"torch assemble(8 ranks) {t_asm * 1e6:.1f}, geo_assemble_bands(8 ranks, 4 frames) "
          f"{t_gasm * 1e6:.1f} host / {gpu_us:.1f} GPU")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
