"""Does the workgroup dispatch order shorten a frame?  (VERDICT r03 "next" 6:
config 2's 71 % against config 3's 85 % is launch and tail.)

Per config: one diagnostic render gives every pixel's steps; a tile's cost is
the sum over its four waves of the wave's largest step count (a wave holds
its slot until its slowest lane stops).  Orders, timed interleaved with
event pairs around each of N back-to-back launches after a spin-up:
  natural  row-major (the product default)
  lpt      most expensive tile first (longest processing time first)
  rev      cheapest first (the worst case, a sanity check that order matters)
  xcd      XCD regions: workgroups are dealt round-robin over the 8 XCDs
           (block i on XCD i % 8), so XCD k gets the k-th eighth of the tiles
           in row-major order, whose sky lines then meet in one L2
  xcd_lpt  the same regions, each in longest-first order
  xcd_blk  XCD regions as a 2 x 4 grid of blocks of tiles (fan mode: every
           tile costs the same, so regions of equal size finish together)
  auto     the product default: GEO_DISPATCH_LONGEST_FIRST, the order learned
           on the device every 16 renders (its recording renders and
           rebuild kernels inside the timed launches)
  python tools/order_probe.py [cfg2_1080p cfg3_4k cfg3_4k:fan cfg3_4k@8 ...]
  (CFG@N: rank 1's share of an N-rank job, the interleaved 8-row bands
  1, 1 + N, ... rendered by one geo_render_band_set, as bench.py's ranks do)
"""
import json
import os
import statistics
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import schwarzschild_raytracer_wgpu_amd as g  # noqa: E402
from schwarzschild_raytracer_wgpu_amd.scenes import CONFIGS, make_sky  # noqa: E402
from schwarzschild_raytracer_wgpu_amd.timing import HipEvent  # noqa: E402

TW, TH, WW, WH = 32, 8, 16, 4  # tile and wave shapes (geo_render.hip)


def xcd_order(packed, rank=None, parts=None):
    """Block i -> XCD i % 8: XCD k's blocks take the k-th eighth of `packed`
    (row-major tiles; or parts[k], indices into packed), in `rank` order
    within the eighth if given."""
    n = packed.size
    parts = np.array_split(np.arange(n), 8) if parts is None else parts
    if rank is not None:
        parts = [p[np.argsort(rank[p], kind="stable")] for p in parts]
    out = np.empty(n, np.uint32)
    pos = 0
    i = 0
    # deal: block i goes to part i % 8 while it has tiles left (parts differ by at most one tile)
    cursors = [0] * 8
    while pos < n:
        k = i % 8
        if cursors[k] < parts[k].size:
            out[pos] = packed[parts[k][cursors[k]]]
            cursors[k] += 1
            pos += 1
        i += 1
    return out


def tile_costs(steps, W, H, th=TH):
    ty, tx = (H + th - 1) // th, (W + TW - 1) // TW
    s = np.zeros((ty * th, tx * TW), np.int64)
    s[:H, :W] = steps
    wh = WH * th // TH  # a fan-mode wave covers 16 x 8 (two pixels per lane)
    waves = s.reshape(ty * th // wh, wh, tx * TW // WW, WW).max(axis=(1, 3))  # (rows of waves, cols of waves)
    return waves.reshape(ty, th // wh, tx, TW // WW).sum(axis=(1, 3)), tx, ty


def main():
    names = sys.argv[1:] or ["cfg2_1080p", "cfg3_4k", "cfg5_8k_adaptive", "cfg3_4k:fan"]
    dev = torch.device("cuda", 0)
    out = {}
    for spec in names:
        spec0, _, nranks = spec.partition("@")
        name, _, mname = spec0.partition(":")
        nranks = int(nranks or 1)
        cfg = CONFIGS[name]
        W, H = cfg.width, cfg.height
        obs = g.Observer(cfg.rs, cfg.fov, W, H)
        obs.set_position(*cfg.position)
        obs.set_camera(*cfg.camera)
        obs.set_energy(cfg.energy)
        frame = obs.calc_transformation_pipeline()
        mname = mname or cfg.mode
        mode = {"direct": g.GEO_MODE_DIRECT, "fan": g.GEO_MODE_FAN, "adaptive": g.GEO_MODE_ADAPTIVE}[mname]
        scene = g.make_scene(cfg.rs, cfg.sphere_r, obs.get_radial_position(), cfg.step, cfg.max_steps, mode,
                             tol=cfg.tol if mode == g.GEO_MODE_ADAPTIVE else 0.0)
        ctx = g.Context(0)
        ctx.set_sky(make_sky(cfg.sky, cfg.sky_size))
        fan = mode == g.GEO_MODE_FAN
        if fan:
            ctx.solve_ray_fan(cfg.sphere_r, cfg.rs, cfg.max_steps, cfg.step, 400, obs.get_radial_position())
        if nranks > 1:  # rank 1's bands of an nranks-way interleave (bench.py's layout, lead 1)
            nb = len(range(1, (H + 7) // 8, nranks))
            rows = nb * 8

            def draw(out, **kw):
                ctx.render_band_set(frame, scene, W, H, 8, 8, 8 * nranks, nb, out, **kw)
        else:
            rows = H

            def draw(out, **kw):
                ctx.render_rows(frame, scene, W, H, 0, H, out, **kw)
        rgba = torch.empty(rows * W * 4, dtype=torch.uint8, device=dev)
        steps = torch.empty(rows * W, dtype=torch.int32, device=dev)
        draw(rgba, out_steps=steps)
        torch.cuda.synchronize()
        cost, tx, ty = tile_costs(steps.view(rows, W).cpu().numpy(), W, rows, th=16 if fan else TH)
        packed = (np.arange(ty)[:, None] << 16 | np.arange(tx)[None, :]).astype(np.uint32).ravel()
        by_cost = np.argsort(-cost.ravel(), kind="stable")
        orders = {"natural": None, "xcd": xcd_order(packed)}
        if fan:
            idx = np.arange(tx * ty).reshape(ty, tx)
            orders["xcd_blk"] = xcd_order(packed, parts=[b.ravel() for rb in np.array_split(idx, 4, axis=0)
                                                         for b in np.array_split(rb, 2, axis=1)])
        if not fan:
            orders["auto"] = "auto"
        if not fan:  # fan-mode pixels have no steps: every tile costs the same
            orders.update(lpt=packed[by_cost], rev=packed[by_cost[::-1]],
                          xcd_lpt=xcd_order(packed, rank=-cost.ravel()))
        keep = os.environ.get("PROBE_ORDERS")  # e.g. "natural,auto"
        if keep:
            orders = {k: v for k, v in orders.items() if k in keep.split(",")}
        n = 400 if rows * W <= 1920 * 1080 else 200
        res = {k: [] for k in orders}
        span = {}
        for rep in range(3):
            for k, o in orders.items():
                if isinstance(o, str):
                    ctx.set_dispatch(g._lib.GEO_DISPATCH_LONGEST_FIRST, 16)
                else:
                    ctx.set_tile_order(tx, ty, o)
                for _ in range(300):  # clock spin-up
                    draw(rgba)
                evs = [(HipEvent(), HipEvent()) for _ in range(n)]
                t0 = HipEvent()
                t0.record()
                for a, b in evs:
                    a.record()
                    draw(rgba)
                    b.record()
                torch.cuda.synchronize()
                res[k].append(statistics.median(a.elapsed_time(b) for a, b in evs))
                span.setdefault(k, []).append(t0.elapsed_time(evs[-1][1]) / n)
        ctx.set_tile_order(tx, ty, None)
        ref = rgba.clone()
        draw(ref)
        ctx.set_tile_order(tx, ty, packed[by_cost])
        draw(rgba)
        torch.cuda.synchronize()
        same = bool(torch.equal(ref, rgba))
        ctx.close()
        out[spec] = {"median_kernel_ms": {k: [round(v, 5) for v in vs] for k, vs in res.items()},
                     "mean_frame_ms": {k: [round(v, 5) for v in vs] for k, vs in span.items()},
                     "tiles": int(tx * ty), "lpt_frame_identical": same,
                     "cost_top1pct_share": float(np.sort(cost.ravel())[::-1][: max(1, cost.size // 100)].sum()
                                                 / cost.sum())}
        print(spec, json.dumps(out[spec]), flush=True)


if __name__ == "__main__":
    main()
