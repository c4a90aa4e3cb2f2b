#!/usr/bin/env python3
"""Bench of the accretion-disk point path: RayConnector
updates per second (PointCloud::update without orbits: update_ray(observer, 1)
on every near- and far-side connector), one JSON line.

  python tools/bench_points.py [--points N] [--steps K] [--warmup W] [--orbits]

Roofline: the connector update streams its 48-node state in and out
(2 x 48 x 4 B), its needs_reset byte in and out, its point (12 B, shared by
the two sides: 6 B per connector) and writes a 16-B vertex: 408 B per
connector update = the algorithmic bytes; bound "hbm" (≈1 kflop per 408 B,
below the gfx950 ridge of ~20 flop/B).  CPU baseline: the oracle's literal
RayConnector (libm transcendentals, the reference algorithm) on one core over
a sample of the same connectors.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
BYTES_PER_CONNECTOR = 2 * 48 * 4 + 2 + 6 + 16


def pmc_traffic(n_conn, orbits):
    """HBM bytes per launch of geo_rays_kernel from the committed rocprofv3 PMC
    summary (the newest profiles/*_points_pmc.json: FETCH_SIZE doubled for
    16-B/lane streaming reads, WRITE_SIZE), for the workload it was taken on,
    else None."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_points_pmc.json")))
    if orbits or not files:
        return None
    with open(files[-1]) as f:
        d = json.load(f)
    return d["derived"]["traffic_bytes"] if d["workload"].startswith(f"{n_conn} connectors") else None


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--points", type=int, default=1 << 21)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=100,
                   help="untimed updates first: the clock ramps for ~25 ms after the set-up's idle gap "
                        "(10 warm-up updates timed 0.307 ms per update, 100 and 300 0.275-0.277; "
                        "tools/gpu_points_warm.sh)")
    p.add_argument("--orbits", action="store_true", help="PointCloud::update with f64 orbits (and respawn)")
    p.add_argument("--cpu-connectors", type=int, default=20000)
    args = p.parse_args()

    import numpy as np
    import torch

    import schwarzschild_raytracer_wgpu_amd as g
    from schwarzschild_raytracer_wgpu_amd.timing import HipEvent
    from test_points import accretion_disk

    n = args.points
    model = accretion_disk(n, seed=1)
    ctx = g.Context(0)
    obs0 = np.array([25.0, 0.0, 1.0], np.float32)
    pc = g.PointCloud(ctx, model, 1.0, obs0, True, args.orbits, seed=5)

    def observer(i):  # slow orbit of the observer (update_ray's regime: small per-frame motion)
        a = 0.002 * i
        return np.array([25.0 * math.cos(a), 25.0 * math.sin(a), 1.0], np.float32)

    for i in range(args.warmup):
        pc.update(observer(i), 1 / 60)
    torch.cuda.synchronize()
    evs = [(HipEvent(), HipEvent()) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        evs[i][0].record()
        pc.update(observer(args.warmup + i), 1 / 60)
        evs[i][1].record()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ms = sorted(a.elapsed_time(b) for a, b in evs)
    ms_avg = sum(ms) / len(ms)
    n_conn = 2 * n
    value = n_conn * args.steps / dt
    achieved = BYTES_PER_CONNECTOR * n_conn / (ms_avg * 1e-3) / 1e9

    # CPU baseline: the oracle's literal RayConnector (reference algorithm, libm) on one core
    import oracle as O

    m = min(args.cpu_connectors // 2, n)
    rays = O.Rays(1.0, model[:m], sides=3, libm=True)
    rays.update(obs0, reset=True)
    t0 = time.perf_counter()
    k = 0
    while True:
        rays.update(observer(k), 1)
        k += 1
        if time.perf_counter() - t0 > 1.0:
            break
    cdt = time.perf_counter() - t0
    out = {
        "metric": "RayConnector updates/s (PointCloud::update, update_ray(observer, 1), near + far side)",
        "value": value,
        "unit": "connector-updates/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "dtype": "f32" + (" (+f64 orbits)" if args.orbits else ""),
        "data": "synthetic accretion disk (r 16..26, |theta| < 0.1), rs = 1, observer circling at r = 25",
        "config": {"workload": f"{n} points x 2 sides = {n_conn} connectors, 48 nodes, 1 Newton iteration",
                   "orbits": bool(args.orbits)},
        "kernel_ms": {"avg": ms_avg, "median": ms[len(ms) // 2], "min": ms[0]},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": achieved / PEAK_HBM_GBS, "traffic": pmc_traffic(n_conn, args.orbits),
                     "algorithmic_bytes_per_connector": BYTES_PER_CONNECTOR},
        "cpu_baseline": {"value": 2 * m * k / cdt, "unit": "connector-updates/s", "cores": 1, "kind": "port",
                         "sample": f"{k} updates of {2 * m} connectors in {cdt:.2f} s (oracle, libm)"},
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
