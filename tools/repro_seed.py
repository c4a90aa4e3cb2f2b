"""Render one fuzz scene (tests/fuzz_scenes.py) on the GPU and compare it with
the oracle's f32 restatement: the pixels that differ, with their steps.

    python tools/repro_seed.py SEED [--adaptive] [--w 64 --h 36]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("seed", type=int)
    p.add_argument("--adaptive", action="store_true")
    p.add_argument("--w", type=int, default=64)
    p.add_argument("--h", type=int, default=36)
    a = p.parse_args()
    import torch

    import oracle as O
    import schwarzschild_raytracer_wgpu_amd as g
    from fuzz_scenes import random_scene
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky
    from test_gpu_parity import make_ctx, render

    frame, scene, desc = random_scene(a.seed, a.w, a.h, adaptive=a.adaptive)
    print(desc)
    sky = make_sky("equirect", (256, 128))
    ctx = make_ctx(g, sky)
    hip = render(g, torch, ctx, frame, scene, a.w, a.h)
    ref = O.render_f32(frame, scene, sky, a.w, a.h, threads=4)
    for f in ("mask", "steps", "rgba"):
        d = np.argwhere((hip[f] != ref[f]).reshape(a.h, a.w, -1).any(axis=2))
        print(f, len(d), [tuple(x) for x in d[:6]])
    d = np.argwhere((hip["uv"].view(np.uint32) != ref["uv"].view(np.uint32)).any(axis=2))
    print("uv", len(d), [tuple(x) for x in d[:6]])
    for y, x in d[:6]:
        print(f"  ({y},{x}) steps hip {hip['steps'][y, x]} ref {ref['steps'][y, x]} mask {hip['mask'][y, x]}/"
              f"{ref['mask'][y, x]} uv {hip['uv'][y, x]} {ref['uv'][y, x]}")


if __name__ == "__main__":
    main()
