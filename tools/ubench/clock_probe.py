"""Per-frame kernel time of the config-3 frame along a long back-to-back run,
and after host gaps of various lengths: how fast the GPU clock ramps and how
fast it falls back when the queue runs dry (bench.py's spin-up/warmup)."""
import math
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

import schwarzschild_raytracer_wgpu_amd as g  # noqa: E402
from schwarzschild_raytracer_wgpu_amd.scenes import make_sky  # noqa: E402
from schwarzschild_raytracer_wgpu_amd.timing import HipEvent  # noqa: E402

W, H = 3840, 2160
o = g.Observer(1.0, math.pi / 2, W, H)
o.set_position(2.5, 0.0, 0.1)
fr = o.calc_transformation_pipeline()
sc = g.make_scene(1.0, 50.0, o.get_radial_position(), math.pi / 100, 2048, flags=g._lib.GEO_FLAG_DEFER_STEPS)
ctx = g.Context(0)
ctx.set_sky(make_sky("equirect", (4096, 2048)))
dev = torch.device("cuda:0")
out = torch.empty(W * H * 4, dtype=torch.uint8, device=dev)
stream = torch.cuda.current_stream().cuda_stream


def frames(n, sync_every=0):
    evs = [(HipEvent(), HipEvent()) for _ in range(n)]
    for i in range(n):
        evs[i][0].record()
        ctx.render_bands(fr, sc, W, H, 8, 0, 1, H // 8, out, stream=stream)
        evs[i][1].record()
        if sync_every and i % sync_every == sync_every - 1:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    return [a.elapsed_time(b) for a, b in evs]


def summ(ks, step):
    return " ".join(f"{sum(ks[i:i + step]) / len(ks[i:i + step]):.3f}" for i in range(0, len(ks), step))


time.sleep(1.0)
ks = frames(3000)
print("cold, 3000 back-to-back frames, mean per 100:", summ(ks, 100), flush=True)
for gap_ms in (0, 1, 3, 10, 30, 100, 300, 1000):
    torch.cuda.synchronize()
    time.sleep(gap_ms / 1e3)
    ks = frames(60)
    print(f"after {gap_ms:4d} ms idle, 60 frames, per 5:", summ(ks, 5), flush=True)
ks = frames(3000, sync_every=50)
print("3000 frames with a sync every 50, mean per 100:", summ(ks, 100), flush=True)
ctx.steps_flush(torch.zeros(1, dtype=torch.int64, device=dev))
