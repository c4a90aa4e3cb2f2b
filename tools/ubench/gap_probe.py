"""Where do the inter-frame gaps come from?  ms/frame for K back-to-back 4K
frames with/without per-frame events and the step counter."""
import math
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

import schwarzschild_raytracer_wgpu_amd as g  # noqa: E402
from schwarzschild_raytracer_wgpu_amd.scenes import make_sky  # noqa: E402

W, H, K = 3840, 2160, 30
o = g.Observer(1.0, math.pi / 2, W, H)
o.set_position(2.5, 0.0, 0.1)
fr = o.calc_transformation_pipeline()
sc = g.make_scene(1.0, 50.0, o.get_radial_position(), math.pi / 100, 2048)
ctx = g.Context(0)
ctx.set_sky(make_sky("equirect", (4096, 2048)))
dev = torch.device("cuda:0")
out = torch.empty(W * H * 4, dtype=torch.uint8, device=dev)
ctr = torch.zeros(1, dtype=torch.int64, device=dev)
stream = torch.cuda.current_stream().cuda_stream


def run(events, counter, bands):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        if events:
            evs[i][0].record()
        if bands:
            ctx.render_bands(fr, sc, W, H, 8, 0, 1, H // 8, out, steps_total=ctr if counter else None, stream=stream)
        else:
            ctx.render_rows(fr, sc, W, H, 0, H, out, steps_total=ctr if counter else None, stream=stream)
        if events:
            evs[i][1].record()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / K * 1e3
    k = sum(a.elapsed_time(b) for a, b in evs) / K if events else float("nan")
    return dt, k


for rep in range(3):
    for ev in (False, True):
        for cnt in (False, True):
            dt, k = run(ev, cnt, True)
            print(f"rep{rep} events={ev:d} counter={cnt:d}: {dt:.4f} ms/frame (event kernel avg {k:.4f})")
t0 = time.perf_counter()
for i in range(200):
    ctx.render_bands(fr, sc, 8, 8, 8, 0, 1, 1, out, stream=stream)
torch.cuda.synchronize()
print(f"tiny-launch host+GPU rate: {(time.perf_counter() - t0) / 200 * 1e6:.1f} us/launch")
