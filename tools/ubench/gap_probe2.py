"""Clock spin-up and per-frame overhead of events / step counting."""
import math
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

import schwarzschild_raytracer_wgpu_amd as g  # noqa: E402
from schwarzschild_raytracer_wgpu_amd.scenes import make_sky  # noqa: E402
from schwarzschild_raytracer_wgpu_amd.timing import HipEvent, hipEventDefault  # noqa: E402

W, H = 3840, 2160
o = g.Observer(1.0, math.pi / 2, W, H)
o.set_position(2.5, 0.0, 0.1)
fr = o.calc_transformation_pipeline()
sc = g.make_scene(1.0, 50.0, o.get_radial_position(), math.pi / 100, 2048)
scd = g.make_scene(1.0, 50.0, o.get_radial_position(), math.pi / 100, 2048, flags=g._lib.GEO_FLAG_DEFER_STEPS)
ctx = g.Context(0)
ctx.set_sky(make_sky("equirect", (4096, 2048)))
dev = torch.device("cuda:0")
out = torch.empty(W * H * 4, dtype=torch.uint8, device=dev)
ctr = torch.zeros(1, dtype=torch.int64, device=dev)
stream = torch.cuda.current_stream().cuda_stream

# spin-up curve from idle: per-frame kernel time of the first 400 frames
time.sleep(2.0)
evs = [(HipEvent(), HipEvent()) for _ in range(400)]
for i in range(400):
    evs[i][0].record()
    ctx.render_bands(fr, sc, W, H, 8, 0, 1, H // 8, out, stream=stream)
    evs[i][1].record()
torch.cuda.synchronize()
ks = [a.elapsed_time(b) for a, b in evs]
for lo in (0, 5, 10, 20, 50, 100, 200, 300, 390):
    print(f"frame {lo:3d}: {ks[lo]:.4f} ms")


def run(K, kind, counter):
    ev = [(HipEvent(hipEventDefault if kind == "default" else 0x20000000),
           HipEvent(hipEventDefault if kind == "default" else 0x20000000)) for _ in range(K)]
    tev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * K)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        if kind == "torch":
            tev[2 * i].record()
        elif kind != "none":
            ev[i][0].record()
        if counter == "defer":
            ctx.render_bands(fr, scd, W, H, 8, 0, 1, H // 8, out, stream=stream)
        else:
            ctx.render_bands(fr, sc, W, H, 8, 0, 1, H // 8, out, steps_total=ctr if counter == "fold" else None,
                             stream=stream)
        if kind == "torch":
            tev[2 * i + 1].record()
        elif kind != "none":
            ev[i][1].record()
    if counter == "defer":
        ctx.steps_flush(ctr)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / K * 1e3
    if kind == "torch":
        k = sum(tev[2 * i].elapsed_time(tev[2 * i + 1]) for i in range(K)) / K
    elif kind != "none":
        k = sum(a.elapsed_time(b) for a, b in ev) / K
    else:
        k = float("nan")
    return dt, k


for rep in range(2):
    for kind in ("none", "torch", "default", "nofence"):
        for counter in ("off", "fold", "defer"):
            dt, k = run(200, kind, counter)
            print(f"rep{rep} events={kind:8s} counter={counter:5s}: {dt:.4f} ms/frame  kernel-event avg {k:.4f}")
