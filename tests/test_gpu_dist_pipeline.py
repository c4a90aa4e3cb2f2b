"""The rank-0 side of the multi-GPU frame pipeline (dist.ShardedFrame with
the RCCL path: batched async gathers, reassembly on a side stream ordered by
events) on ONE GPU: RCCL cannot put two ranks on one device ("Duplicate GPU
detected"), so the peer ranks are simulated by a gather stand-in with NCCL's
stream semantics (the copy runs on its own stream after the caller's stream;
wait() makes the caller's current stream wait).  Peer data = the peers'
bands rendered here with geo_render_bands."""
import math

import numpy as np
import pytest

from helpers import default_frame, default_scene

pytestmark = pytest.mark.gpu


class _Work:
    def __init__(self, torch, ev):
        self.torch, self.ev = torch, ev

    def wait(self):
        self.torch.cuda.current_stream().wait_event(self.ev)


class FakeRcclGather:
    """dist.gather(src, gather_list, dst=0, async_op=True) for rank 0 of a
    `world`-rank group whose peers hold `peer_bufs` (device tensors)."""

    def __init__(self, torch, peer_bufs):
        self.torch, self.peer_bufs = torch, peer_bufs
        self.stream = torch.cuda.Stream()
        self.calls = 0

    def gather(self, src, gather_list=None, dst=0, async_op=True):
        t = self.torch
        ready = t.cuda.Event()
        ready.record(t.cuda.current_stream())
        with t.cuda.stream(self.stream):
            self.stream.wait_event(ready)
            gather_list[0].copy_(src, non_blocking=True)
            for r, pb in enumerate(self.peer_bufs, start=1):
                gather_list[r].copy_(pb, non_blocking=True)
            done = t.cuda.Event()
            done.record(self.stream)
        self.calls += 1
        return _Work(t, done)


@pytest.mark.parametrize("rgb", [True, False], ids=["rgb24", "rgba8"])
@pytest.mark.parametrize("S", [1, 2])
@pytest.mark.parametrize("world,K,nframes", [(2, 4, 41), (3, 3, 10), (8, 4, 16), (8, 1, 5)])
def test_rank0_pipeline_assembles_frames(world, K, nframes, S, rgb):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import schwarzschild_raytracer_wgpu_amd as g
    from schwarzschild_raytracer_wgpu_amd.dist import BandLayout, ShardedFrame
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    W, H, B = 320, 180, 8
    dev = torch.device("cuda:0")
    ctx = g.Context(0)
    ctx.set_sky(make_sky("equirect", (256, 128)))
    frame, scene = default_frame(W, H), default_scene(512)
    fake = FakeRcclGather(torch, [])
    sf = ShardedFrame(ctx, frame, scene, W, H, B, 0, world, dev, dist=fake, frames_per_gather=K, render_streams=S,
                      present_rgb=rgb)
    assert sf.side is not None and sf.bpp == (3 if rgb else 4)
    # the peers' K-frame batches (every frame identical), in the travelling format
    for r in range(1, world):
        L = BandLayout(H, B, world, r)
        sl = L.nb_max * B * W * 4
        one = torch.zeros(sl, dtype=torch.uint8, device=dev)
        if L.nb_mine:
            ctx.render_bands(frame, scene, W, H, B, r, world, L.nb_mine, one)
        if sf.bpp == 3:
            packed = torch.empty(sl // 4 * 3, dtype=torch.uint8, device=dev)
            ctx.pack_rgb(one, sl // 4, packed)
            one = packed
        fake.peer_bufs.append(one.repeat(K))
    for i in range(nframes):
        sf.step(i)
    sf.drain()
    torch.cuda.synchronize()
    assert fake.calls == math.ceil(nframes / K)
    assert sf.frames_done == nframes
    ref = torch.empty(H * W * 4, dtype=torch.uint8, device=dev)
    ctx.render_rows(frame, scene, W, H, 0, H, ref)
    torch.cuda.synchronize()
    assert torch.equal(sf.frame_rgba(), ref)
    # every frame slot of the last (possibly partial) batch was assembled
    last_n = nframes - (math.ceil(nframes / K) - 1) * K
    for k in range(last_n):
        assert torch.equal(sf.frame_rgba(k), ref), k


@pytest.mark.parametrize("S", [1, 2])
def test_peer_rank_pipeline_runs_batches(S):
    """A peer rank (rank 3 of 4): batches of K frames, each sent with one
    gather; the send buffer is re-rendered only after its gather completed."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import schwarzschild_raytracer_wgpu_amd as g
    from schwarzschild_raytracer_wgpu_amd.dist import BandLayout, ShardedFrame
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    class PeerGather:
        def __init__(self):
            self.stream = torch.cuda.Stream()
            self.sent = []

        def gather(self, src, gather_list=None, dst=0, async_op=True):
            assert gather_list is None and dst == 0
            ready = torch.cuda.Event()
            ready.record(torch.cuda.current_stream())
            with torch.cuda.stream(self.stream):
                self.stream.wait_event(ready)
                self.sent.append(src.clone())
                done = torch.cuda.Event()
                done.record(self.stream)
            return _Work(torch, done)

    W, H, B, world, rank, K = 256, 144, 8, 4, 3, 4
    dev = torch.device("cuda:0")
    ctx = g.Context(0)
    ctx.set_sky(make_sky("equirect", (128, 64)))
    frame, scene = default_frame(W, H), default_scene(256)
    pg = PeerGather()
    sf = ShardedFrame(ctx, frame, scene, W, H, B, rank, world, dev, dist=pg, frames_per_gather=K, render_streams=S)
    for i in range(10):
        sf.step(i)
    sf.drain()
    torch.cuda.synchronize()
    assert len(pg.sent) == 3 and sf.frames_done == 10
    L = BandLayout(H, B, world, rank)
    one = torch.zeros(L.nb_max * B * W * 4, dtype=torch.uint8, device=dev)
    ctx.render_bands(frame, scene, W, H, B, rank, world, L.nb_mine, one)
    torch.cuda.synchronize()
    if sf.bpp == 3:
        packed = torch.empty(one.numel() // 4 * 3, dtype=torch.uint8, device=dev)
        ctx.pack_rgb(one, one.numel() // 4, packed)
        torch.cuda.synchronize()
        one = packed
    used = L.nb_mine * B * W * sf.bpp  # rows past the rank's last band are never written
    for j, batch in enumerate(pg.sent):
        for k in range(K if j < 2 else 10 - 2 * K):
            assert torch.equal(batch[k * one.numel():k * one.numel() + used], one[:used]), (j, k)
