"""The rank-0 side of the multi-GPU frame pipeline (dist.ShardedFrame with
the RCCL path: batched async gathers, reassembly on a side stream ordered by
events) on ONE GPU: RCCL cannot put two ranks on one device ("Duplicate GPU
detected"), so the peer ranks are simulated by a gather stand-in with NCCL's
stream semantics (the copy runs on its own stream after the caller's stream;
wait() makes the caller's current stream wait).  Peer data = the peers'
bands rendered here with geo_render_band_set (plain and lead layouts)."""
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


def _peer_bands(ctx, torch, frame, scene, W, H, B, r, world, lead, dev, bpp, pb=1):
    """Peer r's packed bands in the travelling format, padded to rank 1's size."""
    from schwarzschild_raytracer_wgpu_amd.dist import BandLayout

    L = BandLayout(H, B, world, r, lead, pb)
    sl = L.peer_packed_rows * W * 4
    one = torch.zeros(sl, dtype=torch.uint8, device=dev)
    if L.nbands():
        ctx.render_band_set(frame, scene, W, H, L.band_height(), L.row0(), L.cycle_rows, L.nbands(), one)
    if bpp == 3:
        packed = torch.empty(sl // 4 * 3, dtype=torch.uint8, device=dev)
        ctx.pack_rgb(one, sl // 4, packed)
        one = packed
    return one


@pytest.mark.parametrize("batch", [False, True], ids=["per-frame", "batched"])
@pytest.mark.parametrize("rgb", [True, False], ids=["rgb24", "rgba8"])
@pytest.mark.parametrize("S", [1, 2])
@pytest.mark.parametrize("world,K,nframes,lead", [(2, 4, 41, 1), (3, 3, 10, 1), (8, 4, 16, 1), (8, 1, 5, 1),
                                                  (2, 4, 13, 2), (2, 2, 7, 4), (4, 3, 10, 2), (8, 4, 9, 2),
                                                  (8, 2, 6, 4), (2, 3, 8, 3), (8, 4, 9, 3), (4, 2, 5, 6),
                                                  (8, 4, 9, (3, 2)), (4, 3, 7, (5, 2)), (2, 2, 5, (3, 2)),
                                                  (4, 4, 9, (3, 2))])
def test_rank0_pipeline_assembles_frames(world, K, nframes, lead, S, rgb, batch):
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
    lead, pb = lead if isinstance(lead, tuple) else (lead, 1)  # (rank 0's bands, a peer's bands) per cycle
    sf = ShardedFrame(ctx, frame, scene, W, H, B, 0, world, dev, dist=fake, frames_per_gather=K, render_streams=S,
                      present_rgb=rgb, lead=lead, batch_launch=batch, peer_bands=pb)
    assert sf.batch == (batch and K > 1)
    assert sf.side is not None and sf.bpp == (3 if rgb else 4) and sf.layout.lead == lead
    # the peers' K-frame batches (every frame identical), in the travelling format
    for r in range(1, world):
        fake.peer_bufs.append(_peer_bands(ctx, torch, frame, scene, W, H, B, r, world, lead, dev, sf.bpp,
                                          pb).repeat(K))
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


@pytest.mark.parametrize("batch", [False, True], ids=["per-frame", "batched"])
@pytest.mark.parametrize("lead", [1, 2, 3])
@pytest.mark.parametrize("S", [1, 2])
def test_peer_rank_pipeline_runs_batches(S, lead, batch):
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
    sf = ShardedFrame(ctx, frame, scene, W, H, B, rank, world, dev, dist=pg, frames_per_gather=K, render_streams=S,
                      lead=lead, batch_launch=batch)
    for i in range(10):
        sf.step(i)
    sf.drain()
    torch.cuda.synchronize()
    assert len(pg.sent) == 3 and sf.frames_done == 10
    L = BandLayout(H, B, world, rank, lead)
    one = _peer_bands(ctx, torch, frame, scene, W, H, B, rank, world, lead, dev, sf.bpp)
    torch.cuda.synchronize()
    assert pg.sent[0].numel() == K * one.numel()  # every contribution has rank 1's size
    used = L.nbands() * B * W * sf.bpp  # rows past the rank's last band are never written
    for j, batch in enumerate(pg.sent):
        for k in range(K if j < 2 else 10 - 2 * K):
            assert torch.equal(batch[k * one.numel():k * one.numel() + used], one[:used]), (j, k)


@pytest.mark.parametrize("W,H,B,world,lead,bpp,nframes", [
    (320, 180, 8, 2, 2, 3, 3), (320, 180, 8, 8, 4, 4, 2), (36, 50, 8, 3, 2, 3, 1), (33, 27, 8, 2, 4, 4, 2),
    (64, 64, 16, 4, 1, 3, 2), (20, 8, 8, 3, 2, 4, 1), (320, 180, 8, 8, 3, 3, 2), (36, 50, 8, 2, 6, 4, 1),
    (320, 180, 8, 8, (3, 2), 3, 2), (36, 90, 8, 3, (5, 2), 4, 2), (33, 60, 8, 2, (3, 2), 4, 1),
    (64, 100, 8, 4, (1, 2), 3, 1)])
def test_assemble_lead_matches_host_assembly(W, H, B, world, lead, bpp, nframes):
    """geo_assemble_lead on random bytes == dist.assemble (the host reassembly
    the gloo tests check against the oracle), RGB24 and RGBA8 peers, widths
    that are and are not multiples of 4, frames with empty peer shares; with
    a (lead, peer_bands) pair, geo_assemble_shares with rank 0's rows per
    cycle not a multiple of a peer's band."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import schwarzschild_raytracer_wgpu_amd as g
    from schwarzschild_raytracer_wgpu_amd.dist import BandLayout, assemble

    dev = torch.device("cuda:0")
    ctx = g.Context(0)
    lead, pb = lead if isinstance(lead, tuple) else (lead, 1)
    L = BandLayout(H, B, world, 0, lead, pb)
    gen = torch.Generator().manual_seed(W * 7919 + H * 31 + world * 7 + lead * 3 + pb)
    own_sl = L.packed_rows(0) * W * 4
    own_sl += (-own_sl) % 16
    tsl = L.peer_packed_rows * W * bpp
    tsl += (-tsl) % 16
    own = torch.randint(0, 256, (nframes * own_sl,), dtype=torch.uint8, generator=gen)
    peers = torch.randint(0, 256, (world * nframes * max(tsl, 1),), dtype=torch.uint8, generator=gen)
    out = torch.full((nframes * H * W * 4,), 7, dtype=torch.uint8, device=dev)
    if pb == 1:
        ctx.assemble_lead(own.to(dev), own_sl, lead, peers.to(dev), nframes * tsl, tsl, world, B, W, H, nframes, out,
                          src_bpp=bpp)
    else:
        ctx.assemble_shares(own.to(dev), own_sl, lead * B, peers.to(dev), nframes * tsl, tsl, world, pb * B, W, H,
                            nframes, out, src_bpp=bpp)
    torch.cuda.synchronize()
    got = out.cpu()
    for f in range(nframes):
        # host reference: RGBA8 blocks per rank (RGB24 peers widened, alpha 255)
        blocks = [own]
        for r in range(1, world):
            blk = peers[r * nframes * tsl:(r + 1) * nframes * tsl]
            if bpp == 3:
                px = blk.view(nframes, tsl)[:, :L.peer_packed_rows * W * 3].reshape(nframes, -1, 3)
                rgba = torch.cat([px, torch.full(px.shape[:2] + (1,), 255, dtype=torch.uint8)], dim=2)
                blk = rgba.reshape(-1)
            blocks.append(blk)
        peer_stride = L.peer_packed_rows * W * 4 if bpp == 3 else tsl
        ref = torch.zeros(H * W * 4, dtype=torch.uint8)
        assemble(ref, blocks, L, W * 4, frame=f, frame_stride=[own_sl] + [peer_stride] * (world - 1))
        assert torch.equal(got[f * H * W * 4:(f + 1) * H * W * 4], ref), f


@pytest.mark.parametrize("S", [1, 2])
def test_batch_splits_on_scene_change(S):
    """Batch mode, a peer rank: a launch's frames may differ in the observer
    radius (one geo_render_band_set_batch launch), but a step whose scene
    differs otherwise (here the step budget) renders the pending frames
    first (into their slots), and the batch's gather still sends all K
    frames; every sent frame equals that frame's own render with its own
    scene."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import schwarzschild_raytracer_wgpu_amd as g
    from schwarzschild_raytracer_wgpu_amd.dist import ShardedFrame
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    class PeerGather:
        def __init__(self):
            self.stream = torch.cuda.Stream()
            self.sent = []

        def gather(self, src, gather_list=None, dst=0, async_op=True):
            ready = torch.cuda.Event()
            ready.record(torch.cuda.current_stream())
            with torch.cuda.stream(self.stream):
                self.stream.wait_event(ready)
                self.sent.append(src.clone())
                done = torch.cuda.Event()
                done.record(self.stream)
            return _Work(torch, done)

    W, H, B, world, rank, K = 256, 144, 8, 2, 1, 4
    dev = torch.device("cuda:0")
    ctx = g.Context(0)
    ctx.set_sky(make_sky("equirect", (128, 64)))
    poses = []
    for r, budget in ((2.5, 256), (3.4, 256), (2.9, 200)):
        obs = g.Observer(1.0, math.pi / 2, W, H)
        obs.set_position(r, 0.0, 0.1)
        rr = obs.get_radial_position()
        poses.append((obs.calc_transformation_pipeline(),
                      g.make_scene(1.0, 50.0, rr, math.pi / 100, budget, g.GEO_MODE_DIRECT)))
    # radius changes inside every batch; budget changes inside batches 0 and 2 (splits), none in batch 1
    which = [0, 2, 1, 0, 1, 0, 1, 1, 0, 2]
    pg = PeerGather()
    sf = ShardedFrame(ctx, poses[0][0], poses[0][1], W, H, B, rank, world, dev, dist=pg, frames_per_gather=K,
                      render_streams=S, batch_launch=True)
    assert sf.batch and sf.bpp == 3
    for i, p in enumerate(which):
        sf.step(i, frame=poses[p][0], scene=poses[p][1])
    sf.drain()
    torch.cuda.synchronize()
    assert len(pg.sent) == 3 and sf.frames_done == len(which)
    L = sf.layout
    ref = []
    assert len({bytes(p[1]) for p in poses}) == 3
    for frame, scene in poses:
        one = torch.zeros(sf.slice, dtype=torch.uint8, device=dev)
        ctx.render_band_set(frame, scene, W, H, L.band_height(), L.row0(), L.cycle_rows, L.nbands(), one)
        packed = torch.empty(sf.tslice, dtype=torch.uint8, device=dev)
        ctx.pack_rgb(one, sf.slice // 4, packed)
        ref.append(packed)
    torch.cuda.synchronize()
    assert not torch.equal(ref[0], ref[1]) and not torch.equal(ref[0], ref[2])
    for i, p in enumerate(which):
        batch = pg.sent[i // K]
        got = batch[(i % K) * sf.tslice:(i % K + 1) * sf.tslice]
        assert torch.equal(got, ref[p]), i


@pytest.mark.parametrize("S", [1, 2])
def test_batch_snapshots_uniforms_mutated_in_place(S):
    """Batch mode reads a batch's uniforms when it launches, K steps after
    the first was recorded: ShardedFrame must copy them at each step.  One
    GeoFrame object and one GeoScene object are updated in place before every
    step (the pose alternates; the scene's step budget changes once, inside a
    batch); every frame sent equals that step's own render."""
    import ctypes

    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import schwarzschild_raytracer_wgpu_amd as g
    from schwarzschild_raytracer_wgpu_amd.dist import ShardedFrame
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    class PeerGather:
        def __init__(self):
            self.stream = torch.cuda.Stream()
            self.sent = []

        def gather(self, src, gather_list=None, dst=0, async_op=True):
            ready = torch.cuda.Event()
            ready.record(torch.cuda.current_stream())
            with torch.cuda.stream(self.stream):
                self.stream.wait_event(ready)
                self.sent.append(src.clone())
                done = torch.cuda.Event()
                done.record(self.stream)
            return _Work(torch, done)

    W, H, B, world, rank, K = 256, 144, 8, 2, 1, 4
    dev = torch.device("cuda:0")
    ctx = g.Context(0)
    ctx.set_sky(make_sky("equirect", (128, 64)))
    poses = [default_frame(W, H, pos=p) for p in ((2.5, 0.0, 0.1), (3.4, 0.2, 0.0))]
    scenes = [default_scene(256), default_scene(200)]
    fr = g.GeoFrame.from_buffer_copy(poses[0])
    sc = g.GeoScene.from_buffer_copy(scenes[0])
    plan = [(0, 0), (1, 0), (0, 0), (1, 0), (1, 0), (0, 1), (1, 1), (0, 1), (1, 1), (0, 0)]
    pg = PeerGather()
    sf = ShardedFrame(ctx, fr, sc, W, H, B, rank, world, dev, dist=pg, frames_per_gather=K, render_streams=S,
                      batch_launch=True)
    assert sf.batch
    for i, (p, s) in enumerate(plan):
        ctypes.memmove(ctypes.addressof(fr), ctypes.addressof(poses[p]), ctypes.sizeof(fr))
        ctypes.memmove(ctypes.addressof(sc), ctypes.addressof(scenes[s]), ctypes.sizeof(sc))
        sf.step(i, frame=fr if i % 2 else None, scene=sc if i % 3 else None)  # explicit and the object's own
    sf.drain()
    torch.cuda.synchronize()
    assert len(pg.sent) == 3 and sf.frames_done == len(plan)
    L = sf.layout
    for i, (p, s) in enumerate(plan):
        one = torch.zeros(sf.slice, dtype=torch.uint8, device=dev)
        ctx.render_band_set(poses[p], scenes[s], W, H, L.band_height(), L.row0(), L.cycle_rows, L.nbands(), one)
        ref = torch.empty(sf.tslice, dtype=torch.uint8, device=dev)
        ctx.pack_rgb(one, sf.slice // 4, ref)
        torch.cuda.synchronize()
        got = pg.sent[i // K][(i % K) * sf.tslice:(i % K + 1) * sf.tslice]
        assert torch.equal(got, ref), i


def test_timed_step_of_a_rank_without_rows():
    """A rank whose share of a tiny frame is empty still records the caller's
    timing pair (zero length), per frame and batched."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import schwarzschild_raytracer_wgpu_amd as g
    from schwarzschild_raytracer_wgpu_amd.dist import ShardedFrame
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky
    from schwarzschild_raytracer_wgpu_amd.timing import HipEvent

    class Sink:
        def gather(self, src, gather_list=None, dst=0, async_op=True):
            return _Work(torch, torch.cuda.Event())

    W, H = 64, 16  # two 8-row bands: ranks 2 and 3 of 4 own none
    dev = torch.device("cuda:0")
    ctx = g.Context(0)
    ctx.set_sky(make_sky("equirect", (128, 64)))
    for batch in (False, True):
        sf = ShardedFrame(ctx, default_frame(W, H), default_scene(64), W, H, 8, 3, 4, dev, dist=Sink(),
                          frames_per_gather=2, batch_launch=batch)
        assert sf.layout.nbands() == 0
        ev = (HipEvent(), HipEvent())
        sf.step(0)
        sf.step(1, events=ev)
        sf.drain()
        torch.cuda.synchronize()
        assert 0.0 <= ev[0].elapsed_time(ev[1]) < 1.0


@pytest.mark.parametrize("world,K,lead", [(2, 4, 1), (4, 3, (3, 2)), (8, 2, 2)])
def test_rank0_pipeline_ring_f64(world, K, lead):
    """GEO_FLAG_RING_F64 through the multi-GPU pipeline (bench.py --ring-f64
    at N > 1): each frame's bands in their own launch, and each batch's frames
    in one launch, with the capture band in f64; rank 0's assembled frames
    equal the single-launch ring frame byte for byte (the band's pixels are
    per pixel, whatever the band layout, batch or dispatch order)."""
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
    scene.flags |= g._lib.GEO_FLAG_RING_F64
    plain = g.GeoScene.from_buffer_copy(bytes(scene))
    plain.flags &= ~g._lib.GEO_FLAG_RING_F64
    # the ring frame differs from the plain one (the band is in the frame:
    # its lanes' lambda', so their UV bits)
    uv_ring = torch.empty(H * W * 2, dtype=torch.float32, device=dev)
    uv_plain = torch.empty(H * W * 2, dtype=torch.float32, device=dev)
    ref = torch.empty(H * W * 4, dtype=torch.uint8, device=dev)
    tmp = torch.empty(H * W * 4, dtype=torch.uint8, device=dev)
    ctx.render_rows(frame, scene, W, H, 0, H, ref, out_uv=uv_ring)
    ctx.render_rows(frame, plain, W, H, 0, H, tmp, out_uv=uv_plain)
    torch.cuda.synchronize()
    assert int((uv_ring != uv_plain).sum().item()) > 0
    fake = FakeRcclGather(torch, [])
    lead, pb = lead if isinstance(lead, tuple) else (lead, 1)
    sf = ShardedFrame(ctx, frame, scene, W, H, B, 0, world, dev, dist=fake, frames_per_gather=K, render_streams=2,
                      present_rgb=True, lead=lead, batch_launch=False, peer_bands=pb)
    assert not sf.batch
    for r in range(1, world):
        fake.peer_bufs.append(_peer_bands(ctx, torch, frame, scene, W, H, B, r, world, lead, dev, sf.bpp,
                                          pb).repeat(K))
    nframes = 2 * K + 1
    for i in range(nframes):
        sf.step(i)
    sf.drain()
    torch.cuda.synchronize()
    assert torch.equal(sf.frame_rgba(), ref)
    # batched: each batch's frames in one launch, the same frames
    fake2 = FakeRcclGather(torch, fake.peer_bufs)
    sf2 = ShardedFrame(ctx, frame, scene, W, H, B, 0, world, dev, dist=fake2, frames_per_gather=K, render_streams=2,
                       present_rgb=True, lead=lead, batch_launch=True, peer_bands=pb)
    assert sf2.batch == (K > 1)
    for i in range(nframes):
        sf2.step(i)
    sf2.drain()
    torch.cuda.synchronize()
    assert torch.equal(sf2.frame_rgba(), ref)
    last_n = nframes - (math.ceil(nframes / K) - 1) * K
    for k in range(last_n):
        assert torch.equal(sf2.frame_rgba(k), ref), k
