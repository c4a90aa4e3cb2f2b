"""Config 4 (BASELINE.json configs[3]): the 3840x2160 / 2048-step frame
row-sharded over 8 ranks and gathered to rank 0 for present, on ONE GPU.

1. The workload itself: the eight band sets of BandLayout(2160, 8, 8, r)
   rendered as the eight ranks would (geo_render_band_set, the peers packed
   to RGB24 with geo_pack_rgb), laid out as rank 0's gather receives them and
   reassembled with geo_assemble_shares exactly as ShardedFrame._assemble
   calls it; the frame must equal a single-launch geo_render_rows frame byte
   for byte, and that frame's sampled rows equal the oracle bit for bit.
   The default 1:1 share and an a:b share (3:2) are both covered.

2. The RCCL API path: a 1-rank `nccl` process group (RCCL cannot put two
   ranks on one device, "Duplicate GPU detected"), and ShardedFrame driven as
   rank 0 (and as a peer) of an 8-rank layout whose gather goes through real
   dist.gather(async_op=True) calls on RCCL's stream.  ShardedFrame issues the
   gather from its gather stream after its render events and retires it with
   work.wait() on the reassembly stream (dist.py _launch/_retire); the
   loopback below turns one W-rank gather into W one-rank RCCL gathers, one
   per block of the receive list, so the stream semantics under test are
   RCCL's own.  Reference: the per-frame present loop renderer.rs:208-283,
   sharded per SURVEY.md §8e.
"""
import datetime
import socket

import numpy as np
import pytest

import oracle as O
from helpers import default_frame, default_scene

pytestmark = pytest.mark.gpu

W, H, BAND, WORLD, STEPS = 3840, 2160, 8, 8, 2048


@pytest.fixture(scope="module")
def env():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import schwarzschild_raytracer_wgpu_amd as g
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    dev = torch.device("cuda:0")
    sky = make_sky("equirect", (4096, 2048))
    ctx = g.Context(0)
    ctx.set_sky(sky)
    frame, scene = default_frame(W, H), default_scene(STEPS)
    ref = torch.empty(H * W * 4, dtype=torch.uint8, device=dev)
    ctx.render_rows(frame, scene, W, H, 0, H, ref)
    torch.cuda.synchronize()
    return dict(torch=torch, g=g, dev=dev, sky=sky, ctx=ctx, frame=frame, scene=scene, ref=ref)


def test_cfg4_single_launch_frame_matches_oracle_rows(env):
    """The reference frame the shard tests compare against: sampled rows
    bit-exact against the oracle (RGBA; the mask/UV/steps of these rows are
    covered by test_gpu_parity.test_4k_2048_properties)."""
    row0, step = 5, 67
    ref = O.render_f32(env["frame"], env["scene"], env["sky"], W, H, row0=row0, nrows=(H - row0 + step - 1) // step,
                       row_step=step, threads=16)
    got = env["ref"].view(H, W, 4).cpu().numpy()[row0::step]
    assert np.array_equal(got, ref["rgba"])


def _peer_block(env, L, bpp):
    """One rank's packed bands, as it sends them (RGB24 or RGBA8), padded to rank 1's share."""
    torch, ctx = env["torch"], env["ctx"]
    sl = L.peer_packed_rows * W * 4
    one = torch.zeros(sl, dtype=torch.uint8, device=env["dev"])
    if L.nbands():
        ctx.render_band_set(env["frame"], env["scene"], W, H, L.band_height(), L.row0(), L.cycle_rows, L.nbands(), one)
    if bpp == 4:
        return one
    packed = torch.empty(sl // 4 * 3, dtype=torch.uint8, device=env["dev"])
    ctx.pack_rgb(one, sl // 4, packed)
    return packed


@pytest.mark.parametrize("bpp", [3, 4], ids=["rgb24", "rgba8"])
@pytest.mark.parametrize("share", [(1, 1), (3, 2)], ids=["1:1", "3:2"])
def test_cfg4_eight_band_sets_assemble_to_the_frame(env, share, bpp):
    torch, ctx, dev = env["torch"], env["ctx"], env["dev"]
    from schwarzschild_raytracer_wgpu_amd.dist import BandLayout

    lead, pb = share
    layouts = [BandLayout(H, BAND, WORLD, r, lead, pb) for r in range(WORLD)]
    # every frame row is owned by exactly one rank
    owned = sorted(x for L in layouts for x in L.local_to_frame_rows() if x >= 0)
    assert owned == list(range(H))
    L0 = layouts[0]
    own = torch.zeros(L0.packed_rows(0) * W * 4, dtype=torch.uint8, device=dev)
    ctx.render_band_set(env["frame"], env["scene"], W, H, L0.band_height(), L0.row0(), L0.cycle_rows, L0.nbands(), own)
    tslice = L0.peer_packed_rows * W * bpp
    recv = torch.full((WORLD * tslice,), 0xA5, dtype=torch.uint8, device=dev)  # block 0 is never read
    for r in range(1, WORLD):
        recv[r * tslice:(r + 1) * tslice].copy_(_peer_block(env, layouts[r], bpp))
    out = torch.full((H * W * 4,), 7, dtype=torch.uint8, device=dev)
    ctx.assemble_shares(own, own.numel(), L0.band_height(0), recv, tslice, tslice, WORLD, L0.band_height(1), W, H, 1,
                        out, src_bpp=bpp)
    torch.cuda.synchronize()
    assert torch.equal(out, env["ref"])


class _Works:
    def __init__(self, works):
        self.works = works

    def wait(self):
        for w in self.works:
            w.wait()


class RcclLoopback:
    """dist.gather for one rank of a `world`-rank layout over a 1-rank RCCL
    group.  Rank 0: block 0 of the receive list comes from its own send
    buffer, block r (r >= 1) from peer_bufs[r - 1], each by one RCCL gather
    (the peer's bytes were rendered on this device beforehand).  A peer: the
    send buffer is gathered into a fresh capture tensor, kept in `sent`."""

    def __init__(self, dist, peer_bufs=()):
        self.dist, self.peer_bufs = dist, list(peer_bufs)
        self.sent, self.calls = [], 0

    def gather(self, src, gather_list=None, dst=0, async_op=True):
        import torch

        assert dst == 0 and async_op
        self.calls += 1
        if gather_list is None:  # a peer's send
            cap = torch.empty_like(src)
            self.sent.append(cap)
            return self.dist.gather(src, gather_list=[cap], dst=0, async_op=True)
        works = [self.dist.gather(src, gather_list=[gather_list[0]], dst=0, async_op=True)]
        for r, pb in enumerate(self.peer_bufs, start=1):
            works.append(self.dist.gather(pb, gather_list=[gather_list[r]], dst=0, async_op=True))
        return _Works(works)


@pytest.fixture(scope="module")
def rccl(env):
    import torch.distributed as dist

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=env["dev"], timeout=datetime.timedelta(seconds=60))
    assert dist.get_backend() == "nccl"
    yield dist
    dist.destroy_process_group()


def test_rccl_one_rank_gather_is_stream_ordered(env, rccl):
    """The bare API: an async gather launched on a side stream after a
    producer kernel, retired with work.wait() on another stream, reads what
    the producer wrote and is read by what follows the wait."""
    torch, dev = env["torch"], env["dev"]
    prod, gs, cons = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    src = torch.empty(1 << 24, dtype=torch.uint8, device=dev)
    dst = torch.zeros_like(src)
    with torch.cuda.stream(prod):
        torch.cuda._sleep(2_000_000)  # the gather must wait for this stream's work
        src.fill_(0x3C)
        ev = torch.cuda.Event()
        ev.record(prod)
    with torch.cuda.stream(gs):
        gs.wait_event(ev)
        work = rccl.gather(src, gather_list=[dst], dst=0, async_op=True)
    with torch.cuda.stream(cons):
        work.wait()
        total = dst.to(torch.int64).sum()
    torch.cuda.synchronize()
    assert int(total) == 0x3C * src.numel()


@pytest.mark.parametrize("batch", [False, True], ids=["per-frame", "batched"])
@pytest.mark.parametrize("S,K,nframes,share", [(2, 2, 5, (1, 1)), (2, 4, 9, (3, 2)), (1, 1, 3, (1, 1))])
def test_cfg4_rank0_pipeline_over_rccl(env, rccl, S, K, nframes, share, batch):
    """ShardedFrame as rank 0 of config 4 (8 ranks, RGB24 peers) with its
    gathers on RCCL: every assembled frame of the last batch equals the
    single-launch frame."""
    torch, ctx, dev = env["torch"], env["ctx"], env["dev"]
    from schwarzschild_raytracer_wgpu_amd.dist import BandLayout, ShardedFrame

    lead, pb = share
    peers = [_peer_block(env, BandLayout(H, BAND, WORLD, r, lead, pb), 3).repeat(K) for r in range(1, WORLD)]
    lb = RcclLoopback(rccl, peers)
    sf = ShardedFrame(ctx, env["frame"], env["scene"], W, H, BAND, 0, WORLD, dev, dist=lb, frames_per_gather=K,
                      render_streams=S, lead=lead, peer_bands=pb, batch_launch=batch)
    assert sf.gstream is not None and sf.side is not None and sf.bpp == 3
    for i in range(nframes):
        sf.step(i)
    sf.drain()
    torch.cuda.synchronize()
    assert lb.calls == -(-nframes // K) and sf.frames_done == nframes
    last_n = nframes - (lb.calls - 1) * K
    for k in range(last_n):
        assert torch.equal(sf.frame_rgba(k), env["ref"]), k


@pytest.mark.parametrize("batch", [False, True], ids=["per-frame", "batched"])
def test_cfg4_peer_pipeline_over_rccl(env, rccl, batch):
    """ShardedFrame as peer rank 5 of config 4: every frame it sends through
    RCCL is its RGB24 band set, and a batch buffer is re-rendered only after
    its gather read it (two batch buffers, 3 batches)."""
    torch, ctx, dev = env["torch"], env["ctx"], env["dev"]
    from schwarzschild_raytracer_wgpu_amd.dist import BandLayout, ShardedFrame

    K, nframes, rank = 3, 8, 5
    lb = RcclLoopback(rccl)
    sf = ShardedFrame(ctx, env["frame"], env["scene"], W, H, BAND, rank, WORLD, dev, dist=lb, frames_per_gather=K,
                      render_streams=2, batch_launch=batch)
    for i in range(nframes):
        sf.step(i)
    sf.drain()
    torch.cuda.synchronize()
    assert len(lb.sent) == 3 and sf.frames_done == nframes
    one = _peer_block(env, BandLayout(H, BAND, WORLD, rank), 3)
    torch.cuda.synchronize()
    n = one.numel()
    for j, blk in enumerate(lb.sent):
        for k in range(K if j < 2 else nframes - 2 * K):
            assert torch.equal(blk[k * n:(k + 1) * n], one), (j, k)
