"""Multi-rank row-band sharding + gather to rank 0, on CPU with gloo.

Each rank renders ITS interleaved bands (schwarzschild_raytracer_wgpu_amd.dist
.BandLayout) with the CPU oracle into a packed local buffer, rank 0 gathers
and reassembles with dist.assemble, and the frame must equal the oracle's
single-rank frame byte for byte.  The GPU path uses the same layout/assemble
code with geo_render_bands and RCCL (bench.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from schwarzschild_raytracer_wgpu_amd.dist import BandLayout, assemble


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, W, H, B, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle as O
        from helpers import default_frame, default_scene
        from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

        sky = make_sky("equirect", (64, 32))
        frame, scene = default_frame(W, H), default_scene(256)
        L = BandLayout(H, B, world, rank)
        row_bytes = W * 4
        local = torch.zeros(L.nb_max * B * row_bytes, dtype=torch.uint8)
        lv = local.view(L.nb_max * B, row_bytes)
        for i, fr in enumerate(L.local_to_frame_rows()):
            if fr >= 0:
                r = O.render_f32(frame, scene, sky, W, H, row0=fr, nrows=1, threads=1)
                lv[i] = torch.from_numpy(r["rgba"].reshape(-1).copy())
        gl = [torch.empty_like(local) for _ in range(world)] if rank == 0 else None
        dist.gather(local, gather_list=gl, dst=0)
        if rank == 0:
            full = torch.zeros(L.nb_total * B * row_bytes, dtype=torch.uint8)
            assemble(full, gl, L, row_bytes)
            ref = O.render_f32(frame, scene, sky, W, H, threads=2)["rgba"].reshape(-1)
            q.put(bool(np.array_equal(full[: H * row_bytes].numpy(), ref)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,W,H,B", [(2, 48, 40, 8), (2, 33, 27, 8), (3, 40, 50, 16), (8, 24, 88, 8)])
def test_gloo_band_gather_reassembles_frame(world, W, H, B):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, W, H, B, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=10) is True


def test_band_layout_balance_4k_8ranks():
    L = [BandLayout(2160, 8, 8, r) for r in range(8)]
    rows = [l.rows_mine() for l in L]
    assert sum(rows) == 2160
    assert max(rows) / (2160 / 8) < 1.01
    # every frame row is owned exactly once
    owned = sorted(r for l in L for r in l.local_to_frame_rows() if r >= 0)
    assert owned == list(range(2160))


def test_band_layout_single_rank_is_identity():
    L = BandLayout(1080, 8, 1, 0)
    assert L.local_to_frame_rows() == list(range(1080))


def _worker_batched(rank, world, port, W, H, B, K, nframes, q):
    """Several frames per gather (frames_per_gather = K): rank r's buffer holds K
    packed frames back to back; rank 0 reassembles every frame of the batch."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import math

        import oracle as O
        from helpers import default_frame, default_scene
        from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

        sky = make_sky("equirect", (64, 32))
        scene = default_scene(256)
        L = BandLayout(H, B, world, rank)
        row_bytes = W * 4
        sl = L.nb_max * B * row_bytes
        frames = [default_frame(W, H, camera=(math.pi + 0.1 * f, 0.05 * f)) for f in range(nframes)]
        local = torch.zeros(K * sl, dtype=torch.uint8)
        for f in range(nframes):
            lv = local[f * sl:(f + 1) * sl].view(L.nb_max * B, row_bytes)
            for i, fr in enumerate(L.local_to_frame_rows()):
                if fr >= 0:
                    r = O.render_f32(frames[f], scene, sky, W, H, row0=fr, nrows=1, threads=1)
                    lv[i] = torch.from_numpy(r["rgba"].reshape(-1).copy())
        recv = torch.empty(world * K * sl, dtype=torch.uint8) if rank == 0 else None
        dist.gather(local, gather_list=list(recv.chunk(world)) if rank == 0 else None, dst=0)
        if rank == 0:
            ok = True
            gl = list(recv.chunk(world))
            for f in range(nframes):
                full = torch.zeros(L.nb_total * B * row_bytes, dtype=torch.uint8)
                assemble(full, gl, L, row_bytes, frame=f, frame_stride=sl)
                ref = O.render_f32(frames[f], scene, sky, W, H, threads=2)["rgba"].reshape(-1)
                ok = ok and bool(np.array_equal(full[: H * row_bytes].numpy(), ref))
            q.put(ok)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,W,H,B,K,nframes", [(2, 40, 36, 8, 3, 3), (3, 24, 40, 8, 4, 2)])
def test_gloo_batched_gather_reassembles_frames(world, W, H, B, K, nframes):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_batched, args=(r, world, port, W, H, B, K, nframes, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=10) is True


@pytest.mark.parametrize("H,B,world,lead", [(2160, 8, 8, 2), (2160, 8, 2, 4), (180, 8, 3, 2), (27, 8, 2, 2),
                                            (40, 8, 8, 4), (7, 8, 3, 1), (1080, 16, 4, 4), (2160, 8, 8, 3),
                                            (2160, 8, 2, 6), (100, 8, 4, 3)])
def test_lead_layout_owns_every_row_once(H, B, world, lead):
    L = [BandLayout(H, B, world, r, lead) for r in range(world)]
    owned = sorted(x for l in L for x in l.local_to_frame_rows() if x >= 0)
    assert owned == list(range(H))
    assert L[0].band_height() == lead * B and all(l.band_height() == B for l in L[1:])
    # rank 1 holds the largest peer share: the size of every gather contribution
    assert all(l.packed_rows() <= L[0].peer_packed_rows for l in L[1:])
    # rank 0's share is lead times a peer's, up to the last partial cycle
    if H >= 16 * L[0].cycle_rows:
        assert abs(L[0].rows_mine() / L[1].rows_mine() / lead - 1) < 0.03


@pytest.mark.parametrize("H,B,world,lead,pb", [(2160, 8, 8, 3, 2), (2160, 8, 8, 5, 2), (2160, 8, 4, 3, 2),
                                               (180, 8, 3, 3, 2), (41, 8, 2, 1, 2), (1080, 16, 4, 5, 3),
                                               (7, 8, 3, 3, 2), (2160, 8, 2, 2, 2)])
def test_share_layout_owns_every_row_once(H, B, world, lead, pb):
    """Peer bands of pb x band_rows: rank 0's share is lead / pb times a
    peer's (bench.py --rank0-lead a:b); every row owned once."""
    L = [BandLayout(H, B, world, r, lead, pb) for r in range(world)]
    owned = sorted(x for l in L for x in l.local_to_frame_rows() if x >= 0)
    assert owned == list(range(H))
    assert L[0].band_height() == lead * B and all(l.band_height() == pb * B for l in L[1:])
    assert L[0].cycle_rows == (lead + (world - 1) * pb) * B
    assert all(l.packed_rows() <= L[0].peer_packed_rows for l in L[1:])
    if H >= 16 * L[0].cycle_rows:
        assert abs(L[0].rows_mine() / L[1].rows_mine() / (lead / pb) - 1) < 0.05
    if (lead, pb) == (2, 2):  # the same ratio as lead 1 at twice the band height
        same = [BandLayout(H, 2 * B, world, r, 1) for r in range(world)]
        assert [l.local_to_frame_rows() for l in L] == [l.local_to_frame_rows() for l in same]


def test_lead_one_is_the_plain_interleave():
    for H, B, world in [(2160, 8, 8), (33, 8, 3), (1080, 16, 4)]:
        for r in range(world):
            a, b = BandLayout(H, B, world, r), BandLayout(H, B, world, r, lead=1)
            rows = [f for band in a.bands() for f in range(band * B, band * B + B)]
            assert b.local_to_frame_rows() == [f if f < H else -1 for f in rows]


def _worker_lead(rank, world, port, W, H, B, lead, K, q, peer_bands=1):
    """The lead layout as dist.ShardedFrame runs it: peers send their packed
    bands (all contributions the size of rank 1's), rank 0 contributes a
    dummy and reassembles its own rows from its local bands."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import math

        import oracle as O
        from helpers import default_frame, default_scene
        from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

        sky = make_sky("equirect", (64, 32))
        scene = default_scene(256)
        L = BandLayout(H, B, world, rank, lead, peer_bands)
        row_bytes = W * 4
        frames = [default_frame(W, H, camera=(math.pi + 0.1 * f, 0.05 * f)) for f in range(K)]
        rows = L.packed_rows() if rank == 0 else L.peer_packed_rows
        sl = rows * row_bytes
        local = torch.zeros(K * max(sl, 1), dtype=torch.uint8)
        for f in range(K):
            lv = local[f * sl:(f + 1) * sl].view(rows, row_bytes)
            for i, fr in enumerate(L.local_to_frame_rows()):
                if fr >= 0:
                    r = O.render_f32(frames[f], scene, sky, W, H, row0=fr, nrows=1, threads=1)
                    lv[i] = torch.from_numpy(r["rgba"].reshape(-1).copy())
        tsl = L.peer_packed_rows * row_bytes
        send = torch.zeros(K * max(tsl, 1), dtype=torch.uint8) if rank == 0 else local
        recv = torch.empty(world * send.numel(), dtype=torch.uint8) if rank == 0 else None
        dist.gather(send, gather_list=list(recv.chunk(world)) if rank == 0 else None, dst=0)
        if rank == 0:
            gl = list(recv.chunk(world))
            gl[0] = local  # rank 0's rows never travel
            ok = True
            for f in range(K):
                full = torch.zeros(H * row_bytes, dtype=torch.uint8)
                assemble(full, gl, L, row_bytes, frame=f, frame_stride=[sl] + [tsl] * (world - 1))
                ref = O.render_f32(frames[f], scene, sky, W, H, threads=2)["rgba"].reshape(-1)
                ok = ok and bool(np.array_equal(full.numpy(), ref))
            q.put(ok)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,W,H,B,lead,K,pb", [(2, 40, 52, 8, 2, 2, 1), (3, 28, 72, 8, 4, 1, 1),
                                                   (3, 33, 40, 8, 2, 2, 1), (2, 40, 60, 8, 3, 2, 1),
                                                   (3, 28, 88, 8, 3, 1, 2), (2, 36, 70, 8, 5, 2, 2),
                                                   (8, 20, 96, 8, 3, 2, 2)])  # 8: config 4's world, a 3:2 share
def test_gloo_lead_layout_reassembles_frames(world, W, H, B, lead, K, pb):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_lead, args=(r, world, port, W, H, B, lead, K, q, pb)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=10) is True
