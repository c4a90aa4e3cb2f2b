"""Row-band sharding of a frame over the ranks of one node, and the gather to
rank 0 for present (config 4: 3840x2160 over 8 MI355X).

Rank g renders its interleaved bands (BandLayout; geo_render_band_set) into a
packed local buffer; rank 0 gathers the peers' packed buffers (RCCL over xGMI
on GPUs, gloo in the CPU tests) and scatters them, with its own bands, back
into frame order (geo_assemble_lead, one launch per gathered batch).
Interleaving balances the frame, whose cost is concentrated around the black
hole image (8 ranks, 8-row bands: max/mean rows 1.007).  Every peer row
crosses an xGMI link into rank 0 and rank 0's rows cross none, so when the
links bound the present rank 0 takes `lead` times a peer's share.  The reference has no multi-device path; this is
the present-side exchange the north star asks for.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass


@dataclass(frozen=True)
class BandLayout:
    """Rows of a `height`-row frame owned by each of `world` ranks.

    The frame is cut into cycles of (lead + (world - 1) * peer_bands) *
    band_rows rows: rank 0 owns the first lead * band_rows rows of every
    cycle (one band of that height), rank r >= 1 the peer_bands * band_rows
    rows after rank r - 1's.  lead = peer_bands = 1 is the plain interleave
    (band b of band_rows rows belongs to rank b % world).  lead > peer_bands
    is the LEAD layout: rank 0 renders but never sends its rows, so when the
    present gather is link-bound it takes a larger share, lead / peer_bands
    times a peer's (bench.py --rank0-lead picks it by measurement; a ratio
    like 3:2 falls between the whole numbers)."""
    height: int
    band_rows: int
    world: int
    rank: int
    lead: int = 1
    peer_bands: int = 1

    def __post_init__(self):
        if self.lead < 1 or self.peer_bands < 1 or self.band_rows < 1 or self.world < 1:
            raise ValueError("lead, peer_bands, band_rows and world must be >= 1")

    @property
    def cycle_rows(self) -> int:
        return (self.lead + (self.world - 1) * self.peer_bands) * self.band_rows

    def _r(self, rank):
        return self.rank if rank is None else rank

    def band_height(self, rank: int | None = None) -> int:
        """Rows per band of a rank (lead * band_rows for rank 0, peer_bands * band_rows for a peer)."""
        return (self.lead if self._r(rank) == 0 else self.peer_bands) * self.band_rows

    def row0(self, rank: int | None = None) -> int:
        """First frame row of a rank's first band."""
        r = self._r(rank)
        return 0 if r == 0 else (self.lead + (r - 1) * self.peer_bands) * self.band_rows

    def nbands(self, rank: int | None = None) -> int:
        r0 = self.row0(rank)
        return 0 if r0 >= self.height else (self.height - r0 + self.cycle_rows - 1) // self.cycle_rows

    def packed_rows(self, rank: int | None = None) -> int:
        """Rows of a rank's packed buffer (its last band may be clipped)."""
        return self.nbands(rank) * self.band_height(rank)

    @property
    def peer_packed_rows(self) -> int:
        """Packed rows of the largest peer share (rank 1): the size every
        rank's gather contribution has."""
        return self.packed_rows(1) if self.world > 1 else 0

    # the plain interleave's vocabulary (lead = 1)
    @property
    def nb_total(self) -> int:
        return (self.height + self.band_rows - 1) // self.band_rows

    @property
    def nb_max(self) -> int:
        """Bands of the largest share (rank 0's)."""
        return self.packed_rows(0) // self.band_rows

    def bands(self, rank: int | None = None) -> range:
        if self.lead != 1 or self.peer_bands != 1:
            raise ValueError("bands() indexes the plain interleave (lead = peer_bands = 1)")
        r = self._r(rank)
        return range(r, self.nb_total, self.world)

    @property
    def nb_mine(self) -> int:
        return self.nbands()

    def local_to_frame_rows(self, rank: int | None = None) -> list[int]:
        """Frame row of every local (packed) row; -1 for rows past the frame."""
        out = []
        bh, r0 = self.band_height(rank), self.row0(rank)
        for j in range(self.nbands(rank)):
            for i in range(bh):
                r = r0 + j * self.cycle_rows + i
                out.append(r if r < self.height else -1)
        return out

    def rows_mine(self) -> int:
        """Frame rows this rank renders (the last band may be clipped)."""
        return sum(1 for r in self.local_to_frame_rows() if r >= 0)


def assemble(full, recv, layout: BandLayout, row_bytes: int, frame: int = 0, frame_stride=None) -> None:
    """Host (torch) reassembly, for the CPU tests: scatter frame `frame` of the
    gathered packed buffers (recv[r] = rank r's, frames `frame_stride` bytes
    apart: an int for every rank, a per-rank list, or None = the rank's packed
    size) into `full` (>= height*row_bytes elements, frame order).  The GPU
    path uses geo_assemble_bands / geo_assemble_lead."""
    import torch

    fv = full.view(-1, row_bytes)
    for r in range(layout.world):
        rows = layout.local_to_frame_rows(r)
        if not rows:
            continue
        n = len(rows)
        if frame_stride is None:
            fs = n * row_bytes
        elif isinstance(frame_stride, int):
            fs = frame_stride
        else:
            fs = frame_stride[r]
        src = recv[r][frame * fs: frame * fs + n * row_bytes].view(n, row_bytes)
        rt = torch.tensor(rows)
        keep = rt >= 0
        fv[rt[keep]] = src[keep]


class _RawEvent:
    """A HIP event without timing or system-scope release, recorded and waited
    on by stream handle (ctypes): the per-frame ordering of ShardedFrame at
    ~1 us per call instead of torch.cuda.Event's construction + record."""

    def __init__(self):
        from .timing import _hip, hipEventDisableSystemFence

        self._hip = _hip
        self.h = ctypes.c_void_p()
        if _hip.hipEventCreateWithFlags(ctypes.byref(self.h), hipEventDisableSystemFence | 0x2) != 0:
            raise RuntimeError("hipEventCreateWithFlags")
        self.recorded = False

    def record(self, stream: int) -> None:
        if self._hip.hipEventRecord(self.h, ctypes.c_void_p(stream)) != 0:
            raise RuntimeError("hipEventRecord")
        self.recorded = True

    def wait(self, stream: int) -> None:
        """`stream` waits for the last record (no-op before the first)."""
        if self.recorded and self._hip.hipStreamWaitEvent(ctypes.c_void_p(stream), self.h, 0) != 0:
            raise RuntimeError("hipStreamWaitEvent")

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            try:
                self._hip.hipEventDestroy(h)
            except Exception:  # interpreter shutdown
                pass
            self.h = None


def _batch_key(scene) -> bytes:
    """What the frames of one batched launch must share
    (geo_render_band_set_batch): the scene bytes but the observer radius, and
    the side of the horizon it is on (the integration kind); in fan mode the
    radius too (one fan for the launch)."""
    b = bytearray(bytes(scene))
    if scene.mode != 1:
        b[8:12] = b"\0\0\0\0"  # geo_scene.r_obs
        b += b"o" if scene.r_obs > scene.rs else b"i"
    return bytes(b)


def _empty_timing(events, stream: int) -> None:
    """A timed step of a rank with no rows renders nothing: record the
    caller's pair back to back on the stream, so elapsed_time reads ~0
    instead of failing on unrecorded events."""
    if events is not None:
        events[0].record(stream)
        events[1].record(stream)


class ShardedFrame:
    """Render-then-gather pipeline for one rank, K frames per gather.

    step(i) renders this rank's bands of frame i into slot i % K of batch
    buffer (i // K) % 2, on render stream i % S; after the K-th frame of a
    batch one async gather (RCCL, launched from its own stream once the
    batch's renders are done) sends the K packed frames to rank 0, so a
    batch's gather overlaps the next batch's renders.  Rank 0 reassembles all
    K frames of a batch, its own bands and the peers', with one
    geo_assemble_lead launch on a side stream when the batch retires.

    K amortises the host cost of a gather (~26-34 us, tools/host_overhead.py)
    over K frames; S = 2 render streams let frame i+1's waves fill frame i's
    tail (at N = 8 a rank's share of a 4K frame is only ~2 waves per slot:
    0.0417 -> 0.0309 ms/frame back to back, tools/scale_probe.py).  All
    cross-stream hazards are ordered with events: a peer's batch buffer is
    re-rendered only after its gather completed, rank 0's only after the
    reassembly that reads it, and rank 0's receive buffer is re-filled only
    after its reassembly completed.

    The per-frame path is host-bound at N = 8 unless it is lean (a peer's share
    of a 4K frame is ~26 us of GPU time): step() calls the C-ABI directly with
    pointers, stream handles and ctypes references computed once, and orders
    streams with pre-created raw HIP events (tools/host_bound_probe.py).
    Stream 0 is the caller's current stream when the object is built.
    """

    def __init__(self, ctx, frame, scene, width: int, height: int, band_rows: int, rank: int, world: int, device,
                 dist=None, host_gather: bool = False, frames_per_gather: int = 1, render_streams: int = 1,
                 present_rgb: bool = True, lead: int = 1, batch_launch: bool = False, peer_bands: int = 1):
        """host_gather: stage through host memory (gloo backend; rehearsals only).
        present_rgb: peers send RGB24 (geo_pack_rgb after each render; 25 %
        fewer bytes on the links) when the width is a multiple of 4.
        lead: rank 0's band height in band_rows (BandLayout); rank 0 never
        sends its own rows, its reassembly reads them from its local bands
        (geo_assemble_shares); peer_bands: a peer's band height in band_rows
        (BandLayout; rank 0's share is lead / peer_bands times a peer's).
        batch_launch: render each batch's K frames in ONE launch
        (geo_render_band_set_frames) when it is complete, on render stream
        (batch buffer % S): a launch's fixed cost (dispatch, ramp, drain) is
        paid once per batch instead of per frame; a peer's share at N = 8
        draws 10-12 % faster per frame.  K <= GEO_MAX_BATCH_FRAMES."""
        import torch

        from ._lib import lib

        self.torch = torch
        self.lib = lib
        self.host_gather = host_gather
        self.ctx, self.frame, self.scene = ctx, frame, scene
        self.width, self.height = width, height
        self.layout = BandLayout(height, band_rows, world, rank, lead if world > 1 else 1,
                                 peer_bands if world > 1 else 1)
        self.rank, self.world, self.dist = rank, world, dist
        # one rank alone batches frames only to render them in one launch
        self.K = max(1, int(frames_per_gather)) if world > 1 or batch_launch else 1
        self.S = min(2, max(1, int(render_streams)))
        from ._lib import GEO_MAX_BATCH_FRAMES

        self.batch = bool(batch_launch) and self.K > 1
        if self.batch and self.K > GEO_MAX_BATCH_FRAMES:
            raise ValueError(f"batch_launch: at most {GEO_MAX_BATCH_FRAMES} frames per gather")
        self.pending_frames = []     # batch mode: copies of the open batch's uniforms not yet rendered,
        self.pending_scenes = []     # and copies of their scenes (they differ in r_obs at most)
        self._pending_key = b""
        self.pending_first = 0       # and the slot of the first of them
        L = self.layout
        self.row_bytes = width * 4
        # one frame's packed bands: rank 0's share, or the largest peer share
        # (every gather contribution has the same size)
        rows = L.packed_rows(0) if rank == 0 else L.peer_packed_rows
        self.slice = rows * self.row_bytes
        self.bufs = [torch.empty(self.K * self.slice, dtype=torch.uint8, device=device) for _ in range(2)]
        # what travels: RGB24 (3/4 of the bytes) or the RGBA8 bands themselves
        self.bpp = 3 if (present_rgb and world > 1 and width % 4 == 0) else 4
        self.tslice = L.peer_packed_rows * width * self.bpp
        if rank == 0 and world > 1:
            # rank 0's own contribution to the gather is never read (its rows
            # are reassembled from self.bufs): one zero block
            dummy = torch.zeros(self.K * self.tslice, dtype=torch.uint8, device=device)
            self.sbufs = [dummy, dummy]
        else:
            self.sbufs = self.bufs if self.bpp == 4 else [
                torch.empty(self.K * self.tslice, dtype=torch.uint8, device=device) for _ in range(2)]
        self.frame_bytes = height * self.row_bytes  # assembled frames, back to back
        self.stream0 = torch.cuda.current_stream(device)
        self.extra = [torch.cuda.Stream(device) for _ in range(self.S - 1)]
        self.recv = None
        self.frames = None
        self.side = None
        self.gstream = None
        if world > 1 and not host_gather:
            self.gstream = torch.cuda.Stream(device)
        if world > 1 and rank == 0:
            rdev = "cpu" if host_gather else device
            self.recv = [torch.empty(world * self.K * self.tslice, dtype=torch.uint8, device=rdev) for _ in range(2)]
            self.frames = torch.empty(self.K * self.frame_bytes, dtype=torch.uint8, device=device)
            if not host_gather:
                # reassembly (HBM-bound) on its own stream, overlapping the next renders (VALU-bound)
                self.side = torch.cuda.Stream(device)
        # raw events: a batch buffer may be re-rendered after ev_free[b]; rank
        # 0's recv[b] may be re-filled after ev_assembled[b]; ev_rendered[b][k]
        # = the last render (and pack) of stream k into batch buffer b
        self.ev_free = [_RawEvent(), _RawEvent()]
        self.ev_assembled = [_RawEvent(), _RawEvent()]
        self.ev_rendered = [[_RawEvent() for _ in range(self.S)] for _ in range(2)]
        self.rendered_in = [[False] * self.S for _ in range(2)]  # stream k rendered into batch b since its launch
        # the per-frame C-ABI arguments, computed once
        self._sh = [self.stream0.cuda_stream] + [st.cuda_stream for st in self.extra]
        self._ctx_h = ctx._h
        self._frame_ref = ctypes.byref(frame)
        self._scene_ref = ctypes.byref(scene)
        self._band = (L.band_height(), L.row0(), L.cycle_rows, L.nbands())
        self._frame_arr = None  # batch mode: the uniforms of the last batch launched (kept alive for ctypes)
        self._lv = [[self.bufs[b].data_ptr() + sub * self.slice for sub in range(self.K)] for b in range(2)]
        self._sv = [[self.sbufs[b].data_ptr() + sub * self.tslice for sub in range(self.K)] for b in range(2)]
        self.pending = [None, None]  # (work, nframes, batch number, streams that rendered) per batch buffer
        self.rendered = 0            # frames rendered into the open batch
        self.open = 0                # batch buffer being filled
        self.batches = 0             # batches launched
        self.frames_done = 0
        self.last = None             # (batch number, batch buffer, slot) of the newest retired frame

    def local_view(self, i: int):
        b, sub = (i // self.K) % 2, i % self.K
        return self.bufs[b][sub * self.slice:(sub + 1) * self.slice]

    def render_local(self, buf, scene=None, frame=None, **outs) -> None:
        L = self.layout
        if L.nbands() == 0:  # a frame too small to give this rank a band
            return
        self.ctx.render_band_set(self.frame if frame is None else frame, self.scene if scene is None else scene,
                                 self.width, self.height, L.band_height(), L.row0(), L.cycle_rows, L.nbands(), buf,
                                 **outs)

    def _assemble(self, b: int, src, n: int, stream=None) -> None:
        """Rank 0: frames of batch b from its own bands (bufs[b]) and the peers' gathered blocks."""
        L = self.layout
        self.ctx.assemble_shares(self.bufs[b], self.slice, L.band_height(0), src, self.K * self.tslice, self.tslice,
                                 self.world, L.band_height(1), self.width, self.height, n, self.frames,
                                 src_bpp=self.bpp, stream=stream)

    def _render_stream(self, i: int):
        k = (i // self.K) % 2 % self.S if self.batch else i % self.S
        return self.stream0 if k == 0 else self.extra[k - 1]

    def render_batch(self, b: int, frames, scene=None, events=None, stream=None, first: int = 0,
                     scenes=None) -> None:
        """The frames of batch buffer b (slots first .. first + len(frames) - 1)
        in one launch (geo_render_band_set_batch), on `stream` (a handle;
        default the buffer's render stream).  scenes: one per frame (they may
        differ in r_obs only); default `scene` (or the object's) for all."""
        from ._lib import GeoFrame, GeoScene, check

        band_h, row0, cycle, nb = self._band
        sh = self._sh[b % self.S] if stream is None else stream
        if not nb:
            _empty_timing(events, sh)
            return
        if events is not None:
            st = self.lib.geo_time_next_render(self._ctx_h, events[0].h, events[1].h)
            if st != 0:
                check("geo_time_next_render", st)
        n = len(frames)
        if scenes is None:
            scenes = [self.scene if scene is None else scene] * n
        self._frame_arr = (GeoFrame * n)(*frames)
        self._scene_arr = (GeoScene * n)(*scenes)
        st = self.lib.geo_render_band_set_batch(
            self._ctx_h, self._frame_arr, self._scene_arr, n, self.width, self.height, band_h, row0, cycle, nb,
            self._lv[b][first], self.slice, None, sh)
        if st != 0:
            check("geo_render_band_set_batch", st)

    def _join(self) -> None:
        """The current stream waits for every render stream."""
        cur = self.torch.cuda.current_stream()
        for st in [self.stream0] + self.extra:
            if st.cuda_stream == cur.cuda_stream:
                continue
            ev = self.torch.cuda.Event()
            ev.record(st)
            cur.wait_event(ev)

    def _launch(self, b: int, n: int) -> None:
        self.batches += 1
        rendered = [k for k in range(self.S) if self.rendered_in[b][k]]
        self.rendered_in[b] = [False] * self.S
        if self.world == 1 or self.dist is None:  # one rank, or one rank's share alone (no present)
            self.pending[b] = (None, n, self.batches, rendered)
            return
        torch = self.torch
        gl = list(self.recv[b].chunk(self.world)) if self.rank == 0 else None
        if self.host_gather:
            self._join()
            work = self.dist.gather(self.sbufs[b].cpu(), gather_list=gl, dst=0, async_op=True)
        else:
            gsh = self.gstream.cuda_stream
            with torch.cuda.stream(self.gstream):
                # a peer sends after its renders; rank 0 sends nothing it
                # renders, so its receives are posted at once (its reassembly
                # waits for its renders instead)
                if self.rank != 0:
                    for k in rendered:
                        self.ev_rendered[b][k].wait(gsh)
                self.ev_assembled[b].wait(gsh)  # recv[b] is still being reassembled
                work = self.dist.gather(self.sbufs[b], gather_list=gl, dst=0, async_op=True)
        self.pending[b] = (work, n, self.batches, rendered)

    def _retire(self, b: int) -> None:
        p = self.pending[b]
        if p is None:
            return
        torch = self.torch
        work, n, seq, rendered = p
        self.pending[b] = None
        if work is not None and not self.host_gather:
            st = self.side if self.side is not None else self.gstream
            with torch.cuda.stream(st):
                work.wait()  # this stream waits for the gather
            sh = st.cuda_stream
            if self.side is not None:
                for k in rendered:  # rank 0's own bands of the batch
                    self.ev_rendered[b][k].wait(sh)
                self._assemble(b, self.recv[b], n, stream=sh)
                self.ev_assembled[b].record(sh)
            self.ev_free[b].record(sh)  # the gather (peer) or the reassembly (rank 0) read bufs[b]
        elif work is not None:
            work.wait()
            if self.rank == 0:
                src = self.recv[b].to(self.frames.device)
                self._assemble(b, src, n)
                torch.cuda.current_stream().synchronize()  # `src` is a temporary
        self.frames_done += n
        if self.last is None or seq > self.last[0]:
            self.last = (seq, b, n - 1)

    def _step_batch(self, b: int, sub: int, events, scene, frame) -> None:
        """Batch mode: record frame `sub` of the open batch; at its K-th frame
        render the batch in one launch, pack it (peers) and launch its gather.
        A launch's frames may differ in the observer radius only
        (geo_render_band_set_batch: a moving observer): a step whose scene
        differs otherwise from the pending frames' renders those first.  The
        uniform and the scene are copied when the step is recorded (the launch
        reads them later): a caller may update its objects in place between
        steps, as the per-frame path allows."""
        from ._lib import GeoFrame, GeoScene

        sc = GeoScene.from_buffer_copy(self.scene if scene is None else scene)
        key = _batch_key(sc)
        if self.pending_frames and key != self._pending_key:
            self._flush_batch(b)
        if not self.pending_frames:
            self.pending_first = sub
            self._pending_key = key
        self.pending_scenes.append(sc)
        self.pending_frames.append(GeoFrame.from_buffer_copy(self.frame if frame is None else frame))
        self.rendered = sub + 1
        self.open = b
        if sub == self.K - 1:
            self._flush_batch(b, events)
            self._launch(b, self.K)
            self.rendered = 0

    def _flush_batch(self, b: int, events=None) -> None:
        """Render the pending frames (their snapshots and their scenes') in one launch."""
        n, first = len(self.pending_frames), self.pending_first
        if not n:
            return
        k = b % self.S
        sh = self._sh[k]
        self.ev_free[b].wait(sh)
        self.render_batch(b, self.pending_frames, events=events, stream=sh, first=first, scenes=self.pending_scenes)
        self.pending_frames = []
        self.pending_scenes = []
        if self.bpp == 3 and self.rank != 0:
            st = self.lib.geo_pack_rgb(self._ctx_h, self._lv[b][first], n * self.slice // 4, self._sv[b][first], sh)
            if st != 0:
                from ._lib import check

                check("geo_pack_rgb", st)
        if self.world > 1:
            self.ev_rendered[b][k].record(sh)
            self.rendered_in[b][k] = True

    def step(self, i: int, steps_total=None, events=None, scene=None, frame=None) -> None:
        """Frame i: its bands rendered (batch mode: recorded, and the batch
        rendered in one launch at its K-th frame; `events` time that launch)
        into slot i % K of batch buffer (i // K) % 2.  frame: this frame's
        uniform (default the one the object was built with)."""
        b, sub = (i // self.K) % 2, i % self.K
        if sub == 0:
            self._retire(b)  # the batch that used this buffer two batches ago
        if self.batch:
            if steps_total is not None:
                raise ValueError("batch mode counts steps with GEO_FLAG_DEFER_STEPS only")
            self._step_batch(b, sub, events, scene, frame)
            return
        k = i % self.S
        sh = self._sh[k]
        if sub < self.S:
            self.ev_free[b].wait(sh)  # first render of this stream into the batch buffer
        band_h, row0, cycle, nb = self._band
        lib = self.lib
        if not nb:
            _empty_timing(events, sh)  # a rank with no rows: a zero-length pair
        elif events is not None:
            # the render's kernel dispatch carries the pair (no marker packets)
            st = lib.geo_time_next_render(self._ctx_h, events[0].h, events[1].h)
            if st != 0:
                from ._lib import check

                check("geo_time_next_render", st)
        if nb:
            st = lib.geo_render_band_set(
                self._ctx_h, self._frame_ref if frame is None else ctypes.byref(frame),
                self._scene_ref if scene is None else ctypes.byref(scene), self.width,
                self.height, band_h, row0, cycle, nb, self._lv[b][sub], None, None, None,
                None if steps_total is None else steps_total.data_ptr(), sh)
            if st != 0:
                from ._lib import check

                check("geo_render_band_set", st)
        if self.bpp == 3 and self.rank != 0:
            st = lib.geo_pack_rgb(self._ctx_h, self._lv[b][sub], self.slice // 4, self._sv[b][sub], sh)
            if st != 0:
                from ._lib import check

                check("geo_pack_rgb", st)
        if self.world > 1:
            self.ev_rendered[b][k].record(sh)
            self.rendered_in[b][k] = True
        self.rendered = sub + 1
        self.open = b
        if sub == self.K - 1:
            self._launch(b, self.K)
            self.rendered = 0

    def drain(self) -> None:
        """Finish every batch; afterwards the current stream is ordered after all work."""
        if self.rendered:  # a partial batch
            if self.batch:
                self._flush_batch(self.open)
            self._launch(self.open, self.rendered)
            self.rendered = 0
        for b in (0, 1):
            self._retire(b)
        self._join()
        cur = self.torch.cuda.current_stream()
        for st in (self.side, self.gstream):
            if st is not None:
                ev = self.torch.cuda.Event()
                ev.record(st)
                cur.wait_event(ev)

    def frame_rgba(self, i: int | None = None):
        """Rank 0's assembled frame: the last one retired (or frame slot i of
        the assembled batch), height*width*4 uint8."""
        if self.world == 1:
            _, b, k = self.last
            return self.bufs[b][k * self.slice:k * self.slice + self.height * self.row_bytes]
        k = self.last[2] if i is None else i
        return self.frames[k * self.frame_bytes:k * self.frame_bytes + self.height * self.row_bytes]
