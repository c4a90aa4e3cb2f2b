"""Row-band sharding of a frame over the ranks of one node, and the gather to
rank 0 for present (config 4: 3840x2160 over 8 MI355X).

Rank g renders the interleaved bands g, g+N, g+2N, ... (band_rows rows each,
geo_render_bands) into a packed local buffer; rank 0 gathers the N packed
buffers (RCCL over xGMI on GPUs, gloo in the CPU tests) and scatters the bands
back into frame order (geo_assemble_bands, one launch per gathered batch).  Interleaving balances the frame, whose cost is
concentrated around the black hole image (8 ranks, 8-row bands: max/mean
rows 1.007).  The reference has no multi-device path; this is
the present-side exchange the north star asks for.
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class BandLayout:
    height: int
    band_rows: int
    world: int
    rank: int

    @property
    def nb_total(self) -> int:
        return (self.height + self.band_rows - 1) // self.band_rows

    @property
    def nb_max(self) -> int:
        return (self.nb_total + self.world - 1) // self.world

    def bands(self, rank: int | None = None) -> range:
        r = self.rank if rank is None else rank
        return range(r, self.nb_total, self.world)

    @property
    def nb_mine(self) -> int:
        return len(self.bands())

    def rows_mine(self) -> int:
        """Frame rows this rank renders (the last band may be clipped)."""
        return sum(min(self.band_rows, self.height - b * self.band_rows) for b in self.bands())

    def local_to_frame_rows(self, rank: int | None = None) -> list[int]:
        """Frame row of every local (packed) row; -1 for rows past the frame."""
        out = []
        for b in self.bands(rank):
            for i in range(self.band_rows):
                r = b * self.band_rows + i
                out.append(r if r < self.height else -1)
        return out


def assemble(full, recv, layout: BandLayout, row_bytes: int, frame: int = 0, frame_stride: int | None = None) -> None:
    """Host (torch) reassembly, for the CPU tests: scatter frame `frame` of the
    gathered packed buffers (one per rank, frames `frame_stride` bytes apart,
    nb_max bands each) into `full` (nb_total*band_rows*row_bytes elements,
    frame order).  The GPU path uses geo_assemble_bands."""
    band = layout.band_rows * row_bytes
    fs = layout.nb_max * band if frame_stride is None else frame_stride
    fv = full.view(layout.nb_total, band)
    for r in range(layout.world):
        n = len(layout.bands(r))
        if n:
            fv[r::layout.world] = recv[r][frame * fs: frame * fs + layout.nb_max * band].view(layout.nb_max, band)[:n]


class ShardedFrame:
    """Render-then-gather pipeline for one rank, K frames per gather.

    step(i) renders this rank's bands of frame i into slot i % K of batch
    buffer (i // K) % 2 on the current stream; after the K-th frame of a batch
    one async gather (RCCL, on its own stream, ordered after the renders)
    sends the K packed frames to rank 0, so a batch's gather overlaps the next
    batch's renders.  Rank 0 reassembles all K frames of a batch with one
    geo_assemble_bands launch when the batch retires.  K amortises the host
    cost of a gather (~34 us, tools/host_overhead.py) over K frames: at N = 8
    a 4K frame is ~31 us of GPU work per rank.
    """

    def __init__(self, ctx, frame, scene, width: int, height: int, band_rows: int, rank: int, world: int, device,
                 dist=None, host_gather: bool = False, frames_per_gather: int = 1):
        """host_gather: stage through host memory (gloo backend; rehearsals only)."""
        import torch

        self.host_gather = host_gather
        self.ctx, self.frame, self.scene = ctx, frame, scene
        self.width, self.height = width, height
        self.layout = BandLayout(height, band_rows, world, rank)
        self.rank, self.world, self.dist = rank, world, dist
        self.K = max(1, int(frames_per_gather)) if world > 1 else 1
        L = self.layout
        self.row_bytes = width * 4
        self.slice = L.nb_max * band_rows * self.row_bytes  # one frame's packed bands
        self.bufs = [torch.empty(self.K * self.slice, dtype=torch.uint8, device=device) for _ in range(2)]
        self.frame_bytes = height * self.row_bytes  # assembled frames, back to back
        self.recv = None
        self.frames = None
        self.side = None
        if world > 1 and rank == 0:
            rdev = "cpu" if host_gather else device
            self.recv = [torch.empty(world * self.K * self.slice, dtype=torch.uint8, device=rdev) for _ in range(2)]
            self.frames = torch.empty(self.K * self.frame_bytes, dtype=torch.uint8, device=device)
            if not host_gather:
                # reassembly (HBM-bound) on its own stream, overlapping the next renders (VALU-bound)
                self.side = torch.cuda.Stream(device)
                self.ev_gathered = [torch.cuda.Event() for _ in range(2)]
                self.ev_assembled = [None, None]
        self.pending = [None, None]  # (work, nframes, batch number) per batch buffer
        self.rendered = 0            # frames rendered into the open batch
        self.open = 0                # batch buffer being filled
        self.batches = 0             # batches launched
        self.frames_done = 0
        self.last = None             # (batch number, batch buffer, slot) of the newest retired frame

    def local_view(self, i: int):
        b, sub = (i // self.K) % 2, i % self.K
        return self.bufs[b][sub * self.slice:(sub + 1) * self.slice]

    def render_local(self, buf, scene=None, **outs) -> None:
        L = self.layout
        self.ctx.render_bands(self.frame, self.scene if scene is None else scene, self.width, self.height,
                              L.band_rows, self.rank, self.world, L.nb_mine, buf, **outs)

    def _launch(self, b: int, n: int) -> None:
        self.batches += 1
        if self.world == 1:
            self.pending[b] = (None, n, self.batches)
            return
        src = self.bufs[b].cpu() if self.host_gather else self.bufs[b]
        gl = list(self.recv[b].chunk(self.world)) if self.rank == 0 else None
        if self.side is not None and self.ev_assembled[b] is not None:
            import torch

            # recv[b] is read by the reassembly of the batch two back
            torch.cuda.current_stream().wait_event(self.ev_assembled[b])
        work = self.dist.gather(src, gather_list=gl, dst=0, async_op=True)
        self.pending[b] = (work, n, self.batches)

    def _retire(self, b: int) -> None:
        p = self.pending[b]
        if p is None:
            return
        work, n, seq = p
        self.pending[b] = None
        if work is not None:
            if self.side is not None:
                import torch

                with torch.cuda.stream(self.side):
                    work.wait()  # the side stream waits for the gather
                    self.ev_gathered[b].record(self.side)
                    self.ctx.assemble_bands(self.recv[b], self.K * self.slice, self.slice, self.world,
                                            self.layout.band_rows, self.width, self.height, n, self.frames)
                    ev = torch.cuda.Event()
                    ev.record(self.side)
                    self.ev_assembled[b] = ev
                # bufs[b] (this rank's send buffer) is re-rendered next: after the gather
                torch.cuda.current_stream().wait_event(self.ev_gathered[b])
            else:
                work.wait()
                if self.rank == 0:
                    src = self.recv[b]
                    if self.host_gather:
                        src = src.to(self.frames.device)
                    self.ctx.assemble_bands(src, self.K * self.slice, self.slice, self.world, self.layout.band_rows,
                                            self.width, self.height, n, self.frames)
                    if self.host_gather:
                        import torch

                        torch.cuda.current_stream().synchronize()  # `src` is a temporary
        self.frames_done += n
        if self.last is None or seq > self.last[0]:
            self.last = (seq, b, n - 1)

    def step(self, i: int, steps_total=None, events=None, scene=None) -> None:
        b, sub = (i // self.K) % 2, i % self.K
        if sub == 0:
            self._retire(b)  # the batch that used this buffer two batches ago
        if events is not None:
            events[0].record()
        self.render_local(self.local_view(i), scene=scene, steps_total=steps_total)
        if events is not None:
            events[1].record()
        self.rendered = sub + 1
        self.open = b
        if sub == self.K - 1:
            self._launch(b, self.K)
            self.rendered = 0

    def drain(self) -> None:
        if self.rendered:  # a partial batch
            self._launch(self.open, self.rendered)
            self.rendered = 0
        for b in (0, 1):
            self._retire(b)

    def frame_rgba(self, i: int | None = None):
        """Rank 0's assembled frame: the last one retired (or frame slot i of
        the assembled batch), height*width*4 uint8."""
        if self.world == 1:
            _, b, k = self.last
            return self.bufs[b][k * self.slice:k * self.slice + self.height * self.row_bytes]
        k = self.last[2] if i is None else i
        return self.frames[k * self.frame_bytes:k * self.frame_bytes + self.height * self.row_bytes]
