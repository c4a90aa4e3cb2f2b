#!/usr/bin/env python3
"""bench.py — BASELINE.json metric: geodesic-steps·pixels/s at 3840x2160 with a
2048-step budget (config 3 on one GPU; config 4 = the same frame row-sharded
over N GPUs with an RCCL gather to rank 0).

One "step" = one frame: every rank renders its interleaved row bands of the
4K frame with the HIP kernel (geo_render_band_set), then (N > 1) rank 0
gathers the peers' bands over RCCL and reassembles the frame for present
(geo_assemble_lead).  Gathers run on RCCL's stream in batches of
--frames-per-gather frames, double-buffered, so a batch's gather overlaps the
next batch's compute.  Rank 0's share (--rank0-lead) is picked by measuring
the whole pipeline before the timed region.  value = executed RK4 main-loop
steps of all ranks / max-over-ranks wall time of the K timed frames (inputs
resident in HBM, sky uploaded once).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...

`python bench.py --gpus N` with no WORLD_SIZE in the environment starts the
N rank processes itself (launch_ranks, before anything touches the GPU),
waits for them, forwards rank 0's line and exits non-zero if any rank fails.
"""
from __future__ import annotations

import argparse
import datetime
import json
import math
import os
import signal
import socket
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_FP32_TFLOPS = 157.3  # MI355X FP32 vector peak (MI355X_MICROARCH.md, spec)
FLOPS_PER_EVAL = 40  # one RK4 evaluation of u'' = -u + 1.5 rs u^2
NEWTON_EVALS = 3  # per sphere crossing (sphere_ray_tracer.rs:129)
# adaptive mode (config 5): one Dormand-Prince RK5(4) attempt in Nystrom form
# (geo_pixel.h dp5_step, counting an FMA as 2): 77 flops with the error
# estimate and its h^2 scaling, 67 for a Newton evaluation (no estimate)
FLOPS_PER_ATTEMPT = 77
FLOPS_PER_NEWTON_DP5 = 67


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--spinup-frames", type=int, default=300,
                   help="untimed GPU clock spin-up frames x n_gpus before the warmup steps (the clock settles "
                        "after ~100 full frames); a frame count, identical on every rank")
    p.add_argument("--event-every", type=int, default=None,
                   help="time every k-th timed frame's kernel with an event pair on its dispatch (default: --steps "
                        "/ 10, at least 4: about 10 samples; a timed frame costs ~8 us more wall time than an "
                        "untimed one, profiles/r04h_event_cost.txt, so every 4th frame read 1-4 %% slower)")
    p.add_argument("--config", default="cfg3_4k")
    p.add_argument("--band-rows", type=int, default=8)
    p.add_argument("--render-streams", type=int, default=None,
                   help="render streams (1 or 2; default 1 at N = 1, 2 at N > 1): with 2, frame i+1's waves fill "
                        "frame i's tail (a rank's share at N = 8 is only ~2 waves per slot) and the per-launch "
                        "kernel time is measured on 20 back-to-back launches on one stream after the timed region. "
                        "N = 1 keeps one stream so that in-region launch times and rocprofv3's agree (--pipelined "
                        "reports the two-stream throughput beside it)")
    p.add_argument("--frames-per-gather", type=int, default=None,
                   help="N > 1: frames per RCCL gather to rank 0 (amortises the ~34 us host cost of a gather; "
                        "rank 0 reassembles each batch with one geo_assemble_lead launch).  Default: --steps / 10, "
                        "clamped to [1, 8]: the timed region ends with the last batch's gather and reassembly, "
                        "and its first batch's renders run before any gather starts, so a short run wants "
                        "shallow batches (20 steps: 2) and a long one amortises the host cost (200 steps: 8)")
    p.add_argument("--frames-per-launch", type=int, default=1,
                   help="N = 1: render this many consecutive frames in one launch (geo_render_band_set_batch), as "
                        "the ranks at N > 1 do per gather batch; 1 (default) = one launch per frame")
    p.add_argument("--batch-launch", default="auto", choices=["auto", "on", "off"],
                   help="N > 1: render each gather batch's frames in ONE launch (geo_render_band_set_frames), "
                        "paying a launch's fixed cost (~12.6 us: dispatch, ramp, drain) once per batch instead of per "
                        "frame; auto = on when --frames-per-gather > 1")
    p.add_argument("--rank0-lead", default="auto", type=_lead_spec,
                   help="N > 1: rank 0's share per cycle against a peer's, as 'a' or 'a:b' (rank 0 a 8-row bands, "
                        "each peer b; it renders rows that never cross an xGMI link, so a link-bound present wants "
                        "it larger); auto = the fastest of %s measured on the whole pipeline before the timed "
                        "region" % ", ".join("%d:%d" % ab for ab in LEAD_TRIALS))
    p.add_argument("--lead-trial-frames", type=int, default=120,
                   help="frames per --rank0-lead auto trial (after a quarter as many warm-up frames)")
    p.add_argument("--pipelined", action="store_true",
                   help="N = 1: also time the K frames on two render streams (consecutive frames overlap) and report "
                        "it as `pipelined`; off by default, since rocprofv3 would average the overlapped launches "
                        "into the kernel's duration")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=16)
    p.add_argument("--cpu-row-step", type=int, default=None,
                   help="CPU baseline sample: every k-th row (default 1 up to 4K, 4 above)")
    p.add_argument("--mode", default=None, choices=["direct", "fan", "adaptive"],
                   help="default: the config's mode (cfg1-4 direct, cfg5_8k_adaptive adaptive)")
    p.add_argument("--mips", action="store_true",
                   help="sample the sky through its mip chain (GEO_FLAG_MIPS, the reference's textureSample); "
                        "the metric's line is the level-0 path")
    p.add_argument("--ring-f64", action="store_true",
                   help="GEO_FLAG_RING_F64 on every frame: the capture band's lanes integrate in f64 inside the "
                        "render kernel (direct or adaptive mode; batched launches too).  Without it an N = 1 "
                        "direct/adaptive line still measures the mode beside the metric, as its `ring_f64` record")
    p.add_argument("--no-ring-record", action="store_true", help="skip the `ring_f64` record")
    p.add_argument("--no-frame-check", action="store_true",
                   help="skip rank 0's check, after the timed region, that every frame of the timed run's last "
                        "batch (the frames as assembled for present) equals a single-launch render of the frame; "
                        "by default it runs and a mismatch exits non-zero")
    p.add_argument("--check-frame", action="store_true", help=argparse.SUPPRESS)  # the default since round 3
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="nccl (= RCCL over xGMI); gloo stages the gather through host memory (tests only)")
    p.add_argument("--motion", default="none", choices=list(MOTIONS),
                   help="per-frame uniforms of a moving observer for the warmup and timed frames (the reference's "
                        "present loop: Observer::update_position + calc_transformation_pipeline every frame, "
                        "observer.rs:105-125, renderer.rs:208-264): orbit = start_orbit(1.8) from the config's "
                        "position, fall = start_orbit(0) (the Fall button, lib.rs:180), pan = the camera turning "
                        "(move_camera); dt = 1/60 s.  Not the metric's line (that is one pose, config 3)")
    p.add_argument("--dispatch", default="learned", choices=["learned", "natural"],
                   help="workgroup dispatch order: learned longest-first (geo_set_dispatch default) or natural "
                        "row-major")
    p.add_argument("--share", default=None, type=_share_spec,
                   help="'r/n' (N = 1 only): render rank r's band set of an n-rank layout and nothing else (no "
                        "gather, no reassembly): one rank's compute at N = n, on this GPU")
    args = p.parse_args()
    if args.share is not None and args.gpus != 1:
        p.error("--share emulates one rank's share on one GPU: --gpus 1 only")
    return args


def _share_spec(v: str):
    r, _, n = v.partition("/")
    try:
        rn = (int(r), int(n))
    except ValueError:
        raise argparse.ArgumentTypeError(f"--share: 'r/n', got {v!r}")
    if not (rn[1] >= 2 and 0 <= rn[0] < rn[1]):
        raise argparse.ArgumentTypeError("--share: 0 <= r < n, n >= 2")
    return rn


MOTIONS = ("none", "orbit", "fall", "pan")


def motion_frames(g, cfg, kind: str, n: int, mode: int, flags: int, tol: float, dt: float = 1.0 / 60.0):
    """n (uniform, scene) pairs of a moving observer, one per frame, starting
    from the config's pose (see --motion).  The scene follows the observer's
    radius (geo_scene.r_obs), as the reference's per-frame uniform does
    (lib.rs:292)."""
    obs = g.Observer(cfg.rs, cfg.fov, cfg.width, cfg.height)
    obs.set_position(*cfg.position)
    obs.set_camera(*cfg.camera)
    obs.set_energy(cfg.energy)
    if kind in ("orbit", "fall") and not obs.start_orbit(1.8 if kind == "orbit" else 0.0):
        raise SystemExit(f"--motion {kind}: no orbit from {cfg.position}")
    out = []
    for _ in range(n):
        if kind == "pan":
            obs.move_camera(6.0, 0.0)  # pixels of mouse motion per frame (observer.rs:179-188)
        else:
            obs.update_position((0.0, 0.0, 0.0), dt)
        out.append((obs.calc_transformation_pipeline(),
                    g.make_scene(cfg.rs, cfg.sphere_r, obs.get_radial_position(), cfg.step, cfg.max_steps, mode,
                                 flags=flags, tol=tol)))
    return out


# --rank0-lead auto: (rank 0's bands, each peer's bands) per cycle, in the
# order tried (shares of rank 0 at N = 8: 1/15, 1/8, 3/17, 2/9, 5/19, 3/10,
# 4/11, 6/13).  Rank 0 also reassembles every frame, so with fast links it
# may want less than a peer's share (1:2).
LEAD_TRIALS = [(1, 2), (1, 1), (3, 2), (2, 1), (5, 2), (3, 1), (4, 1), (6, 1)]


def _lead_spec(v: str):
    """'auto', 'a' or 'a:b' -> 'auto' or (a, b)."""
    if v == "auto":
        return v
    a, _, b = v.partition(":")
    try:
        ab = (int(a), int(b) if b else 1)
    except ValueError:
        raise argparse.ArgumentTypeError(f"--rank0-lead: 'auto', 'a' or 'a:b', got {v!r}")
    if ab[0] < 1 or ab[1] < 1:
        raise argparse.ArgumentTypeError("--rank0-lead: a and b must be >= 1")
    return ab


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv: list[str], rank_cmd: list[str] | None = None, grace_s: float = 10.0) -> int:
    """Start n rank processes and wait for them: one process per GPU, the
    torch.distributed env contract (RANK, LOCAL_RANK, WORLD_SIZE,
    LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1, a free MASTER_PORT).  The caller
    must not have touched the GPU (this process only forks children; it never
    execs).  Rank 0's JSON lines go to this process's stdout (the one line
    the contract asks for); everything else a rank prints on stdout (the
    peers' output, gloo's connection notices) goes to stderr.  When a rank
    fails, the others are
    terminated (SIGTERM, SIGKILL after grace_s) and its exit code is returned;
    0 when every rank exits 0.  rank_cmd replaces `python -u bench.py` (tests
    use a stub rank)."""
    cmd = (rank_cmd or [sys.executable, "-u", os.path.abspath(__file__)]) + list(argv)
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno()))

    def pump(src):
        for line in iter(src.readline, b""):
            dst = sys.stdout if line.lstrip().startswith(b"{") else sys.stderr
            dst.buffer.write(line)
            dst.flush()

    pumper = threading.Thread(target=pump, args=(procs[0].stdout,), daemon=True)
    pumper.start()

    def stop_all(sig=signal.SIGTERM):
        for p in procs:
            if p.poll() is None:
                try:
                    p.send_signal(sig)
                except ProcessLookupError:
                    pass

    prev = {}

    def forward(signum, _frame):  # the launcher's own SIGTERM/SIGINT end the ranks too
        stop_all(signum)

    for s in (signal.SIGTERM, signal.SIGINT):
        prev[s] = signal.signal(s, forward)
    rc = 0
    try:
        live = set(range(n))
        while live:
            for r in sorted(live):
                code = procs[r].poll()
                if code is None:
                    continue
                live.discard(r)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code  # -signal -> 128 + signal
                    print(f"launch_ranks: rank {r} exited with {code}; stopping the other ranks", file=sys.stderr)
                    stop_all()
                    t_end = time.monotonic() + grace_s
                    while any(p.poll() is None for p in procs) and time.monotonic() < t_end:
                        time.sleep(0.05)
                    stop_all(signal.SIGKILL)
            time.sleep(0.05)
        for p in procs:
            p.wait()
        pumper.join(timeout=5.0)
    finally:
        for s, h in prev.items():
            signal.signal(s, h)
    return rc


def rank_devices(dist, world: int, local: int, rdev) -> list[dict]:
    """Every rank's HIP device: index and PCI bus id (all-gathered, so rank 0
    can print the placement the job actually had)."""
    import torch

    p = torch.cuda.get_device_properties(local)
    mine = torch.tensor([local, p.pci_domain_id, p.pci_bus_id, p.pci_device_id], dtype=torch.int64, device=rdev)
    every = [mine]
    if world > 1:
        every = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(every, mine)
    return [{"rank": r, "device": int(t[0]), "pci": "%04x:%02x:%02x.0" % (int(t[1]), int(t[2]), int(t[3]))}
            for r, t in enumerate(every)]


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # start the N ranks from here, before any GPU call (the parent only waits)
        raise SystemExit(launch_ranks(args.gpus, sys.argv[1:]))
    import numpy as np
    import torch
    import torch.distributed as dist

    import schwarzschild_raytracer_wgpu_amd as g
    from schwarzschild_raytracer_wgpu_amd.scenes import CONFIGS, make_sky

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # --share r/n: this one process renders rank r's share of an n-rank layout
    lay_rank, lay_world = args.share if args.share else (rank, world)
    ndev = torch.cuda.device_count()
    if world > ndev and args.dist_backend == "nccl":
        # RCCL refuses two ranks on one GPU ("Duplicate GPU detected")
        raise SystemExit(f"--gpus {world} with the nccl backend needs {world} GPUs, this node has {ndev} "
                         f"(--dist-backend gloo runs several ranks per GPU, for rehearsals)")
    local = local % max(1, ndev)  # >1 rank per GPU only for gloo rehearsals on a 1-GPU box
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.dist_backend == "nccl":
            # a collective stuck for 5 minutes (a peer died or hangs; the
            # whole bench takes well under one) aborts the rank, so the
            # launcher stops the others instead of waiting for the driver's kill
            dist.init_process_group("nccl", device_id=dev, timeout=datetime.timedelta(minutes=5))
        else:
            dist.init_process_group("gloo", timeout=datetime.timedelta(minutes=5))
        if dist.get_world_size() != world:
            raise SystemExit(f"process group has {dist.get_world_size()} ranks, WORLD_SIZE={world}")

    if args.event_every is None:
        args.event_every = max(4, args.steps // 10)
    if args.frames_per_gather is None:
        args.frames_per_gather = max(1, min(8, args.steps // 10))
    cfg = CONFIGS[args.config]
    W, H = cfg.width, cfg.height
    obs = g.Observer(cfg.rs, cfg.fov, W, H)
    obs.set_position(*cfg.position)
    obs.set_camera(*cfg.camera)
    obs.set_energy(cfg.energy)
    frame = obs.calc_transformation_pipeline()
    args.mode = args.mode or cfg.mode
    mode = {"direct": g.GEO_MODE_DIRECT, "fan": g.GEO_MODE_FAN, "adaptive": g.GEO_MODE_ADAPTIVE}[args.mode]
    if args.motion != "none" and mode == g.GEO_MODE_FAN:
        raise SystemExit("--motion with --mode fan: the fan-mode draw needs a fan solved per radius (not benched)")
    tol = cfg.tol if mode == g.GEO_MODE_ADAPTIVE else 0.0
    sampler_flags = g._lib.GEO_FLAG_MIPS if args.mips else 0
    if args.ring_f64:
        if mode == g.GEO_MODE_FAN or args.mips:
            raise SystemExit("--ring-f64: direct or adaptive mode, level-0 sampler (geo.h)")
        sampler_flags |= g._lib.GEO_FLAG_RING_F64
    scene = g.make_scene(cfg.rs, cfg.sphere_r, obs.get_radial_position(), cfg.step, cfg.max_steps, mode,
                         flags=sampler_flags, tol=tol)
    sky = make_sky(cfg.sky, cfg.sky_size)
    ctx = g.Context(local)
    ctx.set_sky(sky)
    if args.dispatch == "natural":
        ctx.set_dispatch(g._lib.GEO_DISPATCH_ROW_MAJOR)
    if mode == g.GEO_MODE_FAN:
        ctx.solve_ray_fan(cfg.sphere_r, cfg.rs, cfg.max_steps, cfg.step, 400, obs.get_radial_position())

    # interleaved 8-row bands: rank g owns bands g, g+N, ... (balances the centre-heavy frame:
    # 270 bands of the 4K frame -> 34 vs 33.75 per rank at N=8); gather to rank 0 over RCCL.
    # With lead > 1 rank 0 owns lead-times-taller bands (it renders rows that never cross a link).
    from schwarzschild_raytracer_wgpu_amd.dist import ShardedFrame

    rdev = dev if args.dist_backend == "nccl" else "cpu"
    devices = rank_devices(dist, world, local, rdev)

    def make_sf(ld):
        lead, peer_bands = ld
        one = lay_world == 1
        return ShardedFrame(ctx, frame, scene, W, H, args.band_rows, lay_rank, lay_world, dev,
                            dist if world > 1 else None, host_gather=args.dist_backend == "gloo",
                            frames_per_gather=args.frames_per_launch if one else args.frames_per_gather,
                            render_streams=args.render_streams or (1 if world == 1 else 2), lead=lead,
                            peer_bands=peer_bands,
                            batch_launch=(args.frames_per_launch > 1) if one else args.batch_launch != "off")

    # everything that syncs or reads back (lead trials, the diagnostic pass)
    # runs before the clock spin-up below, which flows straight into the
    # warmup and the timed region
    if world == 1:
        leads = [(1, 1)]
    elif args.rank0_lead == "auto":
        leads = list(LEAD_TRIALS)
    else:
        leads = [args.rank0_lead]
    sf = make_sf((1, 1) if (1, 1) in leads else leads[0])
    steps_ctr = torch.zeros(1, dtype=torch.int64, device=dev)

    # rank 0's share (--rank0-lead auto): every layout runs the whole pipeline
    # (render, pack, gather, reassembly) for the same frames, untimed for the
    # metric; the fastest by max-over-ranks wall time is used for the timed
    # region.  Every rank holds the same all-reduced times, so all pick alike.
    lead_trials = None
    link_probe = present_link_probe(sf, dist, args) if world > 1 else None
    if len(leads) > 1:
        spin_up(sf, args.spinup_frames * world)  # the trials compare layouts at the settled clock
        times = []
        for ld in leads:
            t_sf = sf if ld == (sf.layout.lead, sf.layout.peer_bands) else make_sf(ld)
            for i in range(args.lead_trial_frames // 4):
                t_sf.step(i)
            t_sf.drain()
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            for i in range(args.lead_trial_frames):
                t_sf.step(i)
            t_sf.drain()
            torch.cuda.synchronize()
            dist.barrier()
            times.append(time.perf_counter() - t0)
            if t_sf is not sf:
                del t_sf
        tt = torch.tensor(times, dtype=torch.float64, device=rdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        best = leads[int(torch.argmin(tt).item())]
        lead_trials = {"%d:%d" % ld: float(tt[j]) / args.lead_trial_frames * 1e3 for j, ld in enumerate(leads)}
        if best != (sf.layout.lead, sf.layout.peer_bands):
            sf = make_sf(best)
    L = sf.layout

    # --motion: the warmup's and the timed frames' own uniforms and scenes
    # (plain, and with GEO_FLAG_DEFER_STEPS for the timed region)
    scene_defer = g.make_scene(cfg.rs, cfg.sphere_r, obs.get_radial_position(), cfg.step, cfg.max_steps, mode,
                               flags=g._lib.GEO_FLAG_DEFER_STEPS | sampler_flags, tol=tol)
    moving = None
    if args.motion != "none":
        mv = motion_frames(g, cfg, args.motion, args.warmup + args.steps, mode, sampler_flags, tol)
        moving = [(fr, sc, g.make_scene(cfg.rs, cfg.sphere_r, sc.r_obs, cfg.step, cfg.max_steps, mode,
                                         flags=g._lib.GEO_FLAG_DEFER_STEPS | sampler_flags, tol=tol))
                  for fr, sc in mv]

    def pose(i, defer=True):
        """(uniform, scene) of warmup/timed frame i (i counts from the first
        warmup frame); the scene with GEO_FLAG_DEFER_STEPS (the timed region
        counts its steps in the context) or without (the warmup)."""
        return (None, None) if moving is None else (moving[i][0], moving[i][2 if defer else 1])

    # untimed diagnostic pass: per-pixel steps + mask give the RK4 evaluations
    # per launch (main-loop steps + 3 Newton evaluations per sphere crossing);
    # with --motion, of every timed frame (per-frame totals on the device)
    n_loc = max(1, L.packed_rows()) * W
    diag_mask = torch.zeros(n_loc, dtype=torch.uint8, device=dev)
    diag_steps = torch.zeros(n_loc, dtype=torch.int32, device=dev)
    diag_ctr = torch.zeros(1, dtype=torch.int64, device=dev)
    diag_uv = torch.zeros(n_loc * 2, dtype=torch.float32, device=dev) if mode == g.GEO_MODE_FAN else None
    sf.render_local(sf.bufs[0], out_mask=diag_mask, out_uv=diag_uv, out_steps=diag_steps, steps_total=diag_ctr)
    per_frame = None  # --motion: [(steps, hits)] of each timed frame
    if moving is not None:
        f_steps = torch.zeros(args.steps, dtype=torch.int64, device=dev)
        f_hits = torch.zeros(args.steps, dtype=torch.int64, device=dev)
        m_mask = torch.zeros_like(diag_mask)
        m_steps = torch.zeros_like(diag_steps)
        for i in range(args.steps):
            fr, sc = moving[args.warmup + i][:2]
            sf.render_local(sf.bufs[1], scene=sc, frame=fr, out_mask=m_mask, out_steps=m_steps,
                            steps_total=f_steps[i:i + 1])
            f_hits[i] = ((m_mask == 0) & (m_steps > 0)).sum()
        per_frame = list(zip(f_steps.tolist(), f_hits.tolist()))
        del m_mask, m_steps
    torch.cuda.synchronize()
    # the fan-mode draw is a memory-side kernel: its algorithmic bytes are the
    # RGBA8 it writes plus the distinct sky texels its rows sample (and the fan)
    sky_touch = None
    if mode == g.GEO_MODE_FAN:
        valid = torch.zeros(n_loc, dtype=torch.bool, device=dev)
        valid.view(-1, W)[: L.rows_mine()] = True  # the packed rows this rank renders
        sky_touch = sky_bytes_touched(diag_uv.view(-1, 2), (diag_mask == 0) & valid, sky.shape[1], sky.shape[0])
        del valid
    st = diag_steps.to(torch.int64)
    hits = int(((diag_mask == 0) & (st > 0)).sum().item())  # unwritten (clipped) rows are 0
    rows_mine = L.rows_mine()
    steps_diag = int(diag_ctr.item())

    def flops_of(steps, hits):
        if mode == g.GEO_MODE_ADAPTIVE:
            return FLOPS_PER_ATTEMPT * steps + FLOPS_PER_NEWTON_DP5 * NEWTON_EVALS * hits
        return FLOPS_PER_EVAL * (steps + NEWTON_EVALS * hits)

    if per_frame is None:
        per_frame = [(steps_diag, hits)] * args.steps
    frame_flops = [flops_of(st_, h_) for st_, h_ in per_frame]
    steps_timed = sum(st_ for st_, _ in per_frame)  # what the timed region must count
    # per-launch figures: the average timed frame (one pose: the diagnostic frame's)
    evals_per_launch = round(sum(st_ + NEWTON_EVALS * h_ for st_, h_ in per_frame) / args.steps)
    flops_per_launch = flops_mean = sum(frame_flops) / args.steps

    # timed region: K frames; steps counted in the context (GEO_FLAG_DEFER_STEPS)
    # and flushed once at the end; fence-free event pairs on every k-th frame
    from schwarzschild_raytracer_wgpu_amd.timing import HipEvent

    # per-launch kernel time: event pairs inside the timed region with one
    # render stream; with two (N > 1) launches overlap by design, so the
    # launch duration is measured on isolated launches after the timed region
    timed = set(range(0, args.steps, max(1, args.event_every))) if sf.S == 1 and not sf.batch else set()
    evs = {i: (HipEvent(), HipEvent()) for i in timed}
    steps_ctr.zero_()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()

    # GPU clock spin-up (untimed, not counted as warmup), then the warmup,
    # then the timed region, with no host work in between: the clock falls
    # back within ~1 ms of an idle queue and the next ~100 4K frames run
    # 10-30 % slower (tools/ubench/clock_probe.py), so everything that syncs
    # or reads back (the diagnostic pass, the lead trials) comes before this.
    # The short syncs every 50 frames keep the host within reach of the GPU
    # and cost nothing (clock_probe: no ramp after them).
    spin = args.spinup_frames * world
    spin_up(sf, spin)
    for i in range(args.warmup):
        fr, sc = pose(i, defer=False)
        sf.step(i, frame=fr, scene=sc)
    sf.drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        fr, sc = pose(args.warmup + i)
        sf.step(i, events=evs.get(i), scene=scene_defer if sc is None else sc, frame=fr)
    sf.drain()  # joins the render streams into the current one
    ctx.steps_flush(steps_ctr)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    # compute-only pass (SURVEY.md §8e asks for compute-only and end-to-end
    # scaling): the same K frames, rendered on the same streams, without the
    # RGB24 pack, the gather or the reassembly
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    c0 = time.perf_counter()
    if sf.batch:
        for i0 in range(0, args.steps, sf.K):
            n_b = min(sf.K, args.steps - i0)
            if moving is None:
                sf.render_batch((i0 // sf.K) % 2, [frame] * n_b, scene=scene_defer)
            else:
                mb = moving[args.warmup + i0:args.warmup + i0 + n_b]
                sf.render_batch((i0 // sf.K) % 2, [m[0] for m in mb], scenes=[m[2] for m in mb])
    else:
        for i in range(args.steps):
            fr, sc = pose(args.warmup + i)
            with torch.cuda.stream(sf._render_stream(i)):
                sf.render_local(sf.local_view(i), scene=scene_defer if sc is None else sc, frame=fr)
    sf._join()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed_compute = time.perf_counter() - c0
    ctx.steps_flush(torch.zeros(1, dtype=torch.int64, device=dev))  # discard this pass's steps
    # N = 1, informational: the same K frames with two render streams, so
    # that frame i+1's waves fill frame i's tail (what a frame loop gains
    # from pipelining; not the metric's value, whose launches do not overlap)
    pipelined = None
    if args.pipelined and world == 1 and sf.S == 1 and moving is None and args.share is None:
        sf2 = ShardedFrame(ctx, frame, scene, W, H, args.band_rows, rank, world, dev, None, render_streams=2)
        spin_up(sf2, max(100, args.warmup))  # its buffers' allocation idled the GPU
        torch.cuda.synchronize()
        p0 = time.perf_counter()
        for i in range(args.steps):
            sf2.step(i, scene=scene_defer)
        sf2.drain()
        torch.cuda.synchronize()
        el2 = time.perf_counter() - p0
        ctx.steps_flush(torch.zeros(1, dtype=torch.int64, device=dev))  # discard this pass's steps
        pipelined = {"render_streams": 2, "ms_per_step": el2 / args.steps * 1e3,
                     "value": steps_diag * args.steps / el2,
                     "what": "the same K frames on two render streams (consecutive frames overlap); informational"}
        del sf2
    per_launch = 1  # frames per timed launch
    if sf.S > 1 or sf.batch:
        # one launch at a time: 20 launches back to back on ONE stream (no
        # overlap, and no idle gap between them that would let the clock
        # drop), an event pair around each, one sync at the end; with batched
        # launches each is a whole batch of K frames, and its time / K the
        # per-frame figure the flops per frame divide
        iso = [(HipEvent(), HipEvent()) for _ in range(20)]
        cur = torch.cuda.current_stream().cuda_stream
        # with --motion the isolated launches draw the first timed frames (a
        # batch: the first K; one frame: the first), and their flops are those
        # frames'
        nb0 = sf.K if sf.batch else 1
        if moving is not None:
            flops_per_launch = sum(frame_flops[:nb0]) / nb0
        for a, b in iso:
            if sf.batch:
                if moving is None:
                    sf.render_batch(0, [frame] * sf.K, scene=scene_defer, events=(a, b), stream=cur)
                else:
                    mb = moving[args.warmup:args.warmup + sf.K]
                    sf.render_batch(0, [m[0] for m in mb], scenes=[m[2] for m in mb], events=(a, b), stream=cur)
            else:
                fr, sc = pose(args.warmup)
                ctx.time_next_render(a, b)
                sf.render_local(sf.bufs[0], scene=scene_defer if sc is None else sc, frame=fr)
        torch.cuda.synchronize()
        ctx.steps_flush(torch.zeros(1, dtype=torch.int64, device=dev))  # discard the isolated launches' steps
        evs = {i: ab for i, ab in enumerate(iso)}
        per_launch = sf.K if sf.batch else 1
    kernel_ms = sorted(a.elapsed_time(b) / per_launch for a, b in evs.values())
    kernel_ms_avg = sum(kernel_ms) / len(kernel_ms)
    if moving is not None and not (sf.S > 1 or sf.batch):
        # the event-timed frames' own flops over their own times
        flops_per_launch = sum(frame_flops[i] for i in evs) / len(evs)

    steps_done = int(steps_ctr.item())
    if steps_done != steps_timed:
        raise SystemExit(f"step counter mismatch: {steps_done} vs {steps_timed} counted by the diagnostic pass")
    stats = torch.tensor([elapsed, kernel_ms_avg, elapsed_compute], dtype=torch.float64, device=rdev)
    tot = torch.tensor([steps_done, rows_mine * W * args.steps, evals_per_launch], dtype=torch.int64, device=rdev)
    per_rank = None
    if world > 1:
        # per-rank diagnostics for the scaling analysis: each rank's wall and
        # compute-only time, isolated-launch kernel time and rows
        mine = torch.tensor([elapsed, elapsed_compute, kernel_ms_avg, float(rows_mine)], dtype=torch.float64,
                            device=rdev)
        every = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(every, mine)
        per_rank = {"ms_per_step": [round(float(t[0]) / args.steps * 1e3, 5) for t in every],
                    "compute_only_ms_per_step": [round(float(t[1]) / args.steps * 1e3, 5) for t in every],
                    "kernel_ms_avg": [round(float(t[2]), 5) for t in every],
                    "rows": [int(t[3]) for t in every]}
        dist.all_reduce(stats, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    elapsed_max, kernel_ms_max, compute_max = float(stats[0]), float(stats[1]), float(stats[2])
    total_steps, total_pixels, evals_all = (int(x) for x in tot.tolist())

    # rank 0, outside the timed region: the frames of the timed run's last
    # batch, as assembled for present from every rank's bands (RCCL gather +
    # geo_assemble_lead at N > 1), against a single-launch render of the frame
    frame_check = None
    if not args.no_frame_check and rank == 0 and args.share is None:
        # the last timed frame's own pose (with --motion each frame has its own)
        ref = torch.empty(H * W * 4, dtype=torch.uint8, device=dev)
        if moving is None:
            ctx.render_rows(frame, scene, W, H, 0, H, ref)
        else:
            frames_ref = []
            nbatch = sf.last[2] + 1
            i_last = args.steps - 1
            for k in range(nbatch):
                fr, sc = moving[args.warmup + i_last - (nbatch - 1 - k)][:2]
                r_k = torch.empty(H * W * 4, dtype=torch.uint8, device=dev)
                ctx.render_rows(fr, sc, W, H, 0, H, r_k)
                frames_ref.append(r_k)
            ref = frames_ref[-1]
        torch.cuda.synchronize()
        nbatch = sf.last[2] + 1
        if moving is None:
            frames_ref = [ref] * nbatch
        same = [bool(torch.equal(sf.frame_rgba(k), frames_ref[k])) for k in range(nbatch)] if world > 1 else [
            bool(torch.equal(sf.frame_rgba(), ref))]
        frame_check = {"ok": all(same), "frames": len(same), "ranks": world,
                       "what": "rank 0's assembled frames of the timed run's last batch == a single-launch "
                               "geo_render_rows of the whole frame (byte-exact RGBA)"}
        print(f"frame-check: {sum(same)} of {len(same)} assembled {W}x{H} frame(s) from {world} rank(s) equal "
              f"the single-launch frame", file=sys.stderr)

    if world > 1:
        # every rank exits with rank 0's verdict (a peer left running would hang the launcher)
        ok = torch.tensor([0 if frame_check is not None and not frame_check["ok"] else 1], device=rdev)
        dist.broadcast(ok, src=0)
        frame_ok = bool(ok.item())
    else:
        frame_ok = frame_check is None or frame_check["ok"]
    if rank != 0:
        dist.destroy_process_group()
        if not frame_ok:
            raise SystemExit(1)
        return

    value = total_steps / elapsed_max if mode != g.GEO_MODE_FAN else total_pixels / elapsed_max
    # roofline for the dominant kernel, on this rank: algorithmic flops per
    # launch / avg launch time (event pairs on the kernel's own dispatch, the
    # execution time a profiler's timestamps give), and the same flops per
    # frame of the compute-only pass's wall time (no events; launch gaps
    # included)
    achieved_tflops = flops_per_launch / (kernel_ms_avg * 1e-3) / 1e12
    wall_tflops = flops_mean / (compute_max / args.steps) / 1e12
    pmc_file, pmc = pmc_profile(args.config, args.mode, world) if not args.mips else (None, {})
    if mode == g.GEO_MODE_FAN:
        metric = (f"pixels/sec at {W}x{H}, fan-mode draw (the reference's display path: 400-node fan lerp, "
                  f"shader.wgsl:77-105; whole job)")
        unit = "pixels/s"
        stepping = "fan lerp (no per-pixel geodesic)"
    elif mode == g.GEO_MODE_ADAPTIVE:
        metric = (f"geodesic-step-attempts·pixels/sec at {W}x{H}, adaptive RK5(4) tol {cfg.tol:g} "
                  f"(whole job; /GPU = value/n_gpus)")
        unit = "geodesic-step-attempts·pixels/s"
        stepping = f"adaptive Dormand-Prince RK5(4), tol {cfg.tol:g} in u, initial step pi/100, " \
                   f"{cfg.max_steps} max attempts"
    else:
        metric = f"geodesic-steps·pixels/sec at {W}x{H}, {cfg.max_steps} max steps (whole job; /GPU = value/n_gpus)"
        unit = "geodesic-steps·pixels/s"
        stepping = f"step pi/100, {cfg.max_steps} max RK4 steps"
    if args.motion != "none":
        metric += f" [moving observer: {args.motion}]"
    if args.ring_f64:
        metric += " [GEO_FLAG_RING_F64: the capture band redrawn in f64]"
    if args.share:
        metric += f" [rank {lay_rank}'s share of {lay_world}, alone]"
    out = {
        "metric": metric,
        "value": value,
        "unit": unit,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed_max / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",  # one fixed 4K frame per step, split over the ranks
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (reference default scene scaled to rs=1; 4096x2048 equirect checkerboard+xorshift sky)",
        "config": {
            "workload": f"{cfg.name}: {W}x{H}, rs={cfg.rs}, sphere_r={cfg.sphere_r}, observer {cfg.position} "
                        f"FrozenFall E={cfg.energy}, camera {tuple(round(c, 4) for c in cfg.camera)}, fov pi/2, "
                        f"{stepping}, mode {args.mode}, sky {'mip-mapped trilinear' if args.mips else 'level-0 bilinear'}",
            "width": W, "height": H, "max_steps": cfg.max_steps,
            "parallelism": (f"rowbands{world}" if world > 1 else
                            f"share {lay_rank}/{lay_world} alone (no gather)" if args.share else "single"),
            "motion": args.motion,
            "dispatch": args.dispatch,
            "band_rows": args.band_rows,
            "frames_per_gather": sf.K,
            "rank0_lead": "%d:%d" % (L.lead, L.peer_bands),
            "lead_trials_ms_per_frame": lead_trials,
            "render_streams": sf.S,
            "frames_per_launch": sf.K if sf.batch else 1,
            "ring_f64": bool(args.ring_f64),
        },
        "per_gpu": value / world,
        "world_size": dist.get_world_size() if world > 1 else 1,
        "dist_backend": args.dist_backend if world > 1 else None,
        "rank_devices": devices,
        "per_rank": per_rank,
        "pixels_per_s": total_pixels / elapsed_max,
        "frames_per_s": args.steps / elapsed_max,
        "steps_per_frame": total_steps // args.steps,
        "mean_steps_per_pixel": total_steps / total_pixels,
        "kernel_ms": {"avg": kernel_ms_avg, "median": kernel_ms[len(kernel_ms) // 2], "min": kernel_ms[0],
                      "max_over_ranks_avg": kernel_ms_max, "frames_timed": len(kernel_ms),
                      "events": ("event pairs on the render kernel's own dispatch (geo_time_next_render: "
                                 "start/end of its execution, no marker packets) on every %d-th timed frame"
                                 % args.event_every if sf.S == 1 and not sf.batch else
                                 "event pairs on the render kernel's own dispatch (geo_time_next_render) on 20 "
                                 "launches back to back on one stream after the timed region (%d render streams "
                                 "overlap consecutive frames inside it)" % sf.S if not sf.batch else
                                 "event pairs on the render kernel's own dispatch (geo_time_next_render) on 20 "
                                 "batched launches of %d frames back to back on one stream after the timed region, "
                                 "each launch's time / %d (the timed region renders each gather batch in one launch)"
                                 % (sf.K, sf.K))},
        "pipelined": pipelined,
        "link_probe": link_probe,
        "compute_only": {"value": (total_steps if mode != g.GEO_MODE_FAN else total_pixels) / compute_max, "ms_per_step": compute_max / args.steps * 1e3,
                         "what": "the same K frames rendered on the same streams without pack, gather or "
                                 "reassembly (max over ranks)"},
        "spinup_frames": spin,
        "roofline": {
            "bound": "valu",
            "achieved": achieved_tflops,
            "peak": PEAK_FP32_TFLOPS,
            "unit": "TFLOP/s",
            "frac": achieved_tflops / PEAK_FP32_TFLOPS,
            "traffic": pmc.get("traffic_bytes"),
            "kernel": f"geo_render_kernel<{mode}>",
            "flops": ("reference-equivalent algorithmic FP32 flops (FMA = 2): %s; the kernel executes fewer "
                      "instructions for the same arithmetic (14 VALU per RK4 step), so frac is not hardware VALU "
                      "utilisation: see hw_fp32_tflops_pmc and valu_per_simd_cycle_pmc"
                      % ("77 per RK5(4) attempt, 67 per Newton evaluation" if mode == g.GEO_MODE_ADAPTIVE else
                         "40 per RK4 evaluation of the reference's literal form, SURVEY.md §8d")),
            "algorithmic_flops_per_launch": flops_per_launch,
            "evals_per_launch": evals_per_launch,
            "achieved_wall": wall_tflops,
            "frac_wall": wall_tflops / PEAK_FP32_TFLOPS,
            "wall": "flops per launch / (compute-only wall time per frame): no event pairs, launch gaps included",
            "hw_fp32_tflops_pmc": pmc.get("hw_fp32_tflops"),
            "valu_per_simd_cycle_pmc": pmc.get("valu_per_simd_cycle"),
            "pmc_profile": pmc_file,
        },
    }
    out["roofline"]["trace_check"] = trace_profile(out["config"]["workload"], world) if not args.share else None
    if mode == g.GEO_MODE_FAN:
        out["roofline"] = fan_roofline(sky_touch, rows_mine * W, kernel_ms_avg, compute_max / args.steps * 1e3, pmc,
                                       pmc_file, mode)
    cpu_ok = True
    if world == 1 and not args.no_cpu_baseline:
        fan = None
        if mode == g.GEO_MODE_FAN:  # the fan the draws read, as the host's copy
            fan = ctx.solve_ray_fan(cfg.sphere_r, cfg.rs, cfg.max_steps, cfg.step, 400, obs.get_radial_position())
        # (with --ring-f64 the CPU path draws the band in f64 too: geo_band.h on the host)
        out["cpu_baseline"] = cpu_baseline(frame, scene, sky, W, H, args, ctx, fan)
        cpu_ok = out["cpu_baseline"]["matches_gpu"]["ok"]
        if mode != g.GEO_MODE_FAN:
            out["reference_equivalent"] = reference_fan_cost(ctx, cfg, obs.get_radial_position())
    out["frame_check"] = frame_check
    ring_ok = True
    if (world == 1 and mode != g.GEO_MODE_FAN and not args.ring_f64 and not args.mips and not args.share
            and args.motion == "none" and not args.no_ring_record and cfg.rs > 0.0):
        out["ring_f64"] = ring_record(g, ctx, frame, scene, sky, W, H, args, flops_of, dev)
        ring_ok = out["ring_f64"]["matches_cpu"]["ok"]
    print(json.dumps(out), flush=True)
    if not ring_ok and not os.environ.get("GEO_AB_VARIANT"):  # (A/B runs of non-specification variants)
        raise SystemExit("ring_f64: the GPU's band rows differ from the CPU path's (matches_cpu)")
    if not cpu_ok:
        raise SystemExit("cpu_baseline: the CPU path's rows differ from the GPU frame's (matches_gpu)")
    if world > 1:
        dist.destroy_process_group()
    if not frame_ok:
        raise SystemExit("frame check failed: an assembled frame differs from the single-launch frame")


def sky_bytes_touched(uv, sampled, tw: int, th: int) -> dict:
    """Distinct sky bytes a frame's level-0 bilinear samples read (device
    tensors: uv (n, 2) f32, sampled (n,) bool = pixels that take a sample).
    Texel quads as the sampler forms them (geo_pixel.h sample_sky_quad_f:
    n = floor(U tw 256 - 128) in one f32 rounding, x0 = n >> 8; U wraps, V
    clamps), counted once each: the algorithmic read bytes.  Beside them the
    distinct 128-B lines of the padded sky the device reads them from."""
    import torch

    u = uv[sampled, 0].double()
    v = uv[sampled, 1].double()
    # the product of two f32 is exact in f64, so one rounding of U tw256 - 128
    # to f32 is the fma's
    nx = torch.floor((u * (tw * 256.0) - 128.0).float()).to(torch.int64) >> 8
    ny = torch.floor((v * (th * 256.0) - 128.0).float()).to(torch.int64) >> 8
    texels, lines = [], []
    for dx in (0, 1):
        for dy in (0, 1):
            x = torch.remainder(nx + dx, tw)
            y = torch.clamp(ny + dy, 0, th - 1)
            texels.append(y * tw + x)
            lines.append(((ny + dy + 1) * (tw + 2) + (nx + dx + 1)) * 4 // 128)  # padded layout (geo::pad_sky)
    n_tex = int(torch.unique(torch.cat(texels)).numel())
    n_lines = int(torch.unique(torch.cat(lines)).numel())
    return {"sampled_pixels": int(u.numel()), "texel_bytes": 4 * n_tex, "line_bytes_padded": 128 * n_lines,
            "sky_bytes": 4 * tw * th}


HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md §HBM: 8 TB/s spec)


def fan_roofline(touch: dict, pixels: int, kernel_ms: float, wall_ms: float, pmc: dict, pmc_file, mode) -> dict:
    """The fan-mode draw's roofline: HBM.  Algorithmic bytes per launch = 4 B
    of RGBA8 written per pixel + the distinct sky texels sampled x 4 B + the
    400-node fan (1.6 KB), over the kernel's average launch time."""
    written = 4 * pixels
    alg = written + touch["texel_bytes"] + 4 * 400
    achieved = alg / (kernel_ms * 1e-3) / 1e9
    return {
        "bound": "hbm",
        "achieved": achieved,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBS,
        "traffic": pmc.get("traffic_bytes"),
        "kernel": f"geo_render_kernel<{mode}> (fan-mode draw, two pixels per lane)",
        "algorithmic_bytes_per_launch": alg,
        "bytes": "4 B RGBA8 written per pixel + distinct sky texels the frame samples x 4 B (counted once, on the "
                 "device, from the diagnostic pass's UVs) + the 1.6-KB fan",
        "written_bytes": written,
        "sky_texel_bytes": touch["texel_bytes"],
        "sky_line_bytes_padded": touch["line_bytes_padded"],
        "sky_bytes": touch["sky_bytes"],
        "sampled_pixels": touch["sampled_pixels"],
        "achieved_wall": alg / (wall_ms * 1e-3) / 1e9,
        "frac_wall": alg / (wall_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
        "valu_per_simd_cycle_pmc": pmc.get("valu_per_simd_cycle"),
        "pmc_profile": pmc_file,
    }


def spin_up(sf, n):
    """n untimed frames back to back (a short sync every 50 keeps the host
    within reach of the GPU without idling it)."""
    import torch

    for i in range(n):
        sf.step(i)
        if i % 50 == 49:
            sf.drain()
            torch.cuda.synchronize()
    sf.drain()


def present_link_probe(sf, dist, args, reps=10):
    """N > 1, before the lead trials: the present gather alone, timed.  Every
    rank sends one batch contribution of the bench's size (K frames of the
    largest peer share, RGB24 or RGBA8) to rank 0, `reps` times back to back.
    It measures the per-peer link rate that DESIGN.md §6 models, on the node
    the bench runs on.  Diagnostic only, outside the timed region."""
    import torch

    dev = sf.bufs[0].device
    src = torch.zeros(sf.K * sf.tslice, dtype=torch.uint8, device=dev if args.dist_backend == "nccl" else "cpu")
    gl = [torch.empty_like(src) for _ in range(sf.world)] if sf.rank == 0 else None
    for _ in range(3):
        dist.gather(src, gather_list=gl, dst=0)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        dist.gather(src, gather_list=gl, dst=0)
    torch.cuda.synchronize()
    dist.barrier()
    dt = (time.perf_counter() - t0) / reps
    nbytes = src.numel()
    return {"what": "dist.gather of one batch contribution per rank to rank 0, %d back to back (%s)"
                    % (reps, args.dist_backend),
            "bytes_per_peer": nbytes, "ms_per_gather": dt * 1e3,
            "per_peer_gb_s": nbytes / dt / 1e9, "into_rank0_gb_s": nbytes * (sf.world - 1) / dt / 1e9}


def pmc_profile(config, mode, world):
    """The committed rocprofv3 PMC summary of this workload
    (profiles/*_<config>_pmc.json, made by tools/gpu_pmc.sh +
    tools/pmc_to_profile.py): (file name, its derived figures), or (None, {}).
    Only a profile taken on this exact workload counts: same config, same
    mode (its workload string ends in ", <mode>)"), one GPU (the profiles
    hold full-frame figures; at N > 1 a launch renders a partial share)."""
    import glob

    if world != 1:
        return None, {}
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_{config}_pmc.json")) +
                   glob.glob(os.path.join(ROOT, "profiles", f"*_{config}_{mode}_pmc.json")))
    for path in reversed(files):
        with open(path) as f:
            d = json.load(f)
        if d.get("workload", "").startswith(config) and d["workload"].endswith(f", {mode})"):
            return os.path.basename(path), d["derived"]
    return None, {}


def trace_profile(workload: str, world: int):
    """The committed same-invocation capture of this workload
    (profiles/*_trace_window.json, tools/evidence.sh bench step: the bench
    line and a rocprofv3 kernel trace of the SAME run, tools/trace_window.py):
    the profiler's timed-window launch average and the frac it gives beside
    the line's event-timed one, or None.  N = 1 only (a full-frame launch)."""
    import glob

    if world != 1:
        return None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_trace_window.json")), reverse=True):
        with open(path) as f:
            d = json.load(f)
        if d.get("workload") == workload and d.get("n_gpus") == 1:
            return {"profile": os.path.basename(path), "window_avg_ms": d["window_avg_ms"],
                    "events_avg_ms": d["line_kernel_ms_avg"], "frac_events": d["line_frac"],
                    "frac_trace": d["trace_frac"], "trace_over_events": d["trace_over_line"],
                    "what": "one earlier run of this workload under rocprofv3 --kernel-trace: its timed window's "
                            "average launch (profiler timestamps) against the same run's event pairs; the event "
                            "pair on a dispatch reads a few us longer than the profiler's kernel span, and a "
                            "box reads +-3 % from another (DESIGN.md §4, measurement)"}
    return None


def reference_fan_cost(ctx, cfg, r):
    """What the reference actually computes per frame on its CPU: the 400-node
    f64 ray fan of each of its 3 spheres (SphereRayTracer::solve_ray_fan,
    sphere_ray_tracer.rs:35-56; lib.rs:292-295), single-threaded — timed on
    the oracle's literal f64 restatement; beside it the same fans on the GPU
    (geo_solve_ray_fan, f64, one lane per node).  Display semantics differ
    (fan lerp vs per-pixel geodesics), so this is context, not
    the metric."""
    import oracle as O

    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        for sphere_r in (cfg.sphere_r, 1.1, 1.2):  # the reference's 3 spheres (lib.rs:67-89), rs = 1 units
            O.solve_ray_fan(sphere_r, cfg.rs, 1000, math.pi / 100, 400, r)
        n += 1
    cpu_ms = (time.perf_counter() - t0) / n * 1e3
    import torch

    for _ in range(3):
        ctx.solve_ray_fan(cfg.sphere_r, cfg.rs, 1000, math.pi / 100, 400, r)
    torch.cuda.synchronize()
    m = 20
    t0 = time.perf_counter()
    for _ in range(m):
        for sphere_r in (cfg.sphere_r, 1.1, 1.2):
            ctx.solve_ray_fan(sphere_r, cfg.rs, 1000, math.pi / 100, 400, r)
    gpu_ms = (time.perf_counter() - t0) / m * 1e3
    # as a device-side pipeline uses it: each sphere's fan solved into its own
    # context (the fan-mode render reads it there, as the reference's shader
    # reads its fan texture), the three on three streams, one sync per frame
    from schwarzschild_raytracer_wgpu_amd.api import Context
    from schwarzschild_raytracer_wgpu_amd import _lib

    ctxs = [Context(torch.cuda.current_device()) for _ in range(3)]
    streams = [torch.cuda.Stream() for _ in range(3)]

    def fans():
        for c, st, sphere_r in zip(ctxs, streams, (cfg.sphere_r, 1.1, 1.2)):
            _lib.check("geo_solve_ray_fan", _lib.lib.geo_solve_ray_fan(
                c._h, sphere_r, cfg.rs, 1000, math.pi / 100, 400, r, None, st.cuda_stream))
        torch.cuda.synchronize()

    for _ in range(3):
        fans()
    t0 = time.perf_counter()
    for _ in range(m):
        fans()
    gpu_async_ms = (time.perf_counter() - t0) / m * 1e3
    for c in ctxs:
        c.close()
    return {"what": "3 spheres x 400-node f64 ray fan per frame (the reference's per-frame CPU work)",
            "cpu_ms_per_frame_1core": cpu_ms, "gpu_ms_per_frame_geo_solve_ray_fan": gpu_ms,
            "gpu_ms_per_frame_device_fans": gpu_async_ms,
            "note": "geo_solve_ray_fan: one fan after another, each copied to the host synchronously; "
                    "device_fans: the three fans into their contexts on three streams, one sync per frame"}


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform

    return platform.processor() or "unknown"


def cpu_quota() -> float | None:
    """CPUs this process may use per the cgroup v2 quota (cpu.max), or None."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        return None if q == "max" else int(q) / int(p)
    except (OSError, ValueError):
        return None


def _cpu_lib():
    import ctypes

    lib = ctypes.CDLL(os.path.join(ROOT, "schwarzschild_raytracer_wgpu_amd", "libgeo_cpu.so"))
    vp, u32 = ctypes.c_void_p, ctypes.c_uint32
    lib.geo_render_cpu.restype = ctypes.c_int
    lib.geo_render_cpu.argtypes = [vp, vp, vp, u32, u32, vp, u32, u32, u32, u32, u32, u32, ctypes.c_int, vp, vp, vp,
                                   vp, vp]
    return lib


def cpu_baseline(frame, scene, sky, W, H, args, ctx, fan=None):
    """The same per-pixel integrator on the host cores: geo_render_cpu
    (libgeo_cpu.so, include/geo/geo_cpu.h), the product's geo_pixel.h built
    for the host (g++ -O2 -ffp-contract=off), scalar, std::thread row blocks
    (BASELINE.md §3).  Threads = the CPUs this process may run on at once:
    min(sched_getaffinity, ceil(cgroup quota)) (SURVEY.md §8d's
    hardware_concurrency, without oversubscribing the quota); the
    all-affinity figure beside it when it differs.  One warm-up, then the
    median of 3 runs of the frame (every 4th row above 4K).

    North_star's comparator, outside the timed runs: the CPU's rows against
    the same rows of the GPU frame (geo_render_rows): RGBA bytes, the
    hit-classification mask and the UV bits; matches_gpu false exits the
    bench non-zero."""
    import ctypes
    import statistics

    import numpy as np
    import torch

    lib = _cpu_lib()
    fan_arr = None if fan is None else np.ascontiguousarray(fan, dtype=np.float32)
    fan_p, n_fan = (None, 0) if fan_arr is None else (fan_arr.ctypes.data, fan_arr.size)
    all_cores = len(os.sched_getaffinity(0))
    k = args.cpu_row_step or (1 if W * H <= 3840 * 2160 else 4)
    if args.mips and k > 1 and k % 2:
        k += 1  # even rows only, so the partner rows traced for the footprint are the odd rows k m + 1
    nrows = (H + k - 1) // k
    sky = np.ascontiguousarray(sky, dtype=np.uint8)
    rgba = np.empty((nrows, W, 4), np.uint8)
    total = ctypes.c_ulonglong()

    def run(threads, rgba=rgba, mask=None, uv=None, row0=0, n=nrows, flags_scene=scene):
        rc = lib.geo_render_cpu(ctypes.addressof(frame), ctypes.addressof(flags_scene), sky.ctypes.data, sky.shape[1],
                                sky.shape[0], fan_p, n_fan, W, H, row0, n, k, threads, rgba.ctypes.data,
                                None if mask is None else mask.ctypes.data, None if uv is None else uv.ctypes.data,
                                None, ctypes.addressof(total))
        if rc != 0:
            raise SystemExit(f"geo_render_cpu: {rc}")
        return total.value

    def timed(threads):
        times, steps = [], None
        for rep in range(4):
            t0 = time.perf_counter()
            steps = run(threads)
            dt = time.perf_counter() - t0
            if rep > 0:  # rep 0 warms up
                times.append(dt)
        return statistics.median(times), times, steps

    # the headline uses the CPUs this process may actually run on at once:
    # its affinity mask capped by the cgroup quota (an oversubscribed pool of
    # 256 threads on a 16-CPU quota ran ~8 % slower, BENCH_r04); the
    # all-affinity figure is reported beside it
    quota = cpu_quota()
    threads = min(all_cores, math.ceil(quota)) if quota else all_cores
    med, times, steps = timed(threads)
    all_aff = None
    if threads != all_cores:
        _, t_all, _ = timed(all_cores)
        all_aff = {"threads": all_cores, "seconds_per_run": t_all, "value": None,
                   "what": "every core in the affinity mask (oversubscribes the cgroup quota)"}
    # GEO_FLAG_MIPS with k > 1: geo_render_cpu also traces each sampled row's
    # quad partner (row + 1) for the footprint; those rows' steps are work
    # done in the timed runs, counted here (the partner rows alone, untimed)
    partner_steps = 0
    if args.mips and k > 1:
        partner = np.empty(((H - 1 + k - 1) // k, W, 4), np.uint8)
        plain = type(scene).from_buffer_copy(scene)
        plain.flags = scene.flags & ~g_flag_mips()
        partner_steps = run(threads, rgba=partner, row0=1, n=(H - 1 + k - 1) // k, flags_scene=plain)
    work = steps + partner_steps
    if all_aff is not None:
        all_aff["value"] = work / statistics.median(all_aff["seconds_per_run"])

    # the comparator (untimed): CPU rows with mask and UV vs the GPU frame's rows
    mask_c = np.empty((nrows, W), np.uint8)
    uv_c = np.empty((nrows, W, 2), np.float32)
    rgba_c = np.empty_like(rgba)
    run(threads, rgba=rgba_c, mask=mask_c, uv=uv_c)
    dev = torch.device("cuda", torch.cuda.current_device())
    g_rgba = torch.empty(H * W * 4, dtype=torch.uint8, device=dev)
    g_mask = torch.empty(H * W, dtype=torch.uint8, device=dev)
    g_uv = torch.empty(H * W * 2, dtype=torch.float32, device=dev)
    ctx.render_rows(frame, scene, W, H, 0, H, g_rgba, out_mask=g_mask, out_uv=g_uv)
    torch.cuda.synchronize()
    g_rgba = g_rgba.view(H, W, 4)[::k].cpu().numpy()
    g_mask = g_mask.view(H, W)[::k].cpu().numpy()
    g_uv = g_uv.view(H, W, 2)[::k].cpu().numpy()
    rgba_same = bool(np.array_equal(rgba, g_rgba)) and bool(np.array_equal(rgba_c, g_rgba))
    mask_diff = int((mask_c != g_mask).sum())
    uv_bits_diff = int((uv_c.view(np.uint32) != g_uv.view(np.uint32)).any(axis=-1).sum())
    du = np.abs(uv_c[..., 0].astype(np.float64) - g_uv[..., 0])
    du = np.minimum(du, 1.0 - du)  # U wraps
    dv = np.abs(uv_c[..., 1].astype(np.float64) - g_uv[..., 1])
    uv_err = float(max(du.max(initial=0.0), dv.max(initial=0.0)))
    ok = rgba_same and mask_diff == 0 and uv_err <= 1e-4
    what = "full" if k == 1 else f"every {k}th row of the"
    unit = ("geodesic-step-attempts·pixels/s" if scene.mode == 2 else
            "pixels/s" if scene.mode == 1 else "geodesic-steps·pixels/s")
    value = (nrows * W) / med if scene.mode == 1 else work / med
    return {
        "value": value,
        "unit": unit,
        "cores": threads,
        "kind": "port",
        "cpu_model": cpu_model(),
        "cgroup_cpu_quota": cpu_quota(),
        "sample": f"{what} {W}x{H} frame ({nrows * W} pixels, {steps} steps"
                  f"{f' + {partner_steps} in the traced quad-partner rows' if partner_steps else ''}): "
                  f"median of 3 runs after one warm-up, {threads} threads (min(affinity mask {all_cores}, "
                  f"cgroup quota {quota}))",
        "seconds_per_run": times,
        "all_affinity": all_aff,
        "matches_gpu": {
            "ok": ok, "rows_compared": nrows, "pixels_compared": nrows * W,
            "rgba_identical": rgba_same, "mask_mismatches": mask_diff, "uv_bit_mismatches": uv_bits_diff,
            "uv_max_abs_err": uv_err,
            "what": "geo_render_cpu's rows vs the same rows of a geo_render_rows frame (device): RGBA bytes, "
                    "hit mask, UV (north_star: mask pixel for pixel, UV within 1e-4)",
        },
        "implementation": "geo_render_cpu (libgeo_cpu.so): geo_pixel.h compiled for the host, g++ -O2 "
                          "-ffp-contract=off -mfma -msse4.1, scalar, std::thread row blocks",
    }


def ring_record(g, ctx, frame, scene, sky, W, H, args, flops_of, dev):
    """GEO_FLAG_RING_F64 beside the metric's line (geo.h): the
    same frame with the capture band's lanes integrated in f64 inside the
    render kernel, the mode that meets north_star's UV bar against the
    reference's own f64 arithmetic on every pixel.  Plain and ring frames are
    timed interleaved (3 runs each of max(K, ~25 ms) frames, one launch per frame, one stream,
    the learned dispatch order of each), each launch's kernel by an event
    pair on its dispatch; then the GPU's rows through the band against the
    CPU path's (geo_render_cpu: geo_band.h on the host)."""
    import ctypes

    import numpy as np
    import torch

    from schwarzschild_raytracer_wgpu_amd.timing import HipEvent

    def flagged(flags):
        sc = g.GeoScene.from_buffer_copy(bytes(scene))
        sc.flags = (scene.flags | flags) & ~g._lib.GEO_FLAG_DEFER_STEPS
        return sc

    ring = flagged(g._lib.GEO_FLAG_RING_F64)
    plain_d = flagged(g._lib.GEO_FLAG_DEFER_STEPS)
    ring_d = flagged(g._lib.GEO_FLAG_RING_F64 | g._lib.GEO_FLAG_DEFER_STEPS)
    out = torch.empty(H * W * 4, dtype=torch.uint8, device=dev)
    # the ring frame's steps and hits (the band's pixels report their f64 steps)
    mask = torch.empty(H * W, dtype=torch.uint8, device=dev)
    steps = torch.empty(H * W, dtype=torch.int32, device=dev)
    total = torch.zeros(1, dtype=torch.int64, device=dev)
    ctx.render_rows(frame, ring, W, H, 0, H, out, out_mask=mask, out_steps=steps, steps_total=total)
    torch.cuda.synchronize()
    hits = int(((mask == 0) & (steps > 0)).sum().item())
    ring_steps = int(total.item())
    flops = flops_of(ring_steps, hits)
    del mask, steps
    def run(sc, n, events=None):
        for i in range(n):
            if events is not None and i in events:
                ctx.time_next_render(*events[i])
            ctx.render_rows(frame, sc, W, H, 0, H, out)

    run(ring_d, 100)  # its order learned, the clock settled
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(plain_d, 100)
    torch.cuda.synchronize()
    # frames per timed run: at least the line's K and about 25 ms of plain
    # frames (at K = 20 a 1080p run is 1.2 ms, short enough for the clock's
    # transitions between runs to read as several per cent either way)
    K = max(args.steps, min(2000, int(math.ceil(0.025 / max((time.perf_counter() - t0) / 100, 1e-6)))))
    ev = {i: (HipEvent(), HipEvent()) for i in range(0, K, max(1, K // 10))}
    res = {"plain": [], "ring": [], "plain_k": [], "ring_k": []}
    for rep in range(3):
        for name, sc in (("plain", plain_d), ("ring", ring_d)):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run(sc, K, ev)
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) / K * 1e3)
            res[name + "_k"].append(sum(a.elapsed_time(b) for a, b in ev.values()) / len(ev))
    ctx.steps_flush(torch.zeros(1, dtype=torch.int64, device=dev))  # discard
    plain_ms, ring_ms = min(res["plain"]), min(res["ring"])
    ring_kms = sum(res["ring_k"]) / len(res["ring_k"])
    plain_kms = sum(res["plain_k"]) / len(res["plain_k"])
    # the comparator: the rows through the band's widest part, GPU vs CPU
    lib = _cpu_lib()
    rows = list(range(H // 2 - 8, H // 2 + 8))
    n = len(rows)
    sky_c = np.ascontiguousarray(sky, dtype=np.uint8)
    c_rgba = np.empty((n, W, 4), np.uint8)
    c_mask = np.empty((n, W), np.uint8)
    c_uv = np.empty((n, W, 2), np.float32)
    c_steps = np.empty((n, W), np.uint32)
    tot = ctypes.c_ulonglong()
    rc = lib.geo_render_cpu(ctypes.addressof(frame), ctypes.addressof(ring), sky_c.ctypes.data, sky_c.shape[1],
                            sky_c.shape[0], None, 0, W, H, rows[0], n, 1, 16, c_rgba.ctypes.data, c_mask.ctypes.data,
                            c_uv.ctypes.data, c_steps.ctypes.data, ctypes.addressof(tot))
    if rc != 0:
        raise SystemExit(f"geo_render_cpu (ring): {rc}")
    g_rgba = torch.empty(H * W * 4, dtype=torch.uint8, device=dev)
    g_mask = torch.empty(H * W, dtype=torch.uint8, device=dev)
    g_uv = torch.empty(H * W * 2, dtype=torch.float32, device=dev)
    g_steps = torch.empty(H * W, dtype=torch.int32, device=dev)
    ctx.render_rows(frame, ring, W, H, 0, H, g_rgba, out_mask=g_mask, out_uv=g_uv, out_steps=g_steps)
    torch.cuda.synchronize()
    sl = slice(rows[0], rows[0] + n)
    same = (np.array_equal(g_rgba.view(H, W, 4)[sl].cpu().numpy(), c_rgba)
            and np.array_equal(g_mask.view(H, W)[sl].cpu().numpy(), c_mask)
            and np.array_equal(g_uv.view(H, W, 2)[sl].cpu().numpy().view(np.uint32), c_uv.view(np.uint32))
            and np.array_equal(g_steps.view(H, W)[sl].cpu().numpy().view(np.uint32), c_steps))
    # the rows' band pixels: where the f64 path changed the steps or the UV
    p_uv = torch.empty(H * W * 2, dtype=torch.float32, device=dev)
    p_steps = torch.empty(H * W, dtype=torch.int32, device=dev)
    plain = flagged(0)
    ctx.render_rows(frame, plain, W, H, 0, H, out, out_uv=p_uv, out_steps=p_steps)
    torch.cuda.synchronize()
    changed = int(((g_steps != p_steps) | (g_uv.view(-1, 2) != p_uv.view(-1, 2)).any(dim=1)).sum().item())
    achieved = flops / (ring_kms * 1e-3) / 1e12
    return {
        "ms_per_step": ring_ms,
        "plain_ms_per_step": plain_ms,
        "overhead": ring_ms / plain_ms - 1.0,
        "kernel_ms": ring_kms,
        "plain_kernel_ms": plain_kms,
        "kernel_overhead": ring_kms / plain_kms - 1.0,
        "value": ring_steps / (ring_ms * 1e-3),
        "unit": "geodesic-steps·pixels/s" if scene.mode != 2 else "geodesic-step-attempts·pixels/s",
        "roofline": {"achieved": achieved, "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / PEAK_FP32_TFLOPS, "algorithmic_flops_per_launch": flops,
                     "what": "the ring frame's algorithmic flops (its band's steps are f64) over its kernel's "
                             "event-timed duration (the whole frame is one launch: the f32 lanes and the f64 "
                             "band's lanes in one kernel)"},
        "reps": {k: [round(v, 5) for v in vals] for k, vals in res.items()},
        "pixels_changed": changed,
        "matches_cpu": {"ok": bool(same), "rows": [rows[0], rows[-1]],
                        "what": "GPU rows vs geo_render_cpu's (geo_band.h on the host) through the band: RGBA, "
                                "mask, UV bits, steps"},
        "what": "GEO_FLAG_RING_F64: the capture band's lanes (|b/b_c - 1| < 5e-3 by the f32 ray) integrate in f64 "
                "inside the render kernel; ms_per_step and plain_ms_per_step are the best of 3 interleaved "
                "runs of `frames` frames each (one launch per frame, one stream; at least the line's K and "
                "about 25 ms of plain frames)",
        "frames": K,
    }


def g_flag_mips() -> int:
    from schwarzschild_raytracer_wgpu_amd import _lib

    return _lib.GEO_FLAG_MIPS


if __name__ == "__main__":
    main()
