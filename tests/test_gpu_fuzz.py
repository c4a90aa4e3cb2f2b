"""Fuzz parity on the GPU: the HIP kernels (through the C-ABI) equal the
oracle's f32 restatement bit for bit (mask, UV bits, steps, RGBA) on seeded
random scenes (tests/fuzz_scenes.py), direct and adaptive, 64x36 each; the
batched band-set launch on random batches and layouts (test_gpu_fuzz_batch_bitexact)."""
import os

import numpy as np
import pytest

import oracle as O
from fuzz_scenes import REGRESSION_SEEDS, adversarial_scene, random_scene
from test_gpu_parity import geo, make_ctx, render, torch_mod  # noqa: F401  (fixtures)

pytestmark = pytest.mark.gpu

W, H = int(os.environ.get("GEO_FUZZ_W", 64)), int(os.environ.get("GEO_FUZZ_H", 36))


@pytest.mark.parametrize("adaptive", [False, True], ids=["direct", "adaptive"])
def test_gpu_fuzz_bitexact(geo, torch_mod, adaptive):  # noqa: F811
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    sky = make_sky("equirect", (256, 128))
    ctx = make_ctx(geo, sky)
    bad = []
    # GEO_FUZZ_N / GEO_FUZZ_BASE: a longer sweep on other seeds (default: the committed 600 + 300)
    n = int(os.environ.get("GEO_FUZZ_N", 600 if not adaptive else 300))
    base = int(os.environ.get("GEO_FUZZ_BASE", 10_000))
    seeds = [base + i for i in range(n)] + ([] if adaptive else list(REGRESSION_SEEDS))
    for seed in seeds:
        frame, scene, desc = random_scene(seed, W, H, adaptive=adaptive)
        hip = render(geo, torch_mod, ctx, frame, scene, W, H)
        ref = O.render_f32(frame, scene, sky, W, H, threads=4)
        same = all(np.array_equal(hip[f], ref[f]) for f in ("mask", "steps", "rgba")) and np.array_equal(
            hip["uv"].view(np.uint32), ref["uv"].view(np.uint32)) and hip["total"] == ref["steps_total"]
        if not same:
            bad.append(desc)
    print(f"fuzz {'adaptive' if adaptive else 'direct'}: {len(seeds)} scenes at {W}x{H}, {len(bad)} differ")
    assert not bad, f"{len(bad)} of {len(seeds)} scenes differ: {bad[:5]}"


@pytest.mark.parametrize("adaptive", [False, True], ids=["direct", "adaptive"])
def test_gpu_fuzz_adversarial_bitexact(geo, torch_mod, adaptive):  # noqa: F811
    """Near-radial outgoing rays and falling rays at large steps
    (fuzz_scenes.adversarial_scene: steps 0.01..3, budgets 1..4096): the
    exact group exit test against the oracle's literal per-step loop."""
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    sky = make_sky("equirect", (256, 128))
    ctx = make_ctx(geo, sky)
    bad = []
    n = int(os.environ.get("GEO_FUZZ_N", 400 if not adaptive else 200))
    base = int(os.environ.get("GEO_FUZZ_BASE", 0))
    for seed in range(base, base + n):
        frame, scene, desc = adversarial_scene(seed, W, H, adaptive=adaptive)
        hip = render(geo, torch_mod, ctx, frame, scene, W, H)
        ref = O.render_f32(frame, scene, sky, W, H, threads=4)
        same = all(np.array_equal(hip[f], ref[f]) for f in ("mask", "steps", "rgba")) and np.array_equal(
            hip["uv"].view(np.uint32), ref["uv"].view(np.uint32)) and hip["total"] == ref["steps_total"]
        if not same:
            bad.append(desc)
    print(f"fuzz adversarial {'adaptive' if adaptive else 'direct'}: {n} scenes at {W}x{H}, {len(bad)} differ")
    assert not bad, f"{len(bad)} of {n} scenes differ: {bad[:5]}"


def test_gpu_fuzz_fan_mode_bitexact(geo, torch_mod):  # noqa: F811
    """Fan mode (the reference's display path) on the fuzz scenes: each
    scene's 400-node fan solved on the GPU, drawn with the fan lerp, and the
    oracle's f32 lerp over the same fan: mask, UV bits and RGBA equal, and the
    colour-only draw (two pixels per lane) equal to the same RGBA."""
    from schwarzschild_raytracer_wgpu_amd import _lib
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    torch = torch_mod
    sky = make_sky("equirect", (256, 128))
    ctx = make_ctx(geo, sky)
    dev = torch.device("cuda:0")
    n = int(os.environ.get("GEO_FUZZ_N", 300))
    base = int(os.environ.get("GEO_FUZZ_BASE", 10_000))
    bad = []
    for seed in range(base, base + n):
        frame, scene, desc = random_scene(seed, W, H)
        scene.mode = _lib.GEO_MODE_FAN
        fan = ctx.solve_ray_fan(scene.sphere_r, scene.rs, 1000, scene.step, 400, scene.r_obs)
        rgba = torch.empty(W * H * 4, dtype=torch.uint8, device=dev)
        mask = torch.empty(W * H, dtype=torch.uint8, device=dev)
        uv = torch.empty(W * H * 2, dtype=torch.float32, device=dev)
        ctx.render_rows(frame, scene, W, H, 0, H, rgba, mask, uv)
        torch.cuda.synchronize()
        plain = torch.empty(W * H * 4, dtype=torch.uint8, device=dev)
        ctx.render_rows(frame, scene, W, H, 0, H, plain)
        torch.cuda.synchronize()
        ref = O.render_f32(frame, scene, sky, W, H, fan=fan, threads=4)
        same = (np.array_equal(mask.cpu().numpy().reshape(H, W), ref["mask"])
                and np.array_equal(rgba.cpu().numpy().reshape(H, W, 4), ref["rgba"])
                and np.array_equal(plain.cpu().numpy().reshape(H, W, 4), ref["rgba"])
                and np.array_equal(uv.cpu().numpy().reshape(H, W, 2).view(np.uint32), ref["uv"].view(np.uint32)))
        if not same:
            bad.append(desc)
    print(f"fuzz fan: {n} scenes at {W}x{H}, {len(bad)} differ")
    assert not bad, f"{len(bad)} of {n} scenes differ: {bad[:5]}"


def test_gpu_fuzz_mips_bitexact(geo, torch_mod):  # noqa: F811
    """GEO_FLAG_MIPS on the fuzz scenes (ragged 65 x 37 frames: helper lanes
    on the right and bottom quads) with random sky sizes down to 1 x 1, in
    direct, adaptive and fan mode: the oracle's mip restatement, bit for
    bit."""
    from schwarzschild_raytracer_wgpu_amd import _lib

    w, h = W + 1, H + 1
    n = int(os.environ.get("GEO_FUZZ_N", 200))
    base = int(os.environ.get("GEO_FUZZ_BASE", 20_000))
    bad = []
    ctx = geo.Context(0)
    for seed in range(base, base + n):
        rng = np.random.default_rng(seed)
        sw, sh = int(rng.integers(1, 300)), int(rng.integers(1, 160))
        sky = rng.integers(0, 256, size=(sh, sw, 4), dtype=np.uint8)
        if seed % 2:
            sky[..., 3] = 255
        ctx.set_sky(sky)
        frame, scene, desc = random_scene(seed, w, h, adaptive=seed % 3 == 0)
        scene.flags |= _lib.GEO_FLAG_MIPS
        fan = None
        if seed % 3 == 1:
            scene.mode = _lib.GEO_MODE_FAN
            fan = ctx.solve_ray_fan(scene.sphere_r, scene.rs, 1000, scene.step, 400, scene.r_obs)
        hip = render(geo, torch_mod, ctx, frame, scene, w, h)
        ref = O.render_mips_f32(frame, scene, sky, w, h, fan=fan, threads=4)
        same = all(np.array_equal(hip[f], ref[f]) for f in ("mask", "steps", "rgba")) and np.array_equal(
            hip["uv"].view(np.uint32), ref["uv"].view(np.uint32)) and hip["total"] == ref["steps_total"]
        if not same:
            bad.append((desc, (sw, sh)))
    print(f"fuzz mips: {n} scenes at {w}x{h}, {len(bad)} differ")
    assert not bad, f"{len(bad)} of {n} scenes differ: {bad[:5]}"


def test_gpu_fuzz_batch_bitexact(geo, torch_mod):  # noqa: F811
    """geo_render_band_set_batch on seeded random batches: ragged frames,
    1..8 frames per launch, each frame's own uniform and observer radius
    (same side of the horizon; one radius in fan mode), random band layouts
    (world 1..8, any rank, rank 0's taller bands), a gap between frames,
    GEO_FLAG_RING_F64 on half the direct/adaptive batches.  Every frame's packed bands == geo_render_band_set of that frame alone
    (bytes, the gap untouched, step totals), and one frame per batch ==
    the oracle's f32 restatement on its rows."""
    from schwarzschild_raytracer_wgpu_amd import _lib
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    torch = torch_mod
    dev = torch.device("cuda:0")
    sky = make_sky("equirect", (256, 128))
    ctx = make_ctx(geo, sky)
    stream = torch.cuda.current_stream().cuda_stream
    n_seeds = int(os.environ.get("GEO_FUZZ_N", 400))
    base = int(os.environ.get("GEO_FUZZ_BASE", 30_000))
    bad = []
    for seed in range(base, base + n_seeds):
        rng = np.random.default_rng(seed)
        w, h = int(rng.integers(20, 130)), int(rng.integers(9, 90))
        mode = (_lib.GEO_MODE_DIRECT, _lib.GEO_MODE_ADAPTIVE, _lib.GEO_MODE_FAN)[seed % 3]
        frame0, scene0, desc = random_scene(seed, w, h, adaptive=mode == _lib.GEO_MODE_ADAPTIVE)
        scene0.mode = mode
        n = int(rng.integers(1, _lib.GEO_MAX_BATCH_FRAMES + 1))
        frames, scenes = [frame0], [scene0]
        for f in range(1, n):
            frames.append(random_scene(seed * 16 + f + 1_000_000, w, h)[0])
            s = geo.GeoScene.from_buffer_copy(bytes(scene0))
            if mode != _lib.GEO_MODE_FAN:
                r = scene0.r_obs * float(rng.uniform(0.9, 1.1))
                if scene0.r_obs < scene0.rs:  # stay inside the horizon
                    r = min(r, 0.995 * scene0.rs)
                elif scene0.r_obs > scene0.rs:
                    r = max(r, 1.005 * scene0.rs)
                s.r_obs = r
            scenes.append(s)
        # GEO_FLAG_RING_F64 on every frame of half the direct/adaptive batches
        # (each frame's band factor in the batch, its constants derived on the device)
        ring = (mode != _lib.GEO_MODE_FAN and rng.random() < 0.5
                and (scene0.flags & (_lib.GEO_FLAG_COMPOSITE | _lib.GEO_FLAG_MIPS)) == 0)
        if ring:
            for s in scenes:
                s.flags |= _lib.GEO_FLAG_RING_F64
        fan = None
        if mode == _lib.GEO_MODE_FAN:
            fan = ctx.solve_ray_fan(scene0.sphere_r, scene0.rs, 1000, scene0.step, 400, scene0.r_obs)
        world = int(rng.integers(1, 9))
        band = 8 * int(rng.choice([1, 2, 3]))  # band heights: multiples of 8 (geo.h)
        lead = band * int(rng.integers(1, 3)) if rng.random() < 0.7 else 8 * int(rng.integers(1, band // 4 + 1))
        rank = int(rng.integers(0, world))
        row_stride = lead + (world - 1) * band
        row0, band_h = (0, lead) if rank == 0 else (lead + (rank - 1) * band, band)
        if row0 >= h:
            row0, band_h, rank = 0, lead, 0
        nbands = (h - row0 + row_stride - 1) // row_stride
        packed = nbands * band_h * w * 4
        stride = packed + 4 * int(rng.integers(0, 10))
        out = torch.full((n * stride,), 7, dtype=torch.uint8, device=dev)
        tot = torch.zeros(1, dtype=torch.int64, device=dev)
        fa, sa = (geo.GeoFrame * n)(*frames), (geo.GeoScene * n)(*scenes)
        st = _lib.lib.geo_render_band_set_batch(ctx._h, fa, sa, n, w, h, band_h, row0, row_stride, nbands,
                                                out.data_ptr(), stride, tot.data_ptr(), stream)
        layout = (f"n={n} world={world} rank={rank} band={band_h} row0={row0} stride={row_stride} nbands={nbands}"
                  f" ring={ring}")
        if st != _lib.GEO_OK:
            bad.append((desc, layout, f"status {st}"))
            continue
        ref_tot = torch.zeros(1, dtype=torch.int64, device=dev)
        same = True
        for f in range(n):
            ref = torch.full((packed,), 7, dtype=torch.uint8, device=dev)
            ctx.render_band_set(frames[f], scenes[f], w, h, band_h, row0, row_stride, nbands, ref,
                                steps_total=ref_tot)
            got = out[f * stride:(f + 1) * stride]
            same = same and torch.equal(got[:packed], ref) and bool((got[packed:] == 7).all())
        torch.cuda.synchronize()
        if mode != _lib.GEO_MODE_FAN:
            same = same and int(tot.item()) == int(ref_tot.item())
        # one frame of the batch against the oracle, on the rows its bands hold
        f = int(rng.integers(0, n))
        o = O.render_f32(frames[f], scenes[f], sky, w, h, fan=fan, threads=4)["rgba"]
        got = out[f * stride:f * stride + packed].cpu().numpy().reshape(-1, w, 4)
        for k, y in enumerate(y for j in range(nbands) for y in range(row0 + j * row_stride,
                                                                        row0 + j * row_stride + band_h)):
            if y < h and not np.array_equal(got[k], o[y]):
                same = False
                break
        if not same:
            bad.append((desc, layout))
    print(f"fuzz batch: {n_seeds} batches, {len(bad)} differ")
    assert not bad, f"{len(bad)} of {n_seeds} batches differ: {bad[:3]}"
