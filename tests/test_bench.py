"""bench.py's contract (the driver parses its one JSON line).

CPU: the committed PMC traffic is attached only to the workload it was taken
on.  GPU: a short run (the driver's own --steps/--warmup shape, fewer spin-up
frames) prints one JSON line with every field the contract names, and its
numbers are consistent with each other.
"""
import json
import os
import subprocess
import sys

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_pmc_profile_only_for_the_profiled_workload():
    t = bench.pmc_profile("cfg3_4k", "direct", 1)[1].get("traffic_bytes")
    assert t is not None and 5e7 < t < 2e8  # ~90 MB per 4K frame
    assert bench.pmc_profile("cfg3_4k", "adaptive", 1) == (None, {})  # a direct-mode profile
    fan = bench.pmc_profile("cfg3_4k", "fan", 1)  # the fan-mode draw's own profile (profiles/*_cfg3_4k_fan_pmc.json)
    assert fan[0] is not None and "fan" in fan[0] and 3e7 < fan[1]["traffic_bytes"] < 2e8
    assert bench.pmc_profile("cfg3_4k", "direct", 2) == (None, {})  # full-frame bytes vs a rank's share
    assert bench.pmc_profile("cfg5_8k_adaptive", "adaptive", 1)[0] is not None
    assert bench.pmc_profile("cfg2_1080p", "direct", 1)[0] is not None
    assert bench.pmc_profile("cfg1_256_cpu", "direct", 1) == (None, {})  # never profiled


@pytest.mark.gpu
def test_bench_short_run_prints_the_contract_line():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "20", "--warmup", "5",
                        "--spinup-frames", "60", "--cpu-row-step", "8"],
                       cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 20 and d["warmup"] == 5 and d["higher_is_better"] is True
    assert d["dtype"] == "f32" and d["vs_baseline"] is None and "workload" in d["config"]
    # value = executed RK4 steps of the timed frames / their wall time
    assert abs(d["value"] - d["steps_per_frame"] / (d["ms_per_step"] * 1e-3)) < 1e-6 * d["value"]
    assert 70 < d["mean_steps_per_pixel"] < 90  # the default scene: 78.0
    rf = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in rf, k
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-9
    assert abs(rf["achieved"] - rf["algorithmic_flops_per_launch"] / (d["kernel_ms"]["avg"] * 1e-3) / 1e12) < 1e-6
    assert 0.3 < rf["frac"] < 1.0
    cb = d["cpu_baseline"]
    assert cb["kind"] == "port" and cb["cores"] >= 1 and cb["value"] > 0 and cb["cpu_model"]
    assert len(cb["seconds_per_run"]) == 3
    # the frames of the timed run's last batch equal a single-launch frame
    assert d["frame_check"]["ok"] is True and d["frame_check"]["frames"] >= 1


def test_rank0_lead_specs_and_trials():
    """--rank0-lead: 'auto', 'a' or 'a:b'; every layout the auto trial tries
    owns each row of the 4K frame exactly once at every N the driver runs."""
    import argparse

    from schwarzschild_raytracer_wgpu_amd.dist import BandLayout

    assert bench._lead_spec("auto") == "auto"
    assert bench._lead_spec("2") == (2, 1)
    assert bench._lead_spec("3:2") == (3, 2)
    for bad in ("0", "1:0", "x", "2:y"):
        with pytest.raises(argparse.ArgumentTypeError):
            bench._lead_spec(bad)
    assert (1, 1) in bench.LEAD_TRIALS and len(set(bench.LEAD_TRIALS)) == len(bench.LEAD_TRIALS)
    for n in (2, 4, 8):
        for a, b in bench.LEAD_TRIALS:
            L = [BandLayout(2160, 8, n, r, a, b) for r in range(n)]
            owned = sorted(x for lay in L for x in lay.local_to_frame_rows() if x >= 0)
            assert owned == list(range(2160)), (n, a, b)
            assert all(lay.band_height() % 8 == 0 for lay in L)  # a wave's rows lie in one band


def test_share_spec_and_motion_frames():
    """--share r/n and --motion: the per-frame uniforms of a moving observer
    follow the reference's Observer (the scene's radius is the observer's)."""
    import argparse

    import schwarzschild_raytracer_wgpu_amd as g
    from schwarzschild_raytracer_wgpu_amd.scenes import CONFIGS

    assert bench._share_spec("1/8") == (1, 8)
    for bad in ("8/8", "1/1", "x/8", "1"):
        with pytest.raises(argparse.ArgumentTypeError):
            bench._share_spec(bad)
    cfg = CONFIGS["cfg3_4k"]
    for kind in ("orbit", "fall", "pan"):
        mv = bench.motion_frames(g, cfg, kind, 30, g.GEO_MODE_DIRECT, 0, 0.0)
        assert len(mv) == 30
        frames = {bytes(f) for f, _ in mv}
        assert len(frames) == 30, kind  # every frame its own uniform
        radii = [sc.r_obs for _, sc in mv]
        if kind == "pan":
            assert len(set(radii)) == 1
        else:
            assert len(set(radii)) == 30 and all(r > cfg.rs for r in radii)
        for fr, sc in mv:  # the uniform's position is the scene's radius
            x, y, z = fr.psi_factor_and_position[1:]
            assert abs((x * x + y * y + z * z) ** 0.5 - sc.r_obs) < 1e-5
    fall = [sc.r_obs for _, sc in bench.motion_frames(g, cfg, "fall", 60, g.GEO_MODE_DIRECT, 0, 0.0)]
    assert all(b < a for a, b in zip(fall, fall[1:]))  # falling in


def test_batch_key_groups_a_moving_observer():
    """dist._batch_key: frames that differ in the radius only share a batched
    launch (on one side of the horizon; fan mode: one fan, one radius)."""
    import schwarzschild_raytracer_wgpu_amd as g
    from schwarzschild_raytracer_wgpu_amd.dist import _batch_key

    def sc(r, budget=512, mode=g.GEO_MODE_DIRECT):
        return g.make_scene(1.0, 50.0, r, 0.0314, budget, mode)

    assert _batch_key(sc(2.5)) == _batch_key(sc(2.4))
    assert _batch_key(sc(2.5)) != _batch_key(sc(2.5, budget=256))
    assert _batch_key(sc(2.5)) != _batch_key(sc(0.9))       # across the horizon: another integration
    assert _batch_key(sc(0.8)) == _batch_key(sc(0.9))
    assert _batch_key(sc(2.5, mode=g.GEO_MODE_FAN)) != _batch_key(sc(2.4, mode=g.GEO_MODE_FAN))


@pytest.mark.gpu
def test_bench_two_ranks_gloo_frame_check():
    """The N > 1 bench path on one GPU (two ranks share it over gloo, as the
    rehearsals do): the self-launcher, the lead trials, batched launches and
    rank 0's assembled frames equal to the single-launch frame."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                        "--config", "cfg2_1080p", "--steps", "8", "--warmup", "2", "--spinup-frames", "4",
                        "--lead-trial-frames", "8", "--frames-per-gather", "2"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["world_size"] == 2 and d["dist_backend"] == "gloo"
    assert d["config"]["frames_per_launch"] == 2 and len(d["config"]["lead_trials_ms_per_frame"]) == 8
    assert d["frame_check"]["ok"] is True and d["frame_check"]["ranks"] == 2
    assert sum(d["per_rank"]["rows"]) == 1080
