"""The C++ host mirror of the reference's Rust types (include/geo/sr.hpp) and
the reference's own tests through it (tests/native/sr_reference_tests.cpp =
SR/simulation/tests.rs:8-79: same names, loops and 5e-4 tolerances).

CPU: it compiles warning-free against geo.h and links against libgeo.so, and
without a GPU it fails loudly (sr::Error from geo_ctx_create).  GPU: the
tests.rs tests pass; sphere_geodesics_test's fan equals the f64 oracle's
(<= 1 f32 ulp: device vs glibc cos/sin); a Renderer frame of the sky sphere
equals the oracle bit for bit, and with a point cloud it equals the same frame
drawn through the Python host."""
import math
import os
import shutil
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PKG = os.path.join(ROOT, "schwarzschild_raytracer_wgpu_amd")
ROCM = "/opt/rocm"


def build(tmp_path, src=os.path.join(HERE, "native", "sr_reference_tests.cpp")):
    if shutil.which("g++") is None or not os.path.exists(os.path.join(PKG, "libgeo.so")):
        pytest.skip("needs g++ and a built libgeo.so")
    exe = str(tmp_path / os.path.splitext(os.path.basename(src))[0])
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-Werror", "-D__HIP_PLATFORM_AMD__",
                    "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROCM, "include"),
                    src, "-L", PKG, "-lgeo",
                    "-L", os.path.join(ROCM, "lib"), "-lamdhip64", f"-Wl,-rpath,{PKG}",
                    f"-Wl,-rpath,{os.path.join(ROCM, 'lib')}", "-o", exe], check=True)
    return exe


def _has_gpu():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def test_cpp_host_builds(tmp_path):
    build(tmp_path)


def test_cpp_frame_loop_example_builds(tmp_path):
    build(tmp_path, os.path.join(ROOT, "examples", "frame_loop.cpp"))


def test_cpp_host_fails_loudly_without_a_device(tmp_path):
    if _has_gpu():
        pytest.skip("a HIP device is present")
    exe = build(tmp_path)
    r = subprocess.run([exe, "tests"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 3 and "no such HIP device" in r.stderr, (r.returncode, r.stderr)


def fnv1a(b: bytes) -> int:
    h = 1469598103934665603
    for x in np.frombuffer(b, np.uint8).tolist():
        h = ((h ^ x) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


@pytest.mark.gpu
def test_reference_tests_through_cpp_host(tmp_path):
    if not _has_gpu():
        pytest.skip("no HIP device")
    exe = build(tmp_path)
    r = subprocess.run([exe, "tests"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all passed" in r.stdout
    assert "ray_connector_euclidian_test 100/100" in r.stdout
    assert "ray_connector_euclidian_tracing_test 120/120" in r.stdout
    line = next(l for l in r.stdout.splitlines() if l.startswith("sphere_geodesics_test fan"))
    fan = np.array([float.fromhex(t) for t in line.split()[2:]], np.float32)
    import oracle as O

    ref = O.solve_ray_fan(100.0, 10.0, 100, math.pi / 100, 20, 25.0)
    ulp = np.abs(fan.view(np.int32).astype(np.int64) - ref.view(np.int32).astype(np.int64))
    assert fan.shape == (20,) and int(ulp.max()) <= 1, (fan, ref)


@pytest.mark.gpu
def test_cpp_renderer_frames(tmp_path):
    if not _has_gpu():
        pytest.skip("no HIP device")
    exe = build(tmp_path)
    W, H = 160, 90
    r = subprocess.run([exe, "frame", str(W), str(H), str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    got = {l.split(" fnv1a ")[0]: int(l.split(" fnv1a ")[1], 16) for l in r.stdout.splitlines() if "fnv1a" in l}

    import torch

    import oracle as O
    import schwarzschild_raytracer_wgpu_amd as g

    x = np.arange(512, dtype=np.uint32)[None, :]
    y = np.arange(256, dtype=np.uint32)[:, None]
    sky = np.empty((256, 512, 4), np.uint8)
    sky[..., 0] = ((x * 7) ^ (y * 13)) & 0xFF
    sky[..., 1] = (x + y) & 0xFF
    sky[..., 2] = (x * y) & 0xFF
    sky[..., 3] = 255
    obs = g.Observer(1.0, math.pi / 2, W, H)
    obs.set_position(2.5, 0.0, 0.1)
    frame = obs.calc_transformation_pipeline()
    scene = g.make_scene(1.0, 50.0, obs.get_radial_position(), math.pi / 100, 2048)
    ref = O.render_f32(frame, scene, sky, W, H, threads=4)
    assert got["frame sky"] == fnv1a(ref["rgba"].tobytes())

    # the same frame with the point cloud, through the Python host
    model = np.fromfile(str(tmp_path / "model.f32"), dtype=np.float32).reshape(-1, 3)
    sphere = g.BasicSphereBuffer(0, 50.0, 1.0, sky, max_iter=2048)
    sphere.update_ray_fan(obs.get_radial_position())
    pos = obs.get_position()
    cloud = g.PointCloud(sphere.ctx, model, 1.0, pos, True, False)
    cloud.update(pos, 1.0 / 60.0)
    tgt = g.RenderTarget(W, H, torch.empty(W * H * 4, dtype=torch.uint8, device="cuda:0"))
    g.Renderer(obs).render([sphere], tgt, [cloud])
    torch.cuda.synchronize()
    assert got["frame sky+points"] == fnv1a(tgt.rgba.cpu().numpy().tobytes())
    assert got["frame sky+points"] != got["frame sky"]


@pytest.mark.gpu
def test_cpp_frame_loop_runs(tmp_path):
    """examples/frame_loop.cpp: lib.rs's update + render loop from C++ (sky
    sphere + accretion disk), a few frames at a small size."""
    if not _has_gpu():
        pytest.skip("no HIP device")
    exe = build(tmp_path, os.path.join(ROOT, "examples", "frame_loop.cpp"))
    outs = []
    for overlap in ("1", "0"):  # disk update on a side stream / on the render stream
        out = tmp_path / f"f{overlap}.ppm"
        r = subprocess.run([exe, "192", "108", "20", str(out), overlap], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stdout + r.stderr
        assert "frames/s" in r.stdout and out.stat().st_size == len(b"P6\n192 108\n255\n") + 192 * 108 * 3
        outs.append(out.read_bytes())
    assert outs[0] == outs[1]  # the same frame either way (geo_points_draw waits for the update)
