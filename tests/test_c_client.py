"""The C-ABI from plain C (examples/render_frame.c: no Python, no torch; HIP's
C runtime API only for device memory).  CPU: it compiles and links against
libgeo.so.  GPU: the frame it renders equals the oracle's bit for bit (FNV-1a
of the RGBA8 frame)."""
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


def build(tmp_path):
    if shutil.which("gcc") is None or not os.path.exists(os.path.join(PKG, "libgeo.so")):
        pytest.skip("needs gcc and a built libgeo.so")
    exe = str(tmp_path / "render_frame")
    subprocess.run(["gcc", "-std=c99", "-O2", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__",
                    "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROCM, "include"),
                    os.path.join(ROOT, "examples", "render_frame.c"), "-L", PKG, "-lgeo",
                    "-L", os.path.join(ROCM, "lib"), "-lamdhip64", "-lm", f"-Wl,-rpath,{PKG}",
                    f"-Wl,-rpath,{os.path.join(ROCM, 'lib')}", "-o", exe], check=True)
    return exe


def test_c_client_builds(tmp_path):
    build(tmp_path)


def fnv1a(b: bytes) -> int:
    h = 1469598103934665603
    for x in b:
        h = ((h ^ x) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


@pytest.mark.gpu
def test_c_client_frame_equals_oracle(tmp_path):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    exe = build(tmp_path)
    W, H = 192, 108
    r = subprocess.run([exe, str(tmp_path / "f.ppm"), str(W), str(H)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    got = int(r.stdout.split("fnv1a")[1].strip(), 16)

    import oracle as O
    from schwarzschild_raytracer_wgpu_amd import Observer, make_scene

    x = np.arange(512, dtype=np.uint32)[None, :]
    y = np.arange(256, dtype=np.uint32)[:, None]
    sky = np.empty((256, 512, 4), np.uint8)
    sky[..., 0] = ((x * 7) ^ (y * 13)) & 0xFF
    sky[..., 1] = (x + y) & 0xFF
    sky[..., 2] = (x * y) & 0xFF
    sky[..., 3] = 255
    o = Observer(1.0, math.pi / 2, W, H)
    o.set_position(2.5, 0.0, 0.1)
    o.start_frozen_fall()
    frame = o.calc_transformation_pipeline()
    scene = make_scene(1.0, 50.0, o.get_radial_position(), math.pi / 100, 2048)
    ref = O.render_f32(frame, scene, sky, W, H, threads=4)
    assert got == fnv1a(ref["rgba"].tobytes())
    assert f"steps {ref['steps_total']}" in r.stdout
