"""Device math that must equal hipcc's correctly rounded builtins bit for bit,
over all 2^32 inputs on the GPU (built here with hipcc for gfx950):
geo::sqrtf_ against __builtin_sqrtf (tests/native/sqrt_exhaustive.hip) and
geo::rcpf_ against 1.0f / x (tests/native/rcp_exhaustive.hip), geo::sqrt_unit_
against sqrtf(fmaxf(x, 2^-96)) on [0, 1] (tests/native/sqrt_unit_exhaustive.hip); and the sky
UV clamp (one v_med3_f32: NaN -> 0, [0, 1]) against its rule on the bit
pattern (tests/native/clamp_exhaustive.hip)."""
import os
import shutil
import subprocess

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def test_sqrt_exhaustive(tmp_path):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    if not (os.path.exists(HIPCC) or shutil.which("hipcc")):
        pytest.skip("no hipcc")
    exe = str(tmp_path / "sqrt_exhaustive")
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-gpu-flush-denormals-to-zero",
                    os.path.join(HERE, "native", "sqrt_exhaustive.hip"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "mismatches 0" in r.stdout, r.stdout + r.stderr


def test_rcp_exhaustive(tmp_path):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    if not (os.path.exists(HIPCC) or shutil.which("hipcc")):
        pytest.skip("no hipcc")
    exe = str(tmp_path / "rcp_exhaustive")
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-gpu-flush-denormals-to-zero",
                    os.path.join(HERE, "native", "rcp_exhaustive.hip"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "mismatches 0" in r.stdout, r.stdout + r.stderr


def test_uv_clamp_exhaustive(tmp_path):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    if not (os.path.exists(HIPCC) or shutil.which("hipcc")):
        pytest.skip("no hipcc")
    exe = str(tmp_path / "clamp_exhaustive")
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-gpu-flush-denormals-to-zero",
                    os.path.join(HERE, "native", "clamp_exhaustive.hip"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "mismatches 0" in r.stdout, r.stdout + r.stderr


def test_cvt_flr_and_sincos_shifter_exhaustive(tmp_path):
    """geo::floor_i32_ (v_cvt_flr_i32_f32) and sincosf_'s shifter rounding
    against floorf/rintf over their whole input domains on the GPU
    (tests/native/flr_exhaustive.hip)."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    if not (os.path.exists(HIPCC) or shutil.which("hipcc")):
        pytest.skip("no hipcc")
    exe = str(tmp_path / "flr_exhaustive")
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-gpu-flush-denormals-to-zero",
                    os.path.join(HERE, "native", "flr_exhaustive.hip"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "mismatches 0" in r.stdout, r.stdout + r.stderr


def test_sqrt_unit_exhaustive(tmp_path):
    """geo::sqrt_unit_ (acos_pi_'s branch-free sqrt) equals the correctly
    rounded sqrtf(fmaxf(x, 2^-96)) for every f32 x in [0, 1]
    (tests/native/sqrt_unit_exhaustive.hip)."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    if not (os.path.exists(HIPCC) or shutil.which("hipcc")):
        pytest.skip("no hipcc")
    exe = str(tmp_path / "sqrt_unit_exhaustive")
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-gpu-flush-denormals-to-zero",
                    os.path.join(HERE, "native", "sqrt_unit_exhaustive.hip"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "mismatches 0" in r.stdout, r.stdout + r.stderr
