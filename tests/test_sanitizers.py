"""SURVEY.md §5 (sanitizers): the product's host-compilable code — the
per-pixel and point-path headers and the observer — built with
-fsanitize=address,undefined and run against the oracle on small frames
(tests/native/sanitize_main.cpp).  GPU sanitizers are not available on the
MI355X pool (host code only).  CPU only."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None, reason="needs gcc/g++")
def test_asan_ubsan_host_paths(tmp_path):
    exe = str(tmp_path / "sanitize_main")
    flags = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
             "-ffp-contract=off", "-mfma", "-msse4.1"]
    objs = []
    for c in ("geo_oracle.c", "geo_oracle_points.c"):
        o = str(tmp_path / (c + ".o"))
        subprocess.run(["gcc", "-std=gnu11", *flags, "-c", os.path.join(ROOT, "oracle", c), "-o", o], check=True)
        objs.append(o)
    subprocess.run(["g++", "-std=c++17", *flags, os.path.join(HERE, "native", "sanitize_main.cpp"),
                    os.path.join(ROOT, "schwarzschild_raytracer_wgpu_amd", "csrc", "observer.cpp"), *objs,
                    "-o", exe, "-lpthread", "-lm"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300,
                       env={**os.environ, "ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1"})
    assert r.returncode == 0, r.stdout + r.stderr
    assert "clean and bit-identical" in r.stdout
