"""Synthetic inputs for the BASELINE.json configs.

The reference's default scene (rs = 10, sphere 500, observer (25, 0, 1),
camera (PI, 0), fov PI/2, FrozenFall with E = 1: renderer.rs:83-85,
lib.rs:72, observer.rs:70-81) is scale-invariant in rs (the RK4 step is an
angle), so the configs use it divided by 10: rs = 1, sphere 50, observer
(2.5, 0, 0.1).  The sky textures of the reference (.MISSING_LARGE_BLOBS) are
absent; configs 2-5 use a synthetic equirect checkerboard with xorshift noise.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np


@dataclass(frozen=True)
class SceneConfig:
    name: str
    width: int
    height: int
    max_steps: int
    rs: float = 1.0
    sphere_r: float = 50.0
    position: tuple = (2.5, 0.0, 0.1)
    camera: tuple = (math.pi, 0.0)
    fov: float = math.pi / 2
    energy: float = 1.0
    state: int = 1  # GEO_OBSERVER_FROZEN_FALL
    step: float = math.pi / 100.0
    sky: str = "equirect"  # or "flat"
    sky_size: tuple = (4096, 2048)
    mode: str = "direct"  # "direct" (per-pixel fixed RK4), "fan" (reference-exact), "adaptive" (RK5(4))
    tol: float = 0.0      # adaptive mode: local error tolerance in u (0 = 1e-6)
    extra: dict = field(default_factory=dict)


CONFIGS = {
    "cfg1_256_cpu": SceneConfig("cfg1_256_cpu", 256, 256, 128, sky="flat", sky_size=(1, 1)),
    "cfg2_1080p": SceneConfig("cfg2_1080p", 1920, 1080, 512),
    "cfg3_4k": SceneConfig("cfg3_4k", 3840, 2160, 2048),
    "cfg4_4k_8gpu": SceneConfig("cfg4_4k_8gpu", 3840, 2160, 2048),
    # config 5 (a build extension): 8K, error-controlled Dormand-Prince RK5(4)
    # steps (tol 1e-6 in u, budget 2048 attempts), observer off-axis at
    # r = 1.3 rs (inside the photon sphere; (1.2, 0.5, 0) has |pos| = 1.3
    # exactly), camera (PI + 0.6, 0.3)
    "cfg5_8k_adaptive": SceneConfig("cfg5_8k_adaptive", 7680, 4320, 2048, position=(1.2, 0.5, 0.0),
                                    camera=(math.pi + 0.6, 0.3), mode="adaptive", tol=1e-6),
}

FLAT_COLOUR = (64, 128, 255, 255)


def xorshift32(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint32, copy=True)
    x ^= (x << np.uint32(13))
    x ^= (x >> np.uint32(17))
    x ^= (x << np.uint32(5))
    return x


def make_sky(kind: str = "equirect", size=(4096, 2048), seed: int = 0x5C4A) -> np.ndarray:
    """(h, w, 4) uint8.  'flat' = one colour; 'equirect' = 8 deg x 8 deg
    lat/long checkerboard plus per-texel xorshift noise (seed 0x5C4A)."""
    w, h = size
    if kind == "flat":
        sky = np.empty((h, w, 4), dtype=np.uint8)
        sky[:] = np.array(FLAT_COLOUR, dtype=np.uint8)
        return sky
    lon = (np.arange(w, dtype=np.float64) + 0.5) / w * 360.0
    lat = (np.arange(h, dtype=np.float64) + 0.5) / h * 180.0
    cell = ((np.floor(lat / 8.0)[:, None] + np.floor(lon / 8.0)[None, :]) % 2).astype(np.int32)
    idx = np.arange(w * h, dtype=np.uint32).reshape(h, w)
    noise = xorshift32(xorshift32(idx ^ np.uint32(seed)) + np.uint32(0x9E3779B9))
    n = (noise & np.uint32(63)).astype(np.int32) - 32
    base_a = np.array([200, 170, 90], dtype=np.int32)
    base_b = np.array([30, 60, 140], dtype=np.int32)
    rgb = np.where(cell[..., None] == 1, base_a, base_b) + n[..., None]
    sky = np.empty((h, w, 4), dtype=np.uint8)
    sky[..., :3] = np.clip(rgb, 0, 255).astype(np.uint8)
    sky[..., 3] = 255
    return sky
