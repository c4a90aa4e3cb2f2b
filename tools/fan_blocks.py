#!/usr/bin/env python3
"""VALU per pixel of each block of the fan-mode draw, from the gfx950 device
code (tools/ubench/fan_blocks.hip: each block compiled alone between loads and
stores, minus a pass-through kernel with the same loads and stores).

The correctly rounded sqrt/reciprocal fallbacks (`v_sqrt_f32`,
`v_div_scale_f32` sequences behind a wave-uniform branch that no frame pixel
takes: denormal or huge operands, geo_math.h) are listed apart and not
counted.

    python tools/fan_blocks.py [--asm OUT.s]
"""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

BLOCKS = ["kPass", "kRay", "kCentral", "kFanIndex", "kFanLerp", "kSkyUV", "kSincos", "kAtan2", "kAsin", "kSample",
          "kBlend"]
LABEL = {
    "kRay": "camera ray + aberration (pixel_central_dir: 6 FMA, |d| sqrt, 1/(L - k dz))",
    "kCentral": "sin/cos of the central angle (med3 clamp, rho = sqrt, 1/rho)",
    "kFanIndex": "fan index (acos(st)/pi, index and weight)",
    "kFanLerp": "fan lerp (two loads, lerp)",
    "kSkyUV": "sky UV (sincos of lambda', to_cart, M2, U in turns, V = acos/pi)",
    "kSincos": "  of which sincos (sincos_sky_)",
    "kAtan2": "  of which U (atan2_turns_ + clamp)",
    "kAsin": "  of which V (acos_pi_)",
    "kSample": "bilinear sample (texel coordinates, quad loads, packed lerps)",
    "kBlend": "blend over the clear colour",
}


def compile_asm(out):
    import __graft_entry__ as ge

    flags = [f for f in ge.HIP_FLAGS if f not in ("-shared", "-fPIC")]
    src = os.path.join(ROOT, "tools", "ubench", "fan_blocks.hip")
    subprocess.run([ge.HIPCC, *flags, "--cuda-device-only", "-S", "-o", out, src], check=True,
                   stderr=subprocess.DEVNULL)


def kernels(path):
    """{block enum value index: [instructions]} in program order, labels kept."""
    text = open(path).read().split("\n")
    out, cur = {}, None
    for ln in text:
        m = re.match(r"^(_Z\w*blkILi(\d+)E\w*):", ln)
        if m:
            cur = int(m.group(2))
            out[cur] = []
            continue
        if cur is None:
            continue
        s = ln.split(";")[0].strip()
        if s.startswith(".Lfunc_end"):
            cur = None
            continue
        if not s or (s.startswith(".") and not re.match(r"^\.LBB\w+:", s)):
            continue
        out[cur].append(s)
    return out


def count(ins):
    """(counted VALU, VALU in rare fallback segments)."""
    labels = {s[:-1]: k for k, s in enumerate(ins) if s.endswith(":")}
    rare = set()
    for k, s in enumerate(ins):
        op = s.split()[0]
        if op.startswith("s_cbranch"):
            tgt = s.split()[-1]
            if tgt in labels and labels[tgt] > k:
                seg = ins[k + 1:labels[tgt]]
                ops = {re.sub(r"_e(32|64)$", "", x.split()[0]) for x in seg}
                fallback = "v_div_scale_f32" in ops or ("v_sqrt_f32" in ops and "v_rsq_f32" not in ops)
                if fallback:
                    rare.update(range(k + 1, labels[tgt]))
    valu = [k for k, s in enumerate(ins) if s.split()[0].startswith("v_")]
    return sum(1 for k in valu if k not in rare), sum(1 for k in valu if k in rare)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--asm", default=None)
    a = p.parse_args()
    path = a.asm or os.path.join(tempfile.mkdtemp(), "fan_blocks.s")
    if not a.asm or not os.path.exists(path):
        compile_asm(path)
    ks = kernels(path)
    base = count(ks[0])[0]
    print(f"pass-through (loads, stores, addressing): {base} VALU")
    print(f"{'block':72s} {'VALU':>5s} {'fallback':>8s}")
    total = 0
    for i, b in enumerate(BLOCKS[1:], start=1):
        c, r = count(ks[i])
        v = c - base
        if not LABEL[b].startswith("  "):
            total += v
        print(f"{LABEL[b]:72s} {v:5d} {r:8d}")
    print(f"{'sum of the blocks (per pixel)':72s} {total:5d}")


if __name__ == "__main__":
    main()
