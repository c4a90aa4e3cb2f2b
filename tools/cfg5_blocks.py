"""Config 5's VALU budget per wave by block (VERDICT r03 "next" 5): where the
adaptive kernel's instructions go, and the roofline fraction each block
costs.

Static VALU per block from the device asm (tools/isa.sh + isa_blocks.py,
grouped by hand into set-up / attempt loop / Newton crossing / sky epilogue /
step counter), times how often a wave runs it, from the frame itself: every
pixel's attempts and mask of sampled 16 x 4 wave blocks (geo_render_cpu,
bit-identical to the kernel).  A wave runs the set-up once, the loop body as
many times as its slowest lane attempts, Newton if any lane crosses the
sphere, the epilogue unless every lane is a black-hole pixel.

    python tools/cfg5_blocks.py [asm.s] [group_stride]
"""
import ctypes
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools")]
import isa_blocks as IB  # noqa: E402
import schwarzschild_raytracer_wgpu_amd as g  # noqa: E402
from schwarzschild_raytracer_wgpu_amd.scenes import CONFIGS, make_sky  # noqa: E402

SYM = "geo_render_kernelILi2ELi0ELb0ELj1ELb0E"


# the correctly rounded sqrt/reciprocal/division fix-ups (geo_math.h) sit in
# blocks of their own behind a uniform branch that no frame pixel takes
# (denormal or huge operands only): not counted as executed
RARE = ("v_div_scale_f32", "v_sqrt_f32", "v_div_fixup_f32")


def block_valu(path):
    bl = IB.blocks(IB.kernel_lines(path, SYM))
    out = []
    for name, ins in bl:
        v = [i for i in ins if IB.klass(i) == "valu"]
        # a block's rare tail starts at its first fix-up op's operand set-up: count up to the branch before it
        cut = next((k for k, i in enumerate(ins) if i.split()[0] in ("v_div_scale_f32", "v_sqrt_f32")), None)
        if cut is not None:
            head = ins[:cut]
            br = max((k for k, i in enumerate(head) if i.startswith("s_cbranch")), default=None)
            v = [i for i in (head if br is None else head[:br + 1]) if IB.klass(i) == "valu"]
            # the ops between the skipped branch and the fix-up belong to it
            if br is None:
                v = [i for i in head if IB.klass(i) == "valu"]
        out.append((name, len(v)))
    return out


def groups(bv):
    """Blocks in program order: set-up up to the loop, loop body (the blocks
    with the back edge and the two before it), Newton (until the epilogue's
    sincos reduction: 0x3ea2f983 = 1/pi since round 6, 0x3f22f983 = 2/pi
    before), epilogue, step counter/cost tail."""
    names = [n for n, _ in bv]
    valu = dict(bv)
    lines = IB.kernel_lines(sys.argv[1] if len(sys.argv) > 1 else "/tmp/new.s", SYM)
    text = {n: ins for n, ins in IB.blocks(lines)}
    loop_end = next(i for i, n in enumerate(names) if any(x.startswith("s_cbranch_scc1") and names[i - 2] in x
                                                           for x in text[n]))
    loop = names[loop_end - 2:loop_end + 1]
    epi0 = next(i for i, n in enumerate(names) if any("0x3ea2f983" in x or "0x3f22f983" in x for x in text[n]))
    tail0 = next(i for i, n in enumerate(names) if any("row_shr:1" in x for x in text[n]))
    setup = [n for n in names[:loop_end - 2] if n not in loop]
    newton = [n for n in names[loop_end + 1:epi0]]
    epi = names[epi0:tail0]
    tail = names[tail0:]
    return {k: (v, sum(valu[n] for n in v)) for k, v in
            dict(setup=setup, loop=loop, newton=newton, epilogue=epi, tail=tail).items()}


def frame_waves(stride):
    cfg = CONFIGS["cfg5_8k_adaptive"]
    W, H = cfg.width, cfg.height
    obs = g.Observer(cfg.rs, cfg.fov, W, H)
    obs.set_position(*cfg.position)
    obs.set_camera(*cfg.camera)
    obs.set_energy(cfg.energy)
    frame = obs.calc_transformation_pipeline()
    scene = g.make_scene(cfg.rs, cfg.sphere_r, obs.get_radial_position(), cfg.step, cfg.max_steps,
                         g.GEO_MODE_ADAPTIVE, tol=cfg.tol)
    lib = ctypes.CDLL(os.path.join(ROOT, "schwarzschild_raytracer_wgpu_amd", "libgeo_cpu.so"))
    vp, u32 = ctypes.c_void_p, ctypes.c_uint32
    lib.geo_render_cpu.argtypes = [vp, vp, vp, u32, u32, vp, u32, u32, u32, u32, u32, u32, ctypes.c_int, vp, vp, vp,
                                   vp, vp]
    sky = np.ascontiguousarray(make_sky("equirect", (64, 32)))
    steps, mask = [], []
    for gy in range(stride // 2, H // 4, stride):
        rgba = np.empty((4, W, 4), np.uint8)
        m = np.empty((4, W), np.uint8)
        st = np.empty((4, W), np.uint32)
        rc = lib.geo_render_cpu(ctypes.addressof(frame), ctypes.addressof(scene), sky.ctypes.data, sky.shape[1],
                                sky.shape[0], None, 0, W, H, 4 * gy, 4, 1, 8, rgba.ctypes.data, m.ctypes.data, None,
                                st.ctypes.data, None)
        assert rc == 0
        steps.append(st.reshape(4, W // 16, 16).transpose(1, 0, 2).reshape(-1, 64))
        mask.append(m.reshape(4, W // 16, 16).transpose(1, 0, 2).reshape(-1, 64))
    return np.concatenate(steps), np.concatenate(mask)


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else "/tmp/new.s"
    stride = int(sys.argv[2]) if len(sys.argv) > 2 else 27
    gr = groups(block_valu(path))
    st, mk = frame_waves(stride)
    amax = st.max(axis=1).astype(np.float64)
    cross = ((mk == 0) & (st > 0)).any(axis=1)
    epi = (mk == 0).any(axis=1)
    per = {"setup": gr["setup"][1] * np.ones_like(amax), "loop": gr["loop"][1] * amax,
           "newton": gr["newton"][1] * cross, "epilogue": gr["epilogue"][1] * epi,
           "tail": gr["tail"][1] * np.ones_like(amax)}
    tot = sum(v.mean() for v in per.values())
    print(f"waves sampled {amax.size}, black-hole-only waves {1 - epi.mean():.3f}, waves with a crossing "
          f"{cross.mean():.3f}, attempts per wave (slowest lane) mean {amax.mean():.2f}")
    print("static VALU per block group:", {k: v[1] for k, v in gr.items()})
    for k, v in per.items():
        print(f"  {k:9s} {v.mean():7.1f} VALU per wave ({v.mean() / tot:5.1%})")
    print(f"  model total {tot:.1f} VALU per wave (an upper bound: every static VALU of a run block counted)")
    # frac if a block cost nothing: the kernel issues at its ceiling, so time ~ VALU
    for k in ("setup", "newton", "epilogue"):
        print(f"  without {k:9s}: frac x {tot / (tot - per[k].mean()):.3f}")


if __name__ == "__main__":
    main()
