"""Image IO around the render path: textures in, frames out.

  load_texture   image::load_from_memory(..).to_rgba8()  (SR/lib.rs:63-65,
                 basic_sphere_buffer.rs:29): any PIL-readable file (JPEG, PNG,
                 ...) as an (h, w, 4) uint8 RGBA array for Context.set_sky.
  save_png/ppm   the present step of the absent wgpu_renderer loop: a
                 rendered RGBA8 frame (device tensor or host array) to disk.

Host-side plumbing only; nothing here touches the compute path.
"""
from __future__ import annotations

import numpy as np


def load_texture(path: str) -> np.ndarray:
    from PIL import Image

    with Image.open(path) as im:
        return np.ascontiguousarray(np.asarray(im.convert("RGBA"), dtype=np.uint8))


def frame_to_host(rgba, width: int, height: int) -> np.ndarray:
    """(height, width, 4) uint8 host copy of a frame (torch tensor on any device, or array)."""
    if hasattr(rgba, "detach"):
        import torch

        if rgba.is_cuda:
            torch.cuda.synchronize(rgba.device)
        rgba = rgba.detach().cpu().numpy()
    a = np.asarray(rgba, dtype=np.uint8)
    if a.size != width * height * 4:
        raise ValueError(f"frame has {a.size} bytes, expected {width * height * 4}")
    return a.reshape(height, width, 4)


def save_png(path: str, rgba, width: int, height: int) -> None:
    from PIL import Image

    Image.fromarray(frame_to_host(rgba, width, height), "RGBA").save(path, format="PNG")


def save_ppm(path: str, rgba, width: int, height: int) -> None:
    """Binary PPM (P6, RGB; the frames are opaque: alpha 255 after the clear)."""
    a = frame_to_host(rgba, width, height)
    with open(path, "wb") as f:
        f.write(b"P6\n%d %d\n255\n" % (width, height))
        f.write(np.ascontiguousarray(a[..., :3]).tobytes())


def load_ppm(path: str) -> np.ndarray:
    """P6 PPM as (h, w, 4) RGBA (alpha 255)."""
    with open(path, "rb") as f:
        data = f.read()
    fields, pos = [], 0
    while len(fields) < 4:
        while data[pos:pos + 1].isspace():
            pos += 1
        if data[pos:pos + 1] == b"#":
            pos = data.index(b"\n", pos) + 1
            continue
        end = pos
        while not data[end:end + 1].isspace():
            end += 1
        fields.append(data[pos:end])
        pos = end
    if fields[0] != b"P6" or int(fields[3]) != 255:
        raise ValueError("only binary 8-bit PPM (P6) is supported")
    w, h = int(fields[1]), int(fields[2])
    rgb = np.frombuffer(data, dtype=np.uint8, count=w * h * 3, offset=pos + 1).reshape(h, w, 3)
    out = np.empty((h, w, 4), np.uint8)
    out[..., :3] = rgb
    out[..., 3] = 255
    return out
