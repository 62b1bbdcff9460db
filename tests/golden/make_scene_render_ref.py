"""Derives a small fixture from the reference's only rendered output, /root/reference/sceneRender.png
(1920x1080 RGBA8, README.md:3; the upstream camera (13, 2, -3) -> origin of shader.rgen:29).

The image is not a pixel oracle (its spp, its scene time t and the renderer version are unknown),
so only coarse statistics travel: a 48x27 thumbnail of 40x40-pixel block means of R, G, B and
32-bin per-channel histograms. tests/test_gpu_parity.py::test_reference_image_qualitative compares
a render of the same view against them under loose, stated bounds.
Run in this container (the reference is not on the GPU box):
  python tests/golden/make_scene_render_ref.py
"""
import struct
import zlib
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
SRC = Path("/root/reference/sceneRender.png")


def decode_png(data: bytes) -> np.ndarray:
    """8-bit RGB / RGBA non-interlaced PNG -> uint8 [H, W, C] (PNG spec filters 0-4)."""
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    i, idat, hdr = 8, b"", None
    while i < len(data):
        n = struct.unpack(">I", data[i:i + 4])[0]
        t = data[i + 4:i + 8]
        if t == b"IHDR":
            hdr = struct.unpack(">IIBBBBB", data[i + 8:i + 21])
        elif t == b"IDAT":
            idat += data[i + 8:i + 8 + n]
        i += 12 + n
    w, h, depth, ctype, _, _, interlace = hdr
    assert depth == 8 and ctype in (2, 6) and interlace == 0
    c = 4 if ctype == 6 else 3
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + w * c)
    out = np.zeros((h, w * c), np.int32)
    prev = np.zeros(w * c, np.int32)
    for y in range(h):
        f, line = raw[y, 0], raw[y, 1:].astype(np.int32)
        cur = np.zeros(w * c, np.int32)
        if f == 0:
            cur = line
        elif f == 2:
            cur = (line + prev) & 255
        else:
            for x in range(w * c):
                a = cur[x - c] if x >= c else 0
                b = prev[x]
                cc = prev[x - c] if x >= c else 0
                if f == 1:
                    p = a
                elif f == 3:
                    p = (a + b) >> 1
                else:   # Paeth
                    pa, pb, pc = abs(b - cc), abs(a - cc), abs(a + b - 2 * cc)
                    p = a if (pa <= pb and pa <= pc) else (b if pb <= pc else cc)
                cur[x] = (line[x] + p) & 255
        out[y] = cur
        prev = cur
    return out.reshape(h, w, c).astype(np.uint8)


def stats(rgb: np.ndarray, block: int = 40) -> dict:
    h, w = rgb.shape[:2]
    thumb = rgb[: h // block * block, : w // block * block, :3].astype(np.float32)
    thumb = thumb.reshape(h // block, block, w // block, block, 3).mean(axis=(1, 3))
    hist = np.stack([np.histogram(rgb[..., k], bins=32, range=(0, 256))[0] for k in range(3)]).astype(np.float32)
    return {"thumb": thumb.astype(np.float32), "hist": hist / hist.sum(axis=1, keepdims=True)}


def main():
    img = decode_png(SRC.read_bytes())
    s = stats(img)
    np.savez_compressed(HERE / "sceneRender_stats.npz", thumb=s["thumb"], hist=s["hist"],
                        size=np.array(img.shape[:2], np.int32))
    print("thumb", s["thumb"].shape, "mean", s["thumb"].mean(axis=(0, 1)))


if __name__ == "__main__":
    main()
