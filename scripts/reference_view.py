"""Renders the reference's upstream view (shader.rgen:29: camera (13, 2, -3) -> origin, the view of
/root/reference/sceneRender.png) at 1920x1080 and compares coarse statistics with the fixture
tests/golden/sceneRender_stats.npz. Writes gpurun_out/reference_view.png for a visual check.
usage: python scripts/reference_view.py [spp] [t]"""
import struct
import sys
import zlib
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "ray-tracing-gpu-vulkan_amd"))
sys.path.insert(0, str(ROOT / "tests" / "golden"))
import torch  # noqa: E402
import rtvk  # noqa: E402
from make_scene_render_ref import stats  # noqa: E402


def png(path, rgb):
    h, w = rgb.shape[:2]
    raw = b"".join(b"\x00" + rgb[y].tobytes() for y in range(h))
    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)
    Path(path).write_bytes(b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0))
                           + chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b""))


def render_view(spp, t=0.0):
    W, H = 1920, 1080
    rci = rtvk.canonical_render_call_info(spp, W, H)
    rci.camera_pos.x, rci.camera_pos.y, rci.camera_pos.z = 13.0, 2.0, -3.0
    rci.camera_dir.x, rci.camera_dir.y, rci.camera_dir.z = -13.0, -2.0, 3.0
    with rtvk.Renderer(0) as r:
        r.set_scene(rtvk.generateRandomScene(t))
        acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
        out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
        r.render_device(rci, acc, out, options=rtvk.make_options(rng_mode=rtvk.HASH))
        torch.cuda.synchronize()
        return out.cpu().numpy()[..., :3]


def compare(img):
    ref = np.load(ROOT / "tests" / "golden" / "sceneRender_stats.npz")
    s = stats(img)
    d = s["thumb"] - ref["thumb"]
    mse = float(np.mean(d ** 2))
    return {"thumb_psnr_db": round(10 * np.log10(255 ** 2 / mse), 2), "thumb_mean_abs": round(float(np.abs(d).mean()), 2),
            "channel_mean_ours": [round(float(v), 2) for v in s["thumb"].mean(axis=(0, 1))],
            "channel_mean_ref": [round(float(v), 2) for v in ref["thumb"].mean(axis=(0, 1))],
            "hist_l1": [round(float(v), 4) for v in np.abs(s["hist"] - ref["hist"]).sum(axis=1)],
            "blocks_within_16": round(float(np.mean(np.abs(d).max(axis=-1) <= 16)), 3)}


if __name__ == "__main__":
    spp = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    t = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
    img = render_view(spp, t)
    (ROOT / "gpurun_out").mkdir(exist_ok=True)
    png(ROOT / "gpurun_out" / "reference_view.png", np.ascontiguousarray(img))
    print({"spp": spp, "t": t, **compare(img)})
