"""Diagnostic: at which tree depths does the escape-link walk spend its node visits? Builds the
config-5 scene's tree on the device, copies it back, and walks primary + one random-bounce ray per
sampled pixel on the CPU (plain closest-hit culling), histogramming visited-node depths.
Usage: python scripts/visit_depths.py [grid] [n_pixels]"""
import sys

import numpy as np

sys.path.insert(0, "ray-tracing-gpu-vulkan_amd")
import rtvk  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 158
NP = int(sys.argv[2]) if len(sys.argv) > 2 else 400
r = rtvk.Renderer(0)
sc = rtvk.generateRandomScene(0.0, K)
r.set_scene(sc)
nodes = r.scene_array(4).view(np.uint32).reshape(-1, 8)
f = nodes.view(np.float32)
lo, hi = f[:, 0:3], f[:, 4:7]
esc, fc = nodes[:, 3], nodes[:, 7]
geom = r.scene_array(6)   # leaf slots: cx cy cz r
n = len(nodes)
depth = np.zeros(n, np.int32)
stack = [(0, 0)]
while stack:   # left child i+1, right child = escape of the left child
    i, d = stack.pop()
    depth[i] = d
    if fc[i] == 0:
        stack.append((i + 1, d + 1))
        stack.append((int(esc[i + 1]), d + 1))
print(f"{n} nodes, max depth {depth.max()}, nodes per depth: {np.bincount(depth)[:20].tolist()}")
big = r.scene_array(3)
allg = r.scene_array(0)
rng = np.random.default_rng(1)
W, H = 3840, 2160
cam = np.array([13.0, 11.0, -3.0])
fwd = -cam / np.linalg.norm(cam)
right = np.cross(fwd, [0, 1, 0]); right /= np.linalg.norm(right)
up = np.cross(right, fwd)
tanh = np.tan(np.radians(25) / 2)


def walk(o, d, hist):
    inv = 1.0 / np.where(d == 0, 1e-30, d)
    best = 1e4
    for b in big:   # big spheres first, like the kernel
        c = allg[b, :3]; rr = allg[b, 3]
        oc = o - c; bb = oc @ d; cc = oc @ oc - rr; D = bb * bb - cc
        if D >= 0:
            t = -bb - np.sqrt(D)
            if t > 1e-3 and t < best: best = t
    i = 0
    while i != 0xFFFFFFFF:
        hist[depth[i]] += 1
        t0 = (lo[i] - o) * inv; t1 = (hi[i] - o) * inv
        tn = max(np.minimum(t0, t1).max(), 1e-3); tf = min(np.maximum(t0, t1).min(), best)
        if tn <= tf:
            if fc[i]:
                first, cnt = int(fc[i] >> 4), int(fc[i] & 15)
                for s in geom[first:first + cnt]:
                    oc = o - s[:3]; bb = oc @ d; cc = oc @ oc - s[3] * s[3]; D = bb * bb - cc
                    if D >= 0:
                        t = -bb - np.sqrt(D)
                        if t > 1e-3 and t < best: best = t
                i = int(esc[i])
            else:
                i += 1
        else:
            i = int(esc[i])
    return best


hist = np.zeros(64, np.int64)
rays = 0
for _ in range(NP):
    x, y = rng.uniform(0, W), rng.uniform(0, H)
    u = (2 * x / W - 1) * tanh * W / H; v = (1 - 2 * y / H) * tanh
    d = fwd + u * right + v * up; d /= np.linalg.norm(d)
    t = walk(cam, d, hist); rays += 1
    if t < 1e4:
        p = cam + t * d
        d2 = rng.normal(size=3); d2 /= np.linalg.norm(d2)
        if d2[1] < 0: d2[1] = -d2[1]
        walk(p, d2, hist); rays += 1
tot = hist.sum()
cum = np.cumsum(hist) / tot
print(f"{rays} rays, {tot / rays:.1f} visits per ray")
for D in (6, 8, 9, 10, 11, 12, 13, 14):
    print(f"depth <= {D}: {cum[D]:.2%} of visits, {int((depth <= D).sum())} nodes ({int((depth <= D).sum()) * 32 / 1024:.0f} KB)")
