"""ctypes wrapper of the CPU oracle (oracle/rt_oracle.cpp). TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker
and as the timed CPU baseline. The product (librt_mi355x.so, rtvk) never touches it.
Buffers are passed as raw bytes / numpy so this module does not depend on the product's Python.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "liboracle_rt.so"
_lib = None
_P, _U, _I = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        l = ctypes.CDLL(str(LIB))
        l.orc_tea.restype = _U
        l.orc_tea.argtypes = [_U, _U]
        l.orc_lcg.restype = _U
        l.orc_lcg.argtypes = [_U]
        l.orc_random_float.restype = ctypes.c_float
        l.orc_random_float.argtypes = [ctypes.POINTER(_U)]
        l.orc_sinf.restype = ctypes.c_float
        l.orc_sinf.argtypes = [ctypes.c_float]
        l.orc_sample_seed_hash.restype = _U
        l.orc_sample_seed_hash.argtypes = [_U, _U]
        l.orc_sample_fixed.restype = ctypes.c_uint64
        l.orc_sample_fixed.argtypes = [ctypes.c_float]
        l.orc_viewport.restype = None
        l.orc_viewport.argtypes = [_P, _P]
        l.orc_generate_scene.restype = _I
        l.orc_generate_scene.argtypes = [ctypes.c_float, _U, _P, _U, ctypes.POINTER(_U)]
        l.orc_render.restype = _I
        l.orc_render.argtypes = [_P, _U, _P, _P, _U, _U, _P, _P, _P, _P, _I]
        l.orc_resolve.restype = _I
        l.orc_resolve.argtypes = [_P, ctypes.c_uint64, _U, _P]
        _lib = l
    return _lib


def tea(v0: int, v1: int) -> int:
    return lib().orc_tea(v0, v1)


def pixel_seed(x: int, y: int, number: int = 0) -> int:
    return tea(tea(x, y), number)


def random_floats(seed: int, n: int) -> list[float]:
    s = _U(seed)
    return [lib().orc_random_float(ctypes.byref(s)) for _ in range(n)]


def sinf(x: float) -> float:
    return lib().orc_sinf(x)


def sample_seed_hash(pixel_seed: int, s: int) -> int:
    """RT_RNG_SAMPLE_HASH: LCG start of sample s of a pixel."""
    return lib().orc_sample_seed_hash(pixel_seed, s)


def sample_fixed(c: float) -> int:
    """RT_RNG_SAMPLE_HASH: 8.24 fixed-point value of a sample colour channel."""
    return lib().orc_sample_fixed(c)


def generate_scene(t: float = 0.0, grid_half_extent: int = 11) -> np.ndarray:
    """(n, 80) uint8 sphere records (src/scene.h layout)."""
    n = _U()
    lib().orc_generate_scene(ctypes.c_float(t), grid_half_extent, None, 0, ctypes.byref(n))
    buf = np.zeros((n.value, 80), np.uint8)
    rc = lib().orc_generate_scene(ctypes.c_float(t), grid_half_extent, buf.ctypes.data, n.value, ctypes.byref(n))
    assert rc == 0
    return buf


def render_call_info(spp: int, width: int, height: int, offset=(0, 0), number: int = 0) -> np.ndarray:
    """64-byte RenderCallInfo (src/render_call_info.h) with the reference's camera."""
    r = np.zeros(16, np.uint32)
    r[0], r[1], r[2], r[3], r[4], r[5] = number, spp, offset[0], offset[1], width, height
    f = r.view(np.float32)
    f[8:12] = [13.0, 11.0, -3.0, 0.0]
    f[12:16] = [-13.0, -11.0, 3.0, 0.0]
    return r


# Arithmetic forms of the oracle (rt_oracle.cpp LIT_*): the shipped contract (what the kernels
# implement), shader.rint read as written, and every dot / normalize read as written too.
LIT_CONTRACT, LIT_RINT, LIT_ALL = 0, 1, 2


def options(max_depth=50, seed_mode=0, rng_mode=0, accel=0, accumulate=0, sample_base=0,
            lit=LIT_CONTRACT) -> np.ndarray:
    o = np.zeros(8, np.uint32)
    o[:6] = [max_depth, seed_mode, rng_mode, accel, accumulate, sample_base]
    o[7] = lit
    return o


def _as_u8(x) -> np.ndarray:
    if isinstance(x, np.ndarray):
        return np.ascontiguousarray(x).view(np.uint8).reshape(-1)
    return np.frombuffer(bytes(x), dtype=np.uint8).copy()


def render(spheres, rci, band_w: int, band_h: int, rows=None, opts=None, accum=None,
           threads: int = 0):
    """One frame of the hot path on the CPU. Returns (accum f32 [bh,bw,4], rgba8 [bh,bw,4],
    (segments, samples, sphere_tests))."""
    sp = _as_u8(spheres)
    n = sp.size // 80
    rc = _as_u8(rci)
    assert rc.size == 64
    rw = None if rows is None else np.ascontiguousarray(rows, np.uint32)
    op = None if opts is None else _as_u8(opts)
    acc = np.zeros((band_h, band_w, 4), np.float32) if accum is None else np.array(accum, np.float32, copy=True)
    out = np.zeros((band_h, band_w, 4), np.uint8)
    st = np.zeros(3, np.uint64)
    r = lib().orc_render(sp.ctypes.data if n else None, n, rc.ctypes.data,
                         rw.ctypes.data if rw is not None else None, band_w, band_h,
                         op.ctypes.data if op is not None else None, acc.ctypes.data, out.ctypes.data,
                         st.ctypes.data, threads if threads else (os.cpu_count() or 1))
    assert r == 0
    return acc, out, tuple(int(v) for v in st)


def resolve(accum: np.ndarray, spp: int) -> np.ndarray:
    """rgba8 tonemap of a summed float accumulator [h, w, 4] (checker of rt_resolve_rgba8)."""
    a = np.ascontiguousarray(accum, np.float32)
    out = np.zeros(a.shape[:-1] + (4,), np.uint8)
    assert lib().orc_resolve(a.ctypes.data, a.size // 4, spp, out.ctypes.data) == 0
    return out
