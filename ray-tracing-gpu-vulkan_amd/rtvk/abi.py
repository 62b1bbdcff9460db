"""ctypes mirror of include/rt_abi.h, include/rt_mi355x.h (the C-ABI of librt_mi355x.so) and
include/rt_mi355x_debug.h (its diagnostic entry points).

Struct layouts are the reference's byte-exact host<->device ABI:
  Sphere          src/scene.h:16-22            (80 B)
  Scene           src/scene.h:24-29            (41 024 B)
  RenderCallInfo  src/render_call_info.h:5-13  (64 B; std140 twin at shaders/shader.rgen:13-20)

The library is the product; there is no fallback. ``load_library()`` raises if the HIP build is
missing, so nothing above this module can silently run anything else.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parent.parent          # ray-tracing-gpu-vulkan_amd/
LIB_PATH = PKG_ROOT / "lib" / "librt_mi355x.so"

# src/scene.h:5-14
DIFFUSE, METAL, REFRACTIVE = 0, 1, 2
SOLID, CHECKERED = 0, 1
MAX_SPHERE_AMOUNT = 512  # src/scene.h:24

RT_OK = 0
RT_SEED_GLOBAL, RT_SEED_LAUNCH_LOCAL = 0, 1
RT_RNG_PIXEL_STREAM, RT_RNG_SAMPLE_COUNTER, RT_RNG_SAMPLE_HASH = 0, 1, 2
RT_ABI_VERSION = 2
RT_ACCEL_AUTO, RT_ACCEL_BRUTE, RT_ACCEL_LBVH = 0, 1, 2


class Vec4(ctypes.Structure):
    _fields_ = [("x", ctypes.c_float), ("y", ctypes.c_float), ("z", ctypes.c_float), ("w", ctypes.c_float)]


class UVec2(ctypes.Structure):
    _fields_ = [("x", ctypes.c_uint32), ("y", ctypes.c_uint32)]


class Sphere(ctypes.Structure):
    """src/scene.h:16-22 (std140: geometry@0, materialType@16, textureType@20, colors@32, attr@64)."""
    _fields_ = [
        ("geometry", Vec4),
        ("materialType", ctypes.c_uint32),
        ("textureType", ctypes.c_uint32),
        ("_pad0", ctypes.c_uint32 * 2),
        ("colors", Vec4 * 2),
        ("materialSpecificAttribute", ctypes.c_float),
        ("_pad1", ctypes.c_uint32 * 3),
    ]


class Scene(ctypes.Structure):
    """src/scene.h:26-29."""
    _fields_ = [("spheres", Sphere * MAX_SPHERE_AMOUNT), ("sphereAmount", ctypes.c_uint32),
                ("_pad", ctypes.c_uint8 * 60)]


class RenderCallInfo(ctypes.Structure):
    """src/render_call_info.h:5-13."""
    _fields_ = [
        ("number", ctypes.c_uint32),
        ("samplesPerRenderCall", ctypes.c_uint32),
        ("offset", UVec2),
        ("image_size", UVec2),
        ("t", ctypes.c_uint32 * 2),
        ("camera_pos", Vec4),
        ("camera_dir", Vec4),
    ]


class Options(ctypes.Structure):
    """rt_options (include/rt_mi355x.h)."""
    _fields_ = [
        ("max_depth", ctypes.c_uint32),
        ("seed_mode", ctypes.c_uint32),
        ("rng_mode", ctypes.c_uint32),
        ("accel", ctypes.c_uint32),
        ("accumulate", ctypes.c_uint32),
        ("sample_base", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32 * 2),
    ]


class Stats(ctypes.Structure):
    _fields_ = [("segments", ctypes.c_uint64), ("samples", ctypes.c_uint64),
                ("box_tests", ctypes.c_uint64), ("sphere_tests", ctypes.c_uint64)]


assert ctypes.sizeof(Sphere) == 80 and Sphere.materialSpecificAttribute.offset == 64
assert ctypes.sizeof(Scene) == 41024 and Scene.sphereAmount.offset == 40960
assert ctypes.sizeof(RenderCallInfo) == 64 and RenderCallInfo.camera_dir.offset == 48
assert ctypes.sizeof(Options) == 32

# Every symbol include/rt_mi355x.h and include/rt_mi355x_debug.h declare: (name, restype, argtypes).
_P, _U32, _I = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
EXPORTS = {
    "rt_abi_version": (_U32, []),
    "rt_last_error": (ctypes.c_char_p, []),
    "rt_device_count": (_I, [ctypes.POINTER(_I)]),
    "rt_generate_scene": (_I, [ctypes.c_float, _U32, _P, _U32, ctypes.POINTER(_U32)]),
    "rt_canonical_render_call_info": (_I, [_U32, _U32, _U32, ctypes.POINTER(RenderCallInfo)]),
    "rt_context_create": (_I, [_I, ctypes.POINTER(_P)]),
    "rt_context_destroy": (_I, [_P]),
    "rt_set_scene": (_I, [_P, _P, _U32, _P]),
    "rt_set_scene_device": (_I, [_P, _P, _U32, _P]),
    "rt_refit_scene": (_I, [_P, _P, _U32, _P]),
    "rt_refit_scene_device": (_I, [_P, _P, _U32, _P]),
    "rt_render_device": (_I, [_P, ctypes.POINTER(RenderCallInfo), _P, _U32, _U32, _P, _P,
                              ctypes.POINTER(Options), _P]),
    "rt_get_stats": (_I, [_P, ctypes.POINTER(Stats)]),
    "rt_launch_ms": (_I, [_P, _U32, ctypes.POINTER(ctypes.c_float)]),
    "rt_launch_row_weights": (_I, [_P, _U32, _P, _U32]),
    "rt_scatter_rows": (_I, [_P, _P, _P, _P, _U32, _U32, _U32, _P, _P, _P]),
    "rt_resolve_rgba8": (_I, [_P, _P, ctypes.c_uint64, _U32, _P, _P]),
    "rt_gather_rows": (_I, [_P, _P, _P, _U32, _U32, _U32, _P, _P]),
    "rt_multi_create": (_I, [_U32, ctypes.POINTER(_P)]),
    "rt_multi_destroy": (_I, [_P]),
    "rt_multi_device_count": (_I, [_P, ctypes.POINTER(_U32)]),
    "rt_multi_set_scene": (_I, [_P, _P, _U32]),
    "rt_multi_render": (_I, [_P, ctypes.POINTER(RenderCallInfo), ctypes.POINTER(Options), _P, _P, _P]),
    "rt_multi_stats": (_I, [_P, ctypes.POINTER(Stats)]),
    "rt_multi_info": (_I, [_P, _P]),
    "rt_multi_kernel_times": (_I, [_P, _P, _U32, ctypes.POINTER(_U32)]),
    "rt_multi_kernel_times_frames": (_I, [_P, _U32, _P, _U32, ctypes.POINTER(_U32)]),
    "rt_multi_partition": (_I, [_P, _P, _P, _U32]),
    "rt_partition_strips": (_I, [_U32, _U32, _P, _P]),
    "rt_partition_rebalance": (_I, [_U32, _U32, _P, _P, _P, _P, _P, _P, ctypes.c_double, ctypes.POINTER(_U32),
                                    ctypes.POINTER(ctypes.c_double)]),
    "rt_render": (_I, [_P, _U32, _P, _U32, _P, _P, ctypes.POINTER(Options), ctypes.POINTER(Stats)]),
    "rt_store_ppm": (_I, [ctypes.c_char_p, _P, _U32, _U32]),
    "rt_debug_math": (_I, [_I, _I, _P, _P, _U32]),
    "rt_debug_stamps": (_I, [_P, _P]),
    "rt_debug_util": (_I, [_P, _P]),
    "rt_debug_exact_exhaustive": (_I, [ctypes.c_int, _P]),
    "rt_debug_launch_info": (_I, [_P, _P]),
    "rt_debug_kernel_times": (_I, [_P, _P, _U32, ctypes.POINTER(_U32)]),
    "rt_build_info": (ctypes.c_char_p, []),
    "rt_debug_tune": (_I, [_P, ctypes.c_char_p, ctypes.c_double]),
    "rt_debug_walk_hist": (_I, [_P, _P]),
    "rt_debug_walk_split": (_I, [_P, _P]),
    "rt_debug_grid_cells": (_I, [_P, _P]),
    "rt_debug_lane_hist": (_I, [_P, _P]),
    "rt_debug_steals": (_I, [_P, _P]),
    "rt_debug_tile_cost": (_I, [_P, _P, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]),
    "rt_debug_scene": (_I, [_P, _U32, _P, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]),
    "ray_trace": (None, [_U32, ctypes.c_bool, _U32, _U32, _U32]),
    # include/rt_mi355x_debug.h (diagnostics, A/B, the multi-GPU frame plan)
    "rt_debug_multi_plan": (_I, [_U32, _U32, _U32, _P, _U32, _U32, _P, ctypes.c_uint64,
                                 ctypes.POINTER(ctypes.c_uint64)]),
    "rt_debug_multi_plan_rows": (_I, [_U32, _U32, _U32, _P, _P, _U32, _P, ctypes.c_uint64,
                                      ctypes.POINTER(ctypes.c_uint64)]),
    "rt_debug_multi_create_logical": (_I, [_U32, ctypes.POINTER(_P)]),
    "rt_debug_multi_create_logical_rccl": (_I, [_U32, ctypes.POINTER(_P)]),
    "rt_debug_multi_tune": (_I, [_P, ctypes.c_char_p, ctypes.c_double]),
    "rt_debug_multi_feedback": (_I, [_P, _P, _U32]),
    "rt_debug_multi_balance_info": (_I, [_P, _P]),
}

_lib = None


class RtError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"rt error {code}: {msg}")
        self.code = code


def load_library(path: os.PathLike | str | None = None) -> ctypes.CDLL:
    """Load librt_mi355x.so (no fallback: raises FileNotFoundError when it is not built)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    # RT_LIB (diagnostics / A-B profiling only) points at an alternative build of the same ABI.
    p = Path(path) if path else Path(os.environ.get("RT_LIB", LIB_PATH))
    # torch ships its own libamdhip64.so (SONAME libamdhip64.so.7). Importing torch first makes
    # the loader reuse that copy for this library too: one HIP runtime per process, so torch
    # device pointers and streams are valid here. Loading this library first would let torch
    # load a second runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not p.exists():
        raise FileNotFoundError(f"{p} not built: run `make -C {PKG_ROOT}` or __graft_entry__.build()")
    lib = ctypes.CDLL(str(p))
    for name, (res, args) in EXPORTS.items():
        if path is not None and not hasattr(lib, name):
            continue   # an older A/B build may predate a diagnostic entry point
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def source_files() -> list[Path]:
    """The library's sources in the order the Makefile hashes them (SRC_FILES)."""
    csrc, inc = PKG_ROOT / "csrc", PKG_ROOT.parent / "include"
    return (sorted([*csrc.glob("*.hip"), *csrc.glob("*.cpp"), *csrc.glob("*.h")], key=str)
            + sorted(inc.glob("*.h"), key=str))


def sources_sha256() -> str:
    """sha256 (16 hex) of the library sources in this tree: equals the sources_sha256 of
    rt_build_info() when the loaded .so was built from them."""
    import hashlib
    h = hashlib.sha256()
    for p in source_files():
        h.update(p.read_bytes())
    return h.hexdigest()[:16]


def build_info() -> dict:
    """rt_build_info() of the loaded library, parsed, plus whether it matches this tree."""
    raw = load_library().rt_build_info().decode()
    info = dict(kv.split("=", 1) for kv in raw.split(";") if "=" in kv)
    info["tree_sources_sha256"] = sources_sha256()
    info["built_from_tree"] = info.get("sources_sha256") == info["tree_sources_sha256"]
    return info


def check(rc: int) -> None:
    if rc != RT_OK:
        raise RtError(rc, load_library().rt_last_error().decode(errors="replace"))
