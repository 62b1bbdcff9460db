"""C-ABI boundary checks that need no GPU: the library builds, loads, exports every symbol
include/rt_mi355x.h declares, its structs match the reference layout, and its host-side data API
(scene generator, canonical RenderCallInfo) is byte-identical to the oracle's."""
import ctypes
import re
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent


@pytest.fixture(scope="module")
def rtvk():
    import rtvk as m
    m.load_library()
    return m


def declared_functions(header="rt_mi355x.h"):
    text = (ROOT / "include" / header).read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:[A-Za-z_][\w\s\*]*?)\b(rt_\w+|ray_trace)\s*\(", text, flags=re.M)))


@pytest.mark.parametrize("header", ["rt_mi355x.h", "rt_mi355x_debug.h"])
def test_exports_every_declared_symbol(rtvk, header):
    """Both headers' functions are exported by the one library and bound in rtvk.abi; the
    drop-in header (what replaces src/ray_trace.h) declares no diagnostic entry point, the debug
    header declares only those."""
    from rtvk import abi
    lib = ctypes.CDLL(str(abi.LIB_PATH))
    names = declared_functions(header)
    if header == "rt_mi355x.h":
        assert "ray_trace" in names and "rt_render_device" in names and len(names) >= 15
        assert not [n for n in names if n.startswith("rt_debug_")]
    else:
        assert len(names) >= 15 and all(n.startswith("rt_debug_") for n in names)
    for n in names:
        assert hasattr(lib, n), n
        assert n in abi.EXPORTS, f"{n} missing from the Python binding table"


def test_binding_table_has_no_undeclared_symbol():
    from rtvk import abi
    declared = set(declared_functions("rt_mi355x.h")) | set(declared_functions("rt_mi355x_debug.h"))
    assert set(abi.EXPORTS) == declared


def test_ray_trace_signature_matches_reference(rtvk):
    # src/ray_trace.h:9-15: void ray_trace(uint32_t, bool, uint32_t, uint32_t, uint32_t)
    text = (ROOT / "include" / "rt_mi355x.h").read_text()
    m = re.search(r"void ray_trace\(([^)]*)\)", text)
    params = [p.strip().split()[0] for p in m.group(1).replace("\n", " ").split(",")]
    assert params == ["uint32_t", "bool", "uint32_t", "uint32_t", "uint32_t"]


def test_struct_layouts(rtvk):
    from rtvk import abi
    assert ctypes.sizeof(abi.Sphere) == 80
    assert abi.Sphere.materialType.offset == 16 and abi.Sphere.textureType.offset == 20
    assert abi.Sphere.colors.offset == 32 and abi.Sphere.materialSpecificAttribute.offset == 64
    assert ctypes.sizeof(abi.Scene) == 41024 and abi.Scene.sphereAmount.offset == 40960
    assert ctypes.sizeof(abi.RenderCallInfo) == 64
    assert [getattr(abi.RenderCallInfo, f).offset for f in
            ("number", "samplesPerRenderCall", "offset", "image_size", "t", "camera_pos", "camera_dir")] == \
        [0, 4, 8, 16, 24, 32, 48]


def test_abi_version(rtvk):
    assert rtvk.load_library().rt_abi_version() == 2


@pytest.mark.parametrize("t,K", [(0.0, 11), (1.25, 11), (0.0, 3), (0.0, 40)])
def test_scene_generator_matches_oracle(rtvk, oracle, t, K):
    ours = rtvk.spheres_to_numpy(rtvk.generateRandomScene(t, K))
    np.testing.assert_array_equal(ours, oracle.generate_scene(t, K))


def test_canonical_rci_matches_oracle(rtvk, oracle):
    r = rtvk.canonical_render_call_info(100, 1920, 1080)
    assert bytes(r) == oracle.render_call_info(100, 1920, 1080).tobytes()


def test_errors_without_device(rtvk):
    """Without a GPU every device entry point fails loudly (no CPU fallback exists)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    lib = rtvk.load_library()
    n = ctypes.c_int(-1)
    assert lib.rt_device_count(ctypes.byref(n)) == -6 and n.value == 0
    with pytest.raises(rtvk.RtError) as e:
        rtvk.Renderer(0)
    assert e.value.code == -6
    sc = rtvk.generateRandomScene()
    with pytest.raises(rtvk.RtError):
        rtvk.render(sc, rtvk.canonical_render_call_info(1, 8, 8))


def test_invalid_arguments(rtvk):
    lib = rtvk.load_library()
    assert lib.rt_generate_scene(ctypes.c_float(0.0), 11, None, 0, None) == -1
    buf = (rtvk.Sphere * 10)()
    cnt = ctypes.c_uint32()
    assert lib.rt_generate_scene(ctypes.c_float(0.0), 11, ctypes.addressof(buf), 10, ctypes.byref(cnt)) == -1
    assert cnt.value == 488
    assert b"capacity" in lib.rt_last_error()
    assert lib.rt_render(None, 0, None, 0, None, None, None, None) == -1


def test_store_ppm(rtvk, tmp_path):
    img = np.zeros((3, 5, 4), np.uint8)
    img[..., 0] = np.arange(15).reshape(3, 5)
    img[..., 3] = 255
    p = tmp_path / "x.ppm"
    rtvk.store_ppm(str(p), img)
    data = p.read_bytes()
    assert data.startswith(b"P6\n5 3\n255\n")
    px = np.frombuffer(data[len(b"P6\n5 3\n255\n"):], np.uint8).reshape(3, 5, 3)
    np.testing.assert_array_equal(px, img[..., :3])
    with pytest.raises(rtvk.RtError):
        rtvk.store_ppm(str(tmp_path / "no" / "such" / "dir.ppm"), img)


def test_library_reads_only_documented_environment():
    """The shipped library reads exactly the two environment variables INTEGRATION.md §5 lists
    (RT_RNG in ray_trace(), RT_BVH_BUILD in the builder choice); every other launch-plan parameter
    goes through rt_debug_tune."""
    import re
    from pathlib import Path
    csrc = Path(__file__).resolve().parent.parent / "ray-tracing-gpu-vulkan_amd" / "csrc"
    text = "".join(p.read_text() for p in sorted(csrc.iterdir()) if p.suffix in (".cpp", ".hip", ".h"))
    read = set(re.findall(r'getenv\("([A-Z_]+)"\)', text))
    assert read == {"RT_RNG", "RT_BVH_BUILD"}, read
    integ = (Path(__file__).resolve().parent.parent / "INTEGRATION.md").read_text()
    for var in read:
        assert f"`{var}" in integ, var
