import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "ray-tracing-gpu-vulkan_amd"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through librt_mi355x.so)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as orc
    orc.build()
    return orc
