import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# Scenes travel with the repo (tests/golden/scenes, copied data fixtures); the
# reference tree only exists in the build container.
SCENE_DIR = os.path.join(ROOT, "tests", "golden", "scenes")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running")


def scene_path(name):
    return os.path.join(SCENE_DIR, f"{name}.gltf")


@pytest.fixture(scope="session")
def gpu_available():
    import tinypathtracer_amd as T
    if T.device_count() <= 0:
        pytest.fail("no HIP device visible to libtpt.so")
    return True
