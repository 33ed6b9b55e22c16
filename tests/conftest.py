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
    # TPT_TEST_FORCE_FLAGS=<int>: run the whole suite through a render variant
    # (e.g. 32 = TPT_FLAG_WAVEFRONT, tools/gpu_wfsuite.sh); the library's hook,
    # not an environment read inside the product API
    forced = os.environ.get("TPT_TEST_FORCE_FLAGS")
    if forced:
        import tinypathtracer_amd as T
        T.test_force_flags = int(forced, 0)


def scene_path(name):
    """Shipped scenes from tests/golden/scenes; "c5" is synthesized from them
    (tinypathtracer_amd.synth) into the temp dir once."""
    if name == "c5":
        import tempfile
        from tinypathtracer_amd import synth
        out = os.path.join(tempfile.gettempdir(), "tpt_scenes", "c5.gltf")
        synth.write_c5(out, SCENE_DIR)
        return out
    if name.startswith("x1s") or name in ("x2", "x3"):   # exactness scenes (synth.exactness_scene)
        import tempfile
        from tinypathtracer_amd import synth
        out = os.path.join(tempfile.gettempdir(), "tpt_scenes", f"{name}.gltf")
        synth.write_scene(synth.exactness_scene(name, SCENE_DIR), out)
        return out
    return os.path.join(SCENE_DIR, f"{name}.gltf")


@pytest.fixture(scope="session")
def gpu_available():
    import tinypathtracer_amd as T
    if T.device_count() <= 0:
        pytest.fail("no HIP device visible to libtpt.so")
    return True
