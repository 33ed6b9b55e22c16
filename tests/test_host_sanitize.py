"""The host-side parsers under AddressSanitizer + UndefinedBehaviorSanitizer
(SURVEY.md section 5): host/gltf.cpp + json_lite.hpp, host/image.cpp (JPEG
baseline / progressive, PPM) and host/wide_bvh.cpp, built for the CPU by
tests/sanitize/Makefile and fed valid and corrupted inputs -- truncated files,
flipped bytes, bad Huffman tables, absurd dimensions and sampling factors,
malformed JSON, negative / huge / out-of-range accessor fields, broken data
URIs.  Every input must end in "ok" or a parse error; a memory error or
undefined behaviour aborts the harness with the sanitizer's report.

CPU only (the sanitizer build never travels to the GPU box)."""
import base64
import io
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

from tests.conftest import ROOT, SCENE_DIR

SAN = os.path.join(ROOT, "tests", "sanitize")


def _make(target):
    """make under an exclusive lock: pytest-xdist workers each set the module's
    fixtures up, and two concurrent links of one binary fail ("Text file busy")."""
    import fcntl
    with open(os.path.join(SAN, ".build.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        return subprocess.run(["make", "-C", SAN, target], capture_output=True, text=True)


@pytest.fixture(scope="module")
def host_check():
    if not os.path.isdir(SAN) or shutil.which("g++") is None:
        pytest.skip("sanitizer harness not present (GPU box) or no g++")
    r = _make("host_check")
    if r.returncode != 0:
        if "asan" in r.stderr.lower() or "sanitize" in r.stderr.lower():
            pytest.skip("toolchain without ASan/UBSan runtime")
        raise AssertionError(r.stderr)
    return os.path.join(SAN, "host_check")


def run(exe, mode, files):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:allocator_may_return_null=1",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, mode] + [str(f) for f in files], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = r.stdout.strip().split("\n")
    assert len(lines) == len(files), r.stdout
    return lines


def test_valid_scenes(host_check):
    files = sorted(os.path.join(SCENE_DIR, f) for f in os.listdir(SCENE_DIR) if f.endswith(".gltf"))
    out = run(host_check, "gltf", files)
    assert all(x.startswith("ok") for x in out), out


def _mutants(model):
    """Malformed variants of a glTF model (dict) with an embedded buffer."""
    m = json.loads(json.dumps(model))
    out = []

    def mut(fn):
        x = json.loads(json.dumps(m))
        fn(x)
        out.append(json.dumps(x))

    acc = m["accessors"]
    for i in range(min(len(acc), 3)):
        for key, val in (("byteOffset", -4), ("byteOffset", 2 ** 62), ("byteOffset", 1e30), ("count", -1),
                         ("count", 2 ** 40), ("count", 1e300), ("count", 2 ** 61 + 7), ("bufferView", 99),
                         ("bufferView", -3), ("componentType", 5130), ("type", "MAT4"), ("count", 0)):
            mut(lambda x, i=i, key=key, val=val: x["accessors"][i].__setitem__(key, val))
    for key, val in (("byteOffset", -8), ("byteOffset", 10 ** 12), ("buffer", 5), ("byteLength", -1)):
        mut(lambda x, key=key, val=val: x["bufferViews"][0].__setitem__(key, val))
    mut(lambda x: x["buffers"][0].__setitem__("uri", x["buffers"][0]["uri"][:-40]))          # short buffer
    mut(lambda x: x["buffers"][0].__setitem__("uri", x["buffers"][0]["uri"][:60] + "!!@@"))  # bad base64
    mut(lambda x: x["buffers"][0].__setitem__("uri", "data:application/octet-stream;base64,"))
    mut(lambda x: x["buffers"][0].__setitem__("uri", "does_not_exist.bin"))
    mut(lambda x: x["meshes"][0]["primitives"][0].__setitem__("indices", 10 ** 9))
    mut(lambda x: x["meshes"][0]["primitives"][0]["attributes"].__setitem__("POSITION", -1))
    mut(lambda x: x["meshes"][0]["primitives"][0].__setitem__("material", 1e99))
    mut(lambda x: x["meshes"][0].__setitem__("primitives", []))
    mut(lambda x: x["nodes"][0].__setitem__("mesh", 2 ** 31))
    mut(lambda x: x["nodes"][0].__setitem__("mesh", -1e308))
    mut(lambda x: x["nodes"][0].__setitem__("rotation", [1, 2]))
    mut(lambda x: x["nodes"][0].__setitem__("scale", "big"))
    mut(lambda x: x.__setitem__("accessors", {}))
    mut(lambda x: x.__setitem__("nodes", 7))
    return out


def test_corrupted_gltf(host_check, tmp_path):
    files = []
    for name in ("box", "square", "ball"):
        text = open(os.path.join(SCENE_DIR, f"{name}.gltf")).read()
        model = json.loads(text)
        for k, t in enumerate(_mutants(model)):
            p = tmp_path / f"{name}_m{k}.gltf"
            p.write_text(t)
            files.append(p)
        for cut in (0, 1, 10, len(text) // 3, len(text) // 2, len(text) - 2):   # truncated JSON
            p = tmp_path / f"{name}_cut{cut}.gltf"
            p.write_text(text[:cut])
            files.append(p)
    rng = np.random.default_rng(3)
    text = open(os.path.join(SCENE_DIR, "box.gltf")).read()
    for k in range(40):                                  # random byte flips
        b = bytearray(text.encode())
        for _ in range(8):
            b[rng.integers(len(b))] = int(rng.integers(32, 127))
        p = tmp_path / f"flip{k}.gltf"
        p.write_bytes(bytes(b))
        files.append(p)
    for k, t in enumerate(["[" * 200000, "{\"a\":" * 100000, "1e400", "-", "\"\\u12", "{\"a\" 1}", "nan", "\0\0\0",
                           "{\"accessors\": [{\"count\": 1e999}]}", "[1,2,3" + ",4" * 100000]):
        p = tmp_path / f"json{k}.gltf"
        p.write_text(t)
        files.append(p)
    out = run(host_check, "gltf", files)
    assert sum(x.startswith("error") for x in out) > len(files) // 2


def _jpeg(arr, **kw):
    from PIL import Image
    buf = io.BytesIO()
    Image.fromarray(arr).save(buf, "JPEG", **kw)
    return buf.getvalue()


def test_corrupted_images(host_check, tmp_path):
    pytest.importorskip("PIL")
    rng = np.random.default_rng(11)
    sky = (rng.uniform(0, 255, (48, 64, 3))).astype(np.uint8)
    goods = [_jpeg(sky, quality=90), _jpeg(sky, quality=50, progressive=True),
             _jpeg(sky, quality=75, subsampling=0), _jpeg(sky, quality=75, subsampling=2)]
    files = []
    for k, g in enumerate(goods):
        p = tmp_path / f"good{k}.jpg"
        p.write_bytes(g)
        files.append(p)
    out = run(host_check, "image", files)
    assert all(x.startswith("ok") for x in out), out
    files = []
    for k, g in enumerate(goods):
        for cut in sorted(set([2, 4, 20, 100, 200, 400, len(g) // 2, len(g) - 10, len(g) - 2]
                              + list(range(3, len(g), 97)))):
            p = tmp_path / f"cut{k}_{cut}.jpg"
            p.write_bytes(g[:cut])
            files.append(p)
        for j in range(250):                             # flipped bytes, headers included
            b = bytearray(g)
            for _ in range(1 + j % 4):
                pos = int(rng.integers(2, min(len(b), 700))) if j % 2 else int(rng.integers(2, len(b)))
                b[pos] = int(rng.integers(0, 256))
            p = tmp_path / f"flip{k}_{j}.jpg"
            p.write_bytes(bytes(b))
            files.append(p)
    g = bytearray(goods[0])
    i = g.find(b"\xff\xc4")                              # DHT: code counts that overflow 256 symbols
    if i > 0:
        b = bytearray(g)
        for q in range(16):
            b[i + 5 + q] = 255
        (tmp_path / "dht.jpg").write_bytes(bytes(b))
        files.append(tmp_path / "dht.jpg")
    i = g.find(b"\xff\xc0")                              # SOF0: absurd dimensions, components, sampling
    if i > 0:
        for k, (off, val) in enumerate(((5, b"\xff\xff\xff\xff"), (5, b"\x00\x00\x00\x00"), (9, b"\x07"),
                                        (11, b"\x00"), (11, b"\x55"), (11, b"\xff"), (12, b"\x09"))):
            b = bytearray(g)
            b[i + off:i + off + len(val)] = val
            p = tmp_path / f"sof{k}.jpg"
            p.write_bytes(bytes(b))
            files.append(p)
    for k, t in enumerate([b"P6\n64 48\n255\n" + bytes(100), b"P6\n-1 48\n255\n", b"P6\n99999 99999\n255\n",
                           b"P6\n4 4\n0\n" + bytes(48), b"P6\n4 4\n65535\n" + bytes(10), b"P6", b"P3\n1 1\n255\n1 2 3",
                           b"P6\n4 4 255 " + bytes(48), b"P6\n#c\n4 4\n255\n" + bytes(48)]):
        p = tmp_path / f"ppm{k}.ppm"
        p.write_bytes(t)
        files.append(p)
    out = run(host_check, "image", files)
    assert sum(x.startswith("error") for x in out) > len(files) // 3


@pytest.mark.parametrize("n,seed,threads", [(2, 1, -1), (3, 2, -1), (33, 3, -1), (1000, 4, -1), (20000, 5, -1),
                                            (20000, 6, 4)])
def test_wide_tree_builder(host_check, n, seed, threads):
    r = subprocess.run([host_check, "wide", str(n), str(seed), str(threads)], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout + r.stderr[-3000:]


def test_wide_tree_pool_under_tsan():
    """The builder's task pool (chunked binning and scatter, subtree tasks,
    the parallel breadth-first collapse) under ThreadSanitizer, 4 and 8
    threads, each compared byte for byte with the serial build."""
    if not os.path.isdir(SAN) or shutil.which("g++") is None:
        pytest.skip("sanitizer harness not present (GPU box) or no g++")
    r = _make("host_check_tsan")
    if r.returncode != 0:
        if "tsan" in r.stderr.lower() or "sanitize" in r.stderr.lower():
            pytest.skip("toolchain without the TSan runtime")
        raise AssertionError(r.stderr)
    exe = os.path.join(SAN, "host_check_tsan")
    for threads in (4, 8):
        r = subprocess.run([exe, "wide", "40000", "7", str(threads)], capture_output=True, text=True, timeout=600,
                           env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1"))
        assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout + r.stderr[-4000:]
