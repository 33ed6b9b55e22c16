"""Re-trace the mismatched rays a TPT_VERIFY_CULL run logged (gpurun_out/verify_*.bin)
through tpt_debug_trace_rays: mode 0 (reference order) and mode 1 (the render's
traversal) -- tells a traversal bug from a render state-machine bug.
Usage: python tools/verify_rays.py C3:ball C5:c5"""
import sys

import numpy as np

sys.path.insert(0, ".")
import tinypathtracer_amd as T  # noqa: E402
from tests.conftest import scene_path  # noqa: E402


def f32(x):
    return np.asarray(x, np.uint64).astype(np.uint32).view(np.float32)


for spec in sys.argv[1:]:
    cfg, name = spec.split(":")
    d = np.fromfile(f"gpurun_out/verify_{cfg}.bin", dtype=np.uint64).reshape(-1, 16)
    if len(d) == 0:
        continue
    o = f32(d[:, 6:9]).copy()
    di = f32(d[:, 9:12]).copy()
    s = T.Scene(scene_path(name))
    ds = s.copySceneToDevice(0).build()
    for mode in (0, 1, 2):
        h, t, uv = ds.trace_rays(o, di, mode=mode)
        print(cfg, "mode", mode, "hit", h.tolist(), "t", [f"{x:.9g}" for x in t])
    print(cfg, "logged render: culled fid", d[:, 2].astype(np.int64).tolist(), "ref fid", d[:, 3].astype(np.int64).tolist(),
          "mode", d[:, 0].tolist(), "phase", d[:, 1].tolist(), "culled path", (d[:, 15] & 1).tolist(),
          "t culled", [f"{x:.9g}" for x in f32(d[:, 4])], "t ref", [f"{x:.9g}" for x in f32(d[:, 5])],
          "lim", [f"{x:.9g}" for x in f32(d[:, 15] >> 32)], "hpos", d[:, 12].astype(np.int64).tolist(),
          "ref hpos", d[:, 13].astype(np.int64).tolist())
    print(cfg, "o", o.tolist(), "d", di.tolist())
    ds.close()
