"""The N-rank bench path through libtpt on one GPU: two ranks share cuda:0 and
talk over gloo (the driver's N-GPU runs use RCCL, one rank per GPU), and every
frame the ranks exchange is checked bit for bit against a single-rank render
of the same frame (bench.py --verify-gather).

* weak scaling: a batch of N frames, each banded across the N ranks
  (tpt_render_frames), one all-to-all leaves frame f on rank f;
* strong scaling: one frame banded across the ranks, one gather to rank 0;
* with a delta light (ball): pair mode on every rank.

This is the HIP path under N ranks; tests/test_shard_gloo.py covers the band
bookkeeping on the CPU against the oracle."""
import json
import os
import subprocess
import sys

import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode,scene,port", [("weak", "box", 29651), ("strong", "box", 29652),
                                              ("weak", "ball", 29653)])
def test_two_ranks_bit_exact(mode, scene, port):
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "1", "--warmup", "0", "--spp", "8", "--width", "256", "--height", "144",
           "--cpu-baseline", "0", "--dist-backend", "gloo", "--verify-gather", "--scaling", mode,
           "--scene", scene] + (["--env", "sky"] if scene == "ball" else [])
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{") and '"metric"' in ln]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == mode
    assert d.get("gather_verified") is True, d


def test_bench_gpus_flag_starts_the_ranks():
    """`python bench.py --gpus 2` with no external launcher starts the two ranks
    itself (torch.distributed.run under a parent that never touches the GPU):
    n_gpus 2, the cost deal from a probe frame, and the gathered frame verified
    bit for bit.  A --gpus that disagrees with an external WORLD_SIZE fails."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
           "--verify-gather", "--spp", "8", "--width", "256", "--height", "144", "--steps", "1", "--warmup", "0",
           "--cpu-baseline", "0", "--weak-extra", "0", "--deal", "cost"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{") and '"metric"' in ln]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d.get("gather_verified") is True, d
    assert d["deal"]["kind"] == "cost" and sum(d["deal"]["bands_per_rank"]) == 9, d["deal"]
    env2 = dict(env, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r2 = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                        cwd=ROOT, env=env2, capture_output=True, text=True, timeout=120)
    assert r2.returncode != 0 and "WORLD_SIZE" in r2.stderr
