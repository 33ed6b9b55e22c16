#!/usr/bin/env python3
"""bench.py -- Mrays/s of the path-tracing hot path (BASELINE.json `metric`).

Workload (BASELINE.json configs[1]): input box.gltf (Cornell box), 1920x1080,
1024 spp, 8 bounces, seed 42, one frame per step == PathTracer::doTrace
(path_tracer.cu:491-554): setupRandSeed + all spp of the trace megakernel +
copyToFB, inputs resident in HBM.  A "ray" is one traverseBVH call (primary,
extension, direct probe, shadow), counted by the kernel.

N GPUs: one process per GPU (torch.distributed.run).  Default (--scaling
weak): a step is a batch of N frames of the workload above (seeds 42 .. 42+N-1;
the reference re-seeds every frame, path_tracer.cu:493,513), each frame split
across all N GPUs in interleaved 16-row bands, so every GPU renders the pixel
mix of one whole frame in one launch; one all-to-all (RCCL over xGMI) leaves
frame f on rank f inside the timed region.  --scaling strong: one frame split
across the N GPUs, one gather to rank 0 (bounded by the heaviest pixels'
serial sample chains).  value = rays of all frames /
max-over-ranks step time.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E (MI355X_MICROARCH.md)
# algorithmic bytes: binary internal visit = links 8 + 2 child
# AABBs 48; 4-wide visit = links 16 + 4 child AABBs 96; leaf = fid 4 + 3
# indices 12 + 3 vertices 36; shading hit = 3 normals 36 + 3 indices 12 +
# material 60; pixel write = 12
B_INNER, B_WIDE, B_LEAF, B_HIT, B_PIX = 56, 112, 52, 108, 12


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", choices=sorted(PRESETS), default=None,
                    help="SURVEY 8(d) preset; explicit flags after it still override")
    ap.add_argument("--scene", default="box")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="gloo: rehearse the N-rank path on one GPU (all ranks on device 0, gather via host)")
    ap.add_argument("--verify-gather", action="store_true",
                    help="rank 0 re-renders the whole frame alone and checks the gathered frame bit for bit")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak",
                    help="weak: N frames per step, each banded across the N ranks (all-to-all); "
                         "strong: one frame banded across the N ranks (gather)")
    ap.add_argument("--emulate-ranks", type=int, default=0,
                    help="1-GPU rehearsal of an N-rank run: render only rank 0's bands of an N-way split")
    ap.add_argument("--env", choices=["sky", "none"], default=None, help="procedural equirect env on miss")
    ap.add_argument("--env-is", action="store_true",
                    help="opt-in env next-event estimation with importance sampling (A15; changes the image)")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=1024)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--band-rows", type=int, default=16)
    ap.add_argument("--spp-per-launch", type=int, default=0)
    ap.add_argument("--flags", type=int, default=0, help="TPT_FLAG_* (2 = reference traversal order)")
    ap.add_argument("--refill", type=int, default=0, help="0 = library default")
    ap.add_argument("--extra-streams", type=int, default=0,
                    help="diagnostic: create this many busy-once HIP streams before the scene (as a process "
                         "group's communicator streams would), to check the launch pipeline's queue use")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="1: time the CPU port on rank 0 at N=1")
    ap.add_argument("--cpu-spp", type=int, default=16)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_trace_latest.json"),
                    help="per-launch HBM bytes measured by rocprofv3 --pmc (tools/profile.sh)")
    args = ap.parse_args()
    if args.config:
        # preset values, unless the flag was given explicitly on the command line
        given = {a.split("=")[0].lstrip("-").replace("-", "_") for a in sys.argv[1:] if a.startswith("--")}
        for k, v in PRESETS[args.config].items():
            if k not in given:
                setattr(args, k, v)
    return args


# SURVEY 8(d) configurations (C1 is the CPU-only case reported inside cpu_baseline)
PRESETS = {
    "C2": dict(scene="box", width=1920, height=1080, spp=1024, depth=8, env=None),
    "C3": dict(scene="ball", width=1920, height=1080, spp=4096, depth=8, env="sky"),
    "C4": dict(scene="tir", width=1920, height=1080, spp=8192, depth=32, env=None),
    "C5": dict(scene="c5", width=3840, height=2160, spp=2048, depth=8, env=None),
}
SCENE_DIR = os.path.join(ROOT, "tests", "golden", "scenes")


def scene_file(name):
    if name == "c5":   # synthesized from the shipped scenes (tinypathtracer_amd.synth)
        import tempfile
        from tinypathtracer_amd import synth
        out = os.path.join(tempfile.gettempdir(), "tpt_scenes", "c5.gltf")
        synth.write_c5(out, SCENE_DIR)
        return out
    p = os.path.join(SCENE_DIR, f"{name}.gltf")
    if not os.path.exists(p):
        p = name
    return p


def data_note(args):
    if args.scene == "c5":
        src = "synthesized C5 scene (box+box1+box2+light, 3x midpoint subdivision, 131,712 triangles)"
    else:
        src = f"reference asset input/{args.scene}.gltf (tests/golden/scenes)"
    env = "procedural 2048x1024 sky env (the reference's JPG is missing)" if args.env == "sky" \
        else "no env map (black miss)"
    return f"{src}, seed {args.seed}, {env}"


def cpu_baseline(args):
    """The oracle (CPU port of the reference kernels) on the host cores: the
    bench workload at a bounded spp (Mrays/s does not depend on spp), plus
    SURVEY 8(d) C1 (box 256x256, 16 spp, depth 4).  Trace phase only (RNG init
    reported separately, like the reference's per-frame curand_init); best of
    3 runs each."""
    from oracle import oracle as O
    threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))

    def best_of(ps, w, h, spp, depth, n=3):
        best = None
        for _ in range(n):
            _, _, c = O.render(ps, w, h, spp, depth, args.seed, trig_mode=1, threads=threads)
            if best is None or c["trace_ms"] < best["trace_ms"]:
                best = c
        return best

    ps = O.load_scene(scene_file(args.scene))
    c = best_of(ps, args.width, args.height, args.cpu_spp, args.depth)
    mrays = c["traversals"] / (c["trace_ms"] * 1e3)
    c1 = best_of(O.load_scene(scene_file("box")), 256, 256, 16, 4)
    c1_mrays = c1["traversals"] / (c1["trace_ms"] * 1e3)
    return {"value": round(mrays, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{args.scene}.gltf {args.width}x{args.height} x {args.cpu_spp} spp, depth {args.depth}, "
                      f"seed {args.seed}, best of 3: {c['traversals']} rays in {c['trace_ms'] / 1e3:.2f} s trace "
                      f"(+{c['init_ms'] / 1e3:.2f} s RNG init not counted)",
            "c1": {"value": round(c1_mrays, 3), "unit": "Mrays/s",
                   "sample": f"box.gltf 256x256 x 16 spp, depth 4, seed {args.seed}, best of 3: "
                             f"{c1['traversals']} rays in {c1['trace_ms'] / 1e3:.3f} s trace"},
            "cpu_model": _cpu_model()}


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import tinypathtracer_amd as T
    from tinypathtracer_amd import shard

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; the gloo rehearsal maps every rank onto the visible devices
    dev = local if args.dist_backend == "nccl" else local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group("gloo")

    extra = []
    for _ in range(args.extra_streams):
        q = torch.cuda.Stream(device=dev)
        with torch.cuda.stream(q):
            extra.append(torch.ones(1024, device=f"cuda:{dev}") * 2.0)
    torch.cuda.synchronize()
    scene = T.Scene(scene_file(args.scene))
    d_scene = scene.copySceneToDevice(dev)
    t0 = time.perf_counter()
    d_scene.build()
    build_ms = (time.perf_counter() - t0) * 1e3
    W, H = args.width, args.height
    pt = T.PathTracer("", W, H, dev)
    if args.env == "none":
        args.env = None
    if args.env == "sky":
        pt.envLight = T.EnvLight(T.procedural_sky(2048, 1024), device=dev)
    band = (args.band_rows, world, rank)
    ranks = world
    if args.emulate_ranks > 1 and world == 1:
        ranks = args.emulate_ranks
        band = (args.band_rows, ranks, 0)
    # weak scaling: a batch of `ranks` frames, frame f with seed + f, each banded across all ranks
    n_frames = ranks if args.scaling == "weak" else 1
    seeds = [args.seed + f for f in range(n_frames)]
    radiances = [torch.zeros((H, W, 3), dtype=torch.float32, device=f"cuda:{dev}") for _ in range(n_frames)]
    flags = args.flags | (T._lib.FLAG_ENV_IS if args.env_is else 0)

    def step():
        st = pt.doTraceFrames(d_scene, scene.m_camera, seeds, None, args.spp, max_depth=args.depth,
                              radiances=radiances, band=band, spp_per_launch=args.spp_per_launch, flags=flags,
                              refill=args.refill)
        if world == 1:
            return st, radiances[0]
        src = radiances if args.dist_backend == "nccl" else [r.cpu() for r in radiances]   # gloo: host tensors
        if args.scaling == "weak":
            return st, shard.exchange_frames(src, H, args.band_rows, world, rank)
        return st, shard.gather_frame(src[0], H, args.band_rows, world, rank)

    for _ in range(args.warmup):
        step()

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    stats = []
    for _ in range(args.steps):
        st, frame = step()
        stats.append(st)
    barrier()
    elapsed = time.perf_counter() - t0

    keys = ["traversals", "internal_visits", "wide_visits", "leaf_tests", "shade_hits", "pixels", "samples", "trace_ms",
            "rng_init_ms", "resolve_ms", "trace_launches", "trace_kernel_ms"]
    local_tot = {k: float(sum(s[k] for s in stats)) for k in keys}
    vec = torch.tensor([local_tot[k] for k in keys] + [elapsed], dtype=torch.float64,
                       device=f"cuda:{dev}" if args.dist_backend == "nccl" else "cpu")
    if world > 1:
        mx = vec.clone()
        dist.all_reduce(vec, op=dist.ReduceOp.SUM)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        elapsed = float(mx[-1].item())
        tot = {k: float(vec[i].item()) for i, k in enumerate(keys)}
        tot["trace_ms_max"] = float(mx[keys.index("trace_ms")].item())
        tot["trace_launches_max"] = float(mx[keys.index("trace_launches")].item())
    else:
        tot = dict(local_tot)
        tot["trace_ms_max"] = tot["trace_ms"]
        tot["trace_launches_max"] = tot["trace_launches"]

    def verify(frame):
        """This rank's assembled frame (weak: frame `rank`, seed + rank; strong:
        rank 0's whole frame) against one GPU rendering every row of it."""
        full = torch.zeros((H, W, 3), dtype=torch.float32, device=f"cuda:{dev}")
        sd = args.seed + (rank if args.scaling == "weak" else 0)
        pt.doTrace(d_scene, scene.m_camera, None, args.spp, seed=sd, max_depth=args.depth,
                   radiance=full, band=(args.band_rows, 1, 0), flags=flags, refill=args.refill)
        got = frame.to(full.device).contiguous()
        return bool(torch.equal(got.view(torch.int32), full.view(torch.int32)))

    verified = None
    if world > 1 and args.verify_gather and args.scaling == "weak":
        ok = torch.tensor([1.0 if verify(frame) else 0.0], dtype=torch.float64,
                          device=f"cuda:{dev}" if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        verified = bool(ok.item() == 1.0)

    if rank == 0:
        K = args.steps
        rays = tot["traversals"]
        value = rays / elapsed / 1e6
        # roofline of the dominant kernel (k_trace), per launch, rank 0's device
        l_tot = local_tot
        nl = max(l_tot["trace_launches"], 1.0)
        bytes_total = (B_INNER * l_tot["internal_visits"] + B_WIDE * l_tot["wide_visits"] + B_LEAF * l_tot["leaf_tests"] +
                       B_HIT * l_tot["shade_hits"] + B_PIX * l_tot["pixels"])
        bytes_per_launch = bytes_total / nl
        # avg_launch_s: each launch's own duration (HIP events on its stream;
        # what rocprofv3 reports per kernel dispatch).  The launch pipeline runs
        # launches of different band sets concurrently (concurrency = summed
        # launch time / trace-phase wall time), so the kernel's byte rate is
        # bytes per launch / (launch duration / concurrency) -- the algorithmic
        # bytes of the trace phase over its wall time
        avg_launch_s = (l_tot["trace_kernel_ms"] / nl) / 1e3
        concurrency = l_tot["trace_kernel_ms"] / max(l_tot["trace_ms"], 1e-9)
        achieved = bytes_per_launch * concurrency / avg_launch_s / 1e9
        traffic = None
        batch = (f" x {n_frames} frames (seeds {seeds[0]}..{seeds[-1]}), each banded across {ranks} ranks"
                 if n_frames > 1 else "")
        config = {"workload": f"{args.scene}.gltf {W}x{H} {args.spp}spp depth {args.depth}"
                              + (" env sky" if args.env else "") + (" env-IS" if args.env_is else "") + batch,
                  "scene": f"{args.scene}.gltf", "width": W, "height": H, "spp": args.spp,
                  "max_depth": args.depth, "seed": args.seed,
                  "frames_per_step": n_frames,
                  "parallelism": f"pixel-bands x{world} (rows of {args.band_rows}) + "
                                 + ("RCCL " if args.dist_backend == "nccl" else "gloo (1-GPU rehearsal) ")
                                 + ("all-to-all" if args.scaling == "weak" else "gather")
                  if world > 1 else ("1 GPU" if ranks == 1 else f"1 GPU, rank 0 of {ranks} emulated")}
        if os.path.exists(args.pmc_json):
            try:
                with open(args.pmc_json) as f:
                    pm = json.load(f)
                # PMC bytes are per launch of the profiled workload: use them
                # only when that was this exact single-GPU configuration
                if pm.get("bench_config") == config and pm.get("n_gpus") == world:
                    traffic = pm.get("hbm_bytes_per_launch")
            except (OSError, ValueError):
                traffic = None
        out = {
            "metric": "Mrays/s at 1920x1080x1024spp (box.gltf, 8 bounces); achieved algorithmic GB/s vs HBM peak",
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / K * 1e3, 3),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": data_note(args),
            "config": config,
            "msamples_per_s": round(tot["samples"] / elapsed / 1e6, 2),
            "rays_per_sample": round(rays / max(tot["samples"], 1), 4),
            "visits_per_ray": {k: round(l_tot[k] / max(l_tot["traversals"], 1), 3)
                               for k in ("wide_visits", "internal_visits", "leaf_tests")},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "kernel": "k_trace", "bytes_per_launch": bytes_per_launch,
                         "avg_launch_ms": round(avg_launch_s * 1e3, 3),
                         "concurrency": round(concurrency, 3),
                         "launches_per_step": nl / K},
            "phases_ms_per_step": {"rng_init": round(l_tot["rng_init_ms"] / K, 3),
                                   "trace": round(l_tot["trace_ms"] / K, 3),
                                   "resolve": round(l_tot["resolve_ms"] / K, 3),
                                   "bvh_build_once": round(build_ms, 3)},
        }
        if world > 1 and args.verify_gather:
            # the assembled frame(s) must equal one GPU rendering every row (the
            # RNG subsequence is the global pixel index, path_tracer.cu:39,320)
            out["gather_verified"] = verified if args.scaling == "weak" else verify(frame)
        if world == 1 and args.cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
