#!/usr/bin/env python3
"""bench.py -- Mrays/s of the path-tracing hot path (BASELINE.json `metric`).

Workload (BASELINE.json configs[1]): input box.gltf (Cornell box), 1920x1080,
1024 spp, 8 bounces, seed 42, one frame per step == PathTracer::doTrace
(path_tracer.cu:491-554): setupRandSeed + all spp of the trace megakernel +
copyToFB, inputs resident in HBM.  A "ray" is one traverseBVH call (primary,
extension, direct probe, shadow), counted by the kernel.

N GPUs: one process per GPU (torch.distributed.run).  `python bench.py --gpus
N` starts the N ranks itself (a launcher parent that never touches the GPU
runs torch.distributed.run and exits with its code); under an external
launcher WORLD_SIZE must equal --gpus.  Default (--scaling strong, the split
north_star names): a step is ONE frame of the workload above, dealt to the N
GPUs in 16-row pixel bands, and one gather of the framebuffer bands to rank 0
(RCCL over xGMI) inside the timed region.  The deal: band b -> rank b % N
(default), or --deal cost: an untimed probe frame dealt in interleaved bands
records each band's trace cost (tpt_params.band_cost), one all-reduce shares
the costs, and every rank computes the same cost-balanced deal
(shard.cost_deal) for the warm-up and timed steps -- as a renderer deals frame
n+1 by frame n's costs (measured no better than the interleave, DESIGN.md
section 6).
value = the frame's rays / max-over-ranks step time.  The same run then also
times weak scaling (key "weak"; --weak-extra 0 skips it): a step is a batch of
N frames (seeds 42 .. 42+N-1; the reference re-seeds every frame,
path_tracer.cu:493,513), each frame banded across all N GPUs, one all-to-all
leaving frame f on rank f.  --scaling weak makes that the headline instead.

--emulate-ranks N (one GPU): renders every rank's share of an N-way split in
turn and reports the slowest rank's step time (the multi-GPU step is the max
over ranks) and the rays of all N shares; --emulate-rank0-only times rank 0's
share alone.

A step is the reference's doTrace (path_tracer.cu:491-554) in full: the
world transform and BVH build (:536-542, transform + LBVH + the 4-wide
traversal tree), setupRandSeed, the trace launches and copyToFB.

Roofline: the trace kernel's working set is L1/L2
resident, so its algorithmic bytes are set against the guide's L2-resident
gather rate, and the binding resource is read from the rocprofv3 PMC summary
of the same workload committed under profiles/ (VALU issue, lane
utilisation, HBM bytes).

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
# MI355X_MICROARCH.md "Indexed rows: gather into LDS": rows shared by every
# workgroup (the XCD's L2) gather at 16.8-18.8 TB/s chip-wide -- the
# cache-level ceiling for bytes the kernel re-reads from L1/L2
L2_GATHER_PEAK_GBS = 18800.0
# VALU issue: a wave64 VALU instruction holds a SIMD-32 for 2 cycles, 4 SIMDs
# per CU (MI355X_MICROARCH.md, "SIMD" and the cycle constants); the CU count comes
# from the device (torch.cuda.get_device_properties: 256 on MI355X)
VALU_INST_PER_CU_CYCLE = 2.0
# algorithmic bytes: binary internal visit = links 8 + 2 child
# AABBs 48; 4-wide visit = links 16 + 4 child AABBs 96; leaf = fid 4 + 3
# indices 12 + 3 vertices 36; shading hit = 3 normals 36 + 3 indices 12 +
# material 60; pixel write = 12
B_INNER, B_WIDE, B_LEAF, B_HIT, B_PIX = 56, 112, 52, 108, 12


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); N > 1 without an external launcher starts them "
                         "(torch.distributed.run); default: WORLD_SIZE, else 1")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", choices=sorted(PRESETS), default=None,
                    help="SURVEY 8(d) preset; explicit flags after it still override")
    ap.add_argument("--scene", default="box")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="gloo: rehearse the N-rank path on one GPU (all ranks on device 0, gather via host)")
    ap.add_argument("--verify-gather", action="store_true",
                    help="rank 0 re-renders the whole frame alone and checks the gathered frame bit for bit")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="strong",
                    help="strong: one frame banded across the N ranks (gather); "
                         "weak: N frames per step, each banded across the N ranks (all-to-all)")
    ap.add_argument("--deal", choices=["interleaved", "cost", "cost-heavy-first", "interleaved-sets", "cost-sets",
                                       "interleaved-heavy-first"],
                    default="interleaved",
                    help="N > 1 (or --emulate-ranks): interleaved = band b -> rank b %% N (default); cost = bands "
                         "dealt by an untimed probe frame's measured band costs (shard.cost_deal; measured no better, "
                         "DESIGN.md section 6 'Band deals'); cost-heavy-first = the same, each rank's costliest "
                         "bands dispatched first (interleaved-heavy-first: the interleave's); *-sets = that deal's bands ordered so the launch pipeline's three "
                         "band sets carry equal probe costs (shard.set_balanced_order)")
    ap.add_argument("--weak-extra", type=int, default=1,
                    help="N>1 with --scaling strong: also time weak scaling (key 'weak')")
    ap.add_argument("--fast-extra", type=int, default=1,
                    help="1 GPU: also time the tolerance mode (TPT_FLAG_FAST: FMA contraction, hardware "
                         "rcp/sqrt/sin/cos, no culling guards; not bit-exact: within SURVEY 8(d)'s tolerance at C2-C4, "
                         "C5's full-spp band meets the mean only) and report it under the key 'tolerance_mode' "
                         "beside the exact headline")
    ap.add_argument("--emulate-ranks", type=int, default=0,
                    help="1-GPU rehearsal of an N-rank run: every rank's bands of an N-way split in turn, "
                         "the step = the slowest rank's")
    ap.add_argument("--emulate-rank0-only", action="store_true", help="with --emulate-ranks: rank 0's share only")
    ap.add_argument("--emulate-order", default="forward",
                    help="with --emulate-ranks: the order the ranks' shares run in: forward, reverse, or a "
                         "comma list of rank ids (a rank may repeat: its last run counts; a subset times only "
                         "those ranks, a diagnostic), to tell a drift with the position in the run from a property "
                         "of the rank's share")
    ap.add_argument("--build-threads", type=int, default=-2,
                    help="host threads of the traversal-tree build (tpt_scene_set_build_threads); "
                         "-2: this process's share of the usable cores (cores / local ranks)")
    ap.add_argument("--async-build", type=int, default=1,
                    help="1: the per-frame scene build's host SAH trees finish on a background thread while the "
                         "render enqueues its RNG initialisation (tpt_scene_build_async); the render's wait for "
                         "them is phase 'tree_wait'. 0: tpt_scene_build (all of it in 'scene_build')")
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
    ap.add_argument("--lanes-per-pixel", type=int, default=0,
                    help="tpt_params.lanes_per_pixel: 0 auto, 1, 2 = pair mode (delta-light scenes), "
                         "4 = four lanes per pixel (split node visits)")
    ap.add_argument("--pipe-sets", type=int, default=0,
                    help="launch pipeline band sets (tpt_params.pipe_sets): 0 auto, 1 one launch per frame")
    ap.add_argument("--pipe-chunks", type=int, default=0,
                    help="spp chunks per band set (tpt_params.pipe_chunks): 0 auto (8)")
    ap.add_argument("--flags", type=int, default=0, help="TPT_FLAG_* (2 = reference traversal order)")
    ap.add_argument("--refill", type=int, default=0, help="0 = library default")
    ap.add_argument("--wavefront", action="store_true",
                    help="the wavefront / ray-queue variant (TPT_FLAG_WAVEFRONT; DESIGN.md section 5 'N1')")
    ap.add_argument("--wf-slots", type=int, default=0, help="wavefront: concurrent paths (0 = every pixel)")
    ap.add_argument("--wf-refill", type=int, default=0, help="wavefront: traversing lanes below which a trace wave runs its pass (0 = 40)")
    ap.add_argument("--leaf-batch", type=int, default=0, help="tpt_params.leaf_batch: 0 = library default")
    ap.add_argument("--extra-streams", type=int, default=0,
                    help="diagnostic: create this many busy-once HIP streams before the scene (as a process "
                         "group's communicator streams would), to check the launch pipeline's queue use")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="1: time the CPU port on rank 0 at N=1")
    ap.add_argument("--cpu-spp", type=int, default=16)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: every usable host core")
    ap.add_argument("--pmc-dir", default=os.path.join(ROOT, "profiles"),
                    help="rocprofv3 PMC summaries (tools/profile.sh); the one whose bench_config matches is used")
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
    if name.startswith("x1s") or name in ("x2", "x3"):   # the exactness scenes (synth.exactness_scene)
        import tempfile
        from tinypathtracer_amd import synth
        out = os.path.join(tempfile.gettempdir(), "tpt_scenes", f"{name}.gltf")
        synth.write_scene(synth.exactness_scene(name, SCENE_DIR), out)
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


def usable_cores():
    """Host cores this process may use: the affinity mask, capped by a cgroup
    CPU quota and by OMP_NUM_THREADS (set to the box's CPU share on the GPU
    pool).  Returns (threads, facts)."""
    aff = len(os.sched_getaffinity(0))
    facts = {"nproc": os.cpu_count(), "affinity": aff}
    n = aff
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            facts["cgroup_cpu_quota"] = round(int(q) / int(per), 2)
            n = min(n, max(1, int(q) // int(per)))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        facts["OMP_NUM_THREADS"] = int(omp)
        n = min(n, int(omp))
    return n, facts


BASELINE_CFLAGS = ["-O3", "-march=native", "-ffp-contract=off", "-fno-fast-math", "-fopenmp", "-fPIC", "-shared",
                   "-std=c11", "-D_GNU_SOURCE"]


def baseline_library():
    """The CPU baseline build of the oracle: the same C
    restatement compiled -O3 -march=native for THIS host (the checker build,
    oracle/liboracle.so, is -O2 and portable).  Compiled into the temp dir on
    first use; falls back to the checker build if no compiler is present."""
    import subprocess
    import tempfile
    src = os.path.join(ROOT, "oracle", "tpt_oracle.c")
    out = os.path.join(tempfile.gettempdir(), f"tpt_oracle_native_{os.getuid()}.so")
    try:
        if not os.path.exists(out) or os.path.getmtime(out) < os.path.getmtime(src):
            subprocess.run(["gcc"] + BASELINE_CFLAGS + ["-o", out + ".tmp", src, "-lm"], check=True,
                           capture_output=True, timeout=120)
            os.replace(out + ".tmp", out)
        return out, "gcc " + " ".join(BASELINE_CFLAGS)
    except (OSError, subprocess.SubprocessError):
        return None, "oracle/liboracle.so (checker build, -O2)"


def cpu_baseline(args):
    """The oracle (CPU port of the reference kernels, identical BVH and
    semantics) on the host cores, BASELINE.md section 3: -O3 -march=native,
    OpenMP dynamic over pixel rows, every usable core, libm trig (trig_mode 0);
    the bench workload at a bounded spp (Mrays/s does not depend on spp), plus
    SURVEY 8(d) C1 (box 256x256, 16 spp, depth 4).  Trace phase only (RNG init
    reported separately, like the reference's per-frame curand_init); best of 3."""
    from oracle import oracle as O
    threads, facts = usable_cores()
    if args.cpu_threads > 0:
        threads = args.cpu_threads
    path, flags = baseline_library()
    O.use_library(path)

    def best_of(ps, w, h, spp, depth, n=3):
        best = None
        for _ in range(n):
            _, _, c = O.render(ps, w, h, spp, depth, args.seed, trig_mode=0, threads=threads)
            if best is None or c["trace_ms"] < best["trace_ms"]:
                best = c
        return best

    try:
        ps = O.load_scene(scene_file(args.scene))
        c = best_of(ps, args.width, args.height, args.cpu_spp, args.depth)
        c1 = best_of(O.load_scene(scene_file("box")), 256, 256, 16, 4)
    finally:
        O.use_library(None)
    mrays = c["traversals"] / (c["trace_ms"] * 1e3)
    c1_mrays = c1["traversals"] / (c1["trace_ms"] * 1e3)
    return {"value": round(mrays, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{args.scene}.gltf {args.width}x{args.height} x {args.cpu_spp} spp, depth {args.depth}, "
                      f"seed {args.seed}, best of 3: {c['traversals']} rays in {c['trace_ms'] / 1e3:.2f} s trace "
                      f"(+{c['init_ms'] / 1e3:.2f} s RNG init not counted)",
            "build": flags, "trig": "libm float (trig_mode 0)", "host": facts,
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


def pmc_summary(args, world, config, build):
    """The committed rocprofv3 PMC summary of this exact workload (tools/profile.sh
    writes bench_config and the profiled library's build identity into it):
    (path, summary, same_build), preferring one profiled with this very library
    (same code-object hash); a summary of the same workload from another build
    is returned flagged (same_build False), or None."""
    import glob
    best, stale = None, None
    for path in sorted(glob.glob(os.path.join(args.pmc_dir, "*pmc_summary*.json"))):
        try:
            with open(path) as f:
                pm = json.load(f)
        except (OSError, ValueError):
            continue
        if pm.get("bench_config") == config and pm.get("n_gpus") == world:
            if (pm.get("build") or {}).get("lib_sha256") == build.get("lib_sha256"):
                best = (path, pm, True)
            else:
                stale = (path, pm, False)
    return best or stale


def roofline(args, world, config, bytes_step, step_s, launches_per_step, avg_launch_ms, build, n_cu):
    """The trace kernel against the MI355X ceilings.
    Live: algorithmic bytes per step / step time, against the L2-resident gather
    rate.  From the PMC summary of the same workload: per-step VALU
    wave-instructions against the VALU issue ceiling at the measured clock, lane
    utilisation, HBM bytes against 8 TB/s.  `bound` names the largest fraction."""
    alg = bytes_step / step_s / 1e9
    limits = {"l2_gather": {"achieved": round(alg, 1), "peak": L2_GATHER_PEAK_GBS, "unit": "GB/s",
                            "frac": round(alg / L2_GATHER_PEAK_GBS, 4), "what": "algorithmic bytes (SURVEY 8(d))"}}
    traffic = None
    found = pmc_summary(args, world, config, build)
    source, same_build, pmc_build = None, None, None
    if found:
        source, pm, same_build = found
        source = os.path.relpath(source, ROOT)
        pmc_build = pm.get("build")
        c = pm.get("counters_per_launch", {})
        lps = pm.get("launches_per_step") or launches_per_step
        if pm.get("hbm_bytes_per_launch") is not None:
            traffic = pm["hbm_bytes_per_launch"]
            hbm = traffic * lps / step_s / 1e9
            limits["hbm"] = {"achieved": round(hbm, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(hbm / HBM_PEAK_GBS, 6), "what": "2*FETCH_SIZE + WRITE_SIZE"}
        clk = pm.get("effective_clock_ghz")
        if c.get("SQ_INSTS_VALU") and clk:
            inst = c["SQ_INSTS_VALU"] * lps / step_s / 1e9
            peak = VALU_INST_PER_CU_CYCLE * n_cu * clk
            lu = pm.get("valu_lane_utilization")
            limits["valu_issue"] = {"achieved": round(inst, 1), "peak": round(peak, 1), "unit": "G wave-inst/s",
                                    "frac": round(inst / peak, 4), "clock_ghz": clk, "n_cu": n_cu,
                                    "lane_utilization": lu,
                                    # active-lane throughput against every lane of every SIMD issuing
                                    "useful_lane_frac": round(inst / peak * lu, 4) if lu is not None else None}
        for k in ("sq_wait_any_frac", "sq_active_inst_any_frac", "l2_hit_rate", "l1_miss_to_l2_frac",
                  "lds_bank_conflict_cycles_per_lds_inst", "ta_accesses_per_cu_cycle"):
            if pm.get(k) is not None:
                limits.setdefault("pmc", {})[k] = pm[k]
    bound = max((v["frac"], k) for k, v in limits.items() if "frac" in v)[1]
    top = limits[bound]
    return {"bound": {"l2_gather": "l2", "hbm": "hbm", "valu_issue": "valu"}[bound],
            "achieved": top["achieved"], "peak": top["peak"], "unit": top["unit"], "frac": top["frac"],
            "traffic": traffic, "kernel": "k_trace",
            "bytes_per_step": bytes_step, "launches_per_step": launches_per_step,
            "avg_launch_ms": round(avg_launch_ms, 3), "limits": limits, "pmc_source": source,
            # the PMC summary's library == the one this bench ran (code-object hash)
            "pmc_same_build": same_build, "pmc_build": pmc_build}


KEYS = ["traversals", "internal_visits", "wide_visits", "leaf_tests", "shade_hits", "pixels", "samples", "trace_ms",
        "rng_init_ms", "resolve_ms", "trace_launches", "trace_kernel_ms", "local_rays", "tree_wait_ms"]


def launch_ranks(n):
    """--gpus N > 1 without an external launcher: run N ranks of this script under
    torch.distributed.run (127.0.0.1, a free port) and return its exit code.  The
    parent never initialises the GPU (it only starts a child process)."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if args.gpus is not None and args.gpus > 1:
            sys.exit(launch_ranks(args.gpus))
    elif args.gpus is not None and args.gpus != int(env_world):
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world} (one rank per GPU)")
    import torch
    import torch.distributed as dist

    import tinypathtracer_amd as T
    from tinypathtracer_amd import shard

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    # one process per GPU; the gloo rehearsal maps every rank onto the visible devices
    dev = local if args.dist_backend == "nccl" else local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group("gloo")
    on_dev = args.dist_backend == "nccl"

    extra = []
    for _ in range(args.extra_streams):
        q = torch.cuda.Stream(device=dev)
        with torch.cuda.stream(q):
            extra.append(torch.ones(1024, device=f"cuda:{dev}") * 2.0)
    torch.cuda.synchronize()
    scene = T.Scene(scene_file(args.scene))
    d_scene = scene.copySceneToDevice(dev)
    # the per-frame traversal-tree build runs on the host: each process (one per
    # GPU) takes its share of the cores this host lets it use
    build_threads = args.build_threads
    if build_threads == -2:
        build_threads = max(1, usable_cores()[0] // max(local_world, 1))
    d_scene.set_build_threads(build_threads)
    W, H = args.width, args.height
    pt = T.PathTracer("", W, H, dev)
    if args.env == "none":
        args.env = None
    if args.env == "sky":
        pt.envLight = T.EnvLight(T.procedural_sky(2048, 1024), device=dev)
    flags = args.flags | (T._lib.FLAG_ENV_IS if args.env_is else 0) | (T._lib.FLAG_WAVEFRONT if args.wavefront else 0)
    emulate = args.emulate_ranks if (args.emulate_ranks > 1 and world == 1) else 0
    ranks = emulate or world
    if world > 1 and args.dist_backend == "nccl" and torch.cuda.device_count() < local_world:
        raise SystemExit(f"bench.py: {local_world} local ranks but {torch.cuda.device_count()} visible GPUs "
                         "(one rank per GPU; --dist-backend gloo rehearses several ranks on one GPU)")

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def probe_costs():
        """The cost deal's input: one untimed frame of the workload dealt in
        interleaved bands, every band's measured trace cost (tpt_params.band_cost;
        this process's bands, or every emulated rank's in turn), summed over the
        ranks by one all-reduce so every rank holds all of them."""
        costs = np.zeros(shard.n_bands(H, args.band_rows), np.float32)
        for r in (range(emulate) if emulate else [rank]):
            d_scene.build(asynchronous=bool(args.async_build))
            pt.doTraceFrames(d_scene, scene.m_camera, [args.seed], None, args.spp, max_depth=args.depth,
                             band=(args.band_rows, ranks, r), flags=flags, refill=args.refill,
                             pipe_sets=args.pipe_sets, pipe_chunks=args.pipe_chunks,
                             lanes_per_pixel=args.lanes_per_pixel, leaf_batch=args.leaf_batch, band_cost=costs)
        if world > 1:
            t = torch.from_numpy(costs.astype(np.float64)).to(f"cuda:{dev}" if on_dev else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            costs = t.cpu().numpy()
        return costs

    deal, deal_info = None, None
    # (at N = 1, --deal cost-heavy-first orders the frame's own bands heaviest first)
    if (((ranks > 1 and args.deal != "interleaved") or args.deal in ("cost-heavy-first", "interleaved-sets",
                                                                     "interleaved-heavy-first"))
            and not args.wavefront):
        tp = time.perf_counter()
        costs = probe_costs()
        nbands = shard.n_bands(H, args.band_rows)
        short = nbands - 1 if H % args.band_rows else None
        nset = args.pipe_sets if args.pipe_sets > 0 else 3   # (tpt_render's default band sets)
        if args.deal == "interleaved-sets":
            deal = [shard.set_balanced_order(b, costs, nset, short)
                    for b in shard.interleaved_deal(H, args.band_rows, ranks)]
        elif args.deal == "interleaved-heavy-first":   # the interleave's bands, each rank's costliest first
            deal = [sorted(b, key=lambda i: (i == short, -float(costs[i]), i))
                    for b in shard.interleaved_deal(H, args.band_rows, ranks)]
        else:
            order = {"cost-heavy-first": "heavy_first", "cost-sets": "sets"}.get(args.deal, "ascending")
            deal = shard.cost_deal(costs, ranks, order=order, short_band=short, nset=nset)
        il = shard.deal_loads(costs, shard.interleaved_deal(H, args.band_rows, ranks))
        cl = shard.deal_loads(costs, deal)
        deal_info = {"kind": args.deal, "probe_s": round(time.perf_counter() - tp, 3),
                     "band_costs_ms": [round(float(v) / 1e3, 2) for v in costs],
                     "predicted_rank_ms": {"interleaved": [round(v / 1e3, 1) for v in il],
                                           "cost": [round(v / 1e3, 1) for v in cl]},
                     "predicted_max_over_mean": {"interleaved": round(max(il) / (sum(il) / ranks), 4),
                                                 "cost": round(max(cl) / (sum(cl) / ranks), 4)},
                     "bands_per_rank": [len(d) for d in deal]}

    def measure(scaling, band_index, extra_flags=0):
        """Warm-up + K timed steps of one scaling mode with this process
        rendering band `band_index` of `ranks` (its share of `deal`, or of the
        interleaved deal); returns (max-over-ranks elapsed, summed stats over
        ranks, this rank's stats, build ms, the last step's frame output)."""
        n_frames = ranks if scaling == "weak" else 1
        seeds = [args.seed + f for f in range(n_frames)]
        radiances = [torch.zeros((H, W, 3), dtype=torch.float32, device=f"cuda:{dev}") for _ in range(n_frames)]
        band = (args.band_rows, ranks, band_index)
        band_list = deal[band_index] if deal is not None else None
        build_ms = []

        def step():
            # doTrace rebuilds the world transform and the BVH every frame (path_tracer.cu:536-542)
            tb = time.perf_counter()
            d_scene.build(asynchronous=bool(args.async_build))
            build_ms.append((time.perf_counter() - tb) * 1e3)
            st = pt.doTraceFrames(d_scene, scene.m_camera, seeds, None, args.spp, max_depth=args.depth,
                                  radiances=radiances, band=band, spp_per_launch=args.spp_per_launch,
                                  flags=flags | extra_flags,
                                  refill=args.refill, pipe_sets=args.pipe_sets, pipe_chunks=args.pipe_chunks,
                                  lanes_per_pixel=args.lanes_per_pixel, leaf_batch=args.leaf_batch,
                                  wf_slots=args.wf_slots, wf_refill=args.wf_refill, band_list=band_list)
            if world == 1:
                return st, radiances[0]
            src = radiances if on_dev else [r.cpu() for r in radiances]   # gloo: host tensors
            if scaling == "weak":
                return st, shard.exchange_frames(src, H, args.band_rows, world, rank, deal=deal)
            return st, shard.gather_frame(src[0], H, args.band_rows, world, rank, deal=deal)

        for _ in range(args.warmup):
            step()
        barrier()
        t0 = time.perf_counter()
        stats, frame = [], None
        for _ in range(args.steps):
            st, frame = step()
            stats.append(st)
        barrier()
        elapsed = time.perf_counter() - t0
        mine = {k: float(sum(x[k] for x in stats)) for k in KEYS}
        vec = torch.tensor([mine[k] for k in KEYS] + [elapsed], dtype=torch.float64,
                           device=f"cuda:{dev}" if on_dev else "cpu")
        if world > 1:
            mx = vec.clone()
            dist.all_reduce(vec, op=dist.ReduceOp.SUM)
            dist.all_reduce(mx, op=dist.ReduceOp.MAX)
            elapsed = float(mx[-1].item())
        tot = {k: float(vec[i].item()) for i, k in enumerate(KEYS)}
        return elapsed, tot, mine, build_ms[-args.steps:], frame, n_frames, seeds

    def measure_all(scaling):
        """measure() on this process's band, or every emulated rank's in turn
        (the step of an N-GPU run is its slowest rank's)."""
        if not emulate:
            return measure(scaling, rank) + ([], [])
        if args.emulate_rank0_only:
            order = [0]
        elif args.emulate_order == "forward":
            order = list(range(emulate))
        elif args.emulate_order == "reverse":
            order = list(range(emulate))[::-1]
        else:
            order = [int(v) for v in args.emulate_order.split(",")]
            if not set(order) <= set(range(emulate)):
                raise SystemExit("--emulate-order names ranks 0..N-1")
        runs = [(r, measure(scaling, r)) for r in order]
        last = {r: m for r, m in runs}   # a repeated rank: its last run
        # (a subset of the ranks: the step and the rays are those ranks' -- a diagnostic)
        per = [last[r] for r in sorted(last)]
        slow = max(range(len(per)), key=lambda i: per[i][0])
        tot = {k: sum(p[1][k] for p in per) for k in KEYS}
        e, _, mine, bms, frame, nfr, seeds = per[slow]
        # per_rank_ms by rank id; run_ms in the order the shares ran
        run_ms = [[r, round(m[0] / args.steps * 1e3, 3)] for r, m in runs]
        return e, tot, mine, bms, frame, nfr, seeds, [round(p[0] / args.steps * 1e3, 3) for p in per], run_ms

    elapsed, tot, local_tot, build_ms, frame, n_frames, seeds, per_rank_ms, run_ms = measure_all(args.scaling)

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
    if world > 1 and args.verify_gather:
        ok = verify(frame) if (args.scaling == "weak" or rank == 0) else True
        okt = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64, device=f"cuda:{dev}" if on_dev else "cpu")
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        verified = bool(okt.item() == 1.0)

    weak = None
    if ranks > 1 and args.scaling == "strong" and args.weak_extra:
        we, wt, _, _, _, wnf, _, wper, _ = measure_all("weak")
        weak = {"value": round(wt["traversals"] / we / 1e6, 2), "unit": "Mrays/s",
                "ms_per_step": round(we / args.steps * 1e3, 3), "frames_per_step": wnf,
                "step": f"{wnf} frames (seeds {args.seed}..{args.seed + wnf - 1}), each banded across {ranks} ranks"
                        + (", RCCL all-to-all" if world > 1 else ""),
                "msamples_per_s": round(wt["samples"] / we / 1e6, 2)}
        if wper:
            weak["per_rank_ms"] = wper

    tolerance = None
    if world == 1 and not emulate and args.fast_extra and not args.wavefront:
        fe, ft, _, _, _, _, _ = measure(args.scaling, 0, T._lib.FLAG_FAST)
        tolerance = {"value": round(ft["traversals"] / fe / 1e6, 2), "unit": "Mrays/s",
                     "ms_per_step": round(fe / args.steps * 1e3, 3), "flags": "TPT_FLAG_FAST",
                     "what": "tolerance mode: FMA contraction and FMA slab tests, hardware rcp/sqrt/sin/cos, no "
                             "culling guards; not bit-exact.  Within SURVEY 8(d)'s per-channel tolerance of the "
                             "reference (mean |d| <= 1e-3, p99 <= 1e-2, >= 99.5 % within one 8-bit step) at every "
                             "BASELINE config at 1-2 spp and on the full-spp bands of C2, C3, C3 + env IS and C4; "
                             "C5's full-spp band (2048 spp) meets the mean only (p99 0.0128, 96.0 % within one "
                             "step) -- tests/test_gpu_tolerance.py, test_gpu_fullsize.py mode fast",
                     "meets_survey_tolerance": args.scene != "c5",
                     "vs_exact": None}

    if rank == 0:
        K = args.steps
        rays = tot["traversals"]
        value = rays / elapsed / 1e6
        step_s = elapsed / K
        # algorithmic bytes of the dominant kernel (k_trace), this device (the slowest
        # emulated rank's), per step
        l_tot = local_tot
        nl = max(l_tot["trace_launches"], 1.0)
        bytes_step = (B_INNER * l_tot["internal_visits"] + B_WIDE * l_tot["wide_visits"] + B_LEAF * l_tot["leaf_tests"]
                      + B_HIT * l_tot["shade_hits"] + B_PIX * l_tot["pixels"]) / K
        avg_launch_ms = l_tot["trace_kernel_ms"] / nl   # each launch's own HIP-event time (= rocprof's per dispatch)
        batch = (f" x {n_frames} frames (seeds {seeds[0]}..{seeds[-1]}), each banded across {ranks} ranks"
                 if n_frames > 1 else "")
        if world > 1:
            par = (f"pixel-bands x{world} (rows of {args.band_rows}) + "
                   + ("RCCL " if on_dev else "gloo (1-GPU rehearsal) ")
                   + ("all-to-all" if args.scaling == "weak" else "gather"))
        elif emulate:
            par = (f"1 GPU, rank 0 of {emulate} emulated" if args.emulate_rank0_only else
                   f"1 GPU, {emulate} ranks emulated in turn (step = slowest rank)")
        else:
            par = "1 GPU"
        config = {"workload": f"{args.scene}.gltf {W}x{H} {args.spp}spp depth {args.depth}"
                              + (" env sky" if args.env else "") + (" env-IS" if args.env_is else "") + batch,
                  "scene": f"{args.scene}.gltf", "width": W, "height": H, "spp": args.spp,
                  "max_depth": args.depth, "seed": args.seed,
                  "frames_per_step": n_frames,
                  "step": "doTrace: transform + BVH build + setupRandSeed + trace + copyToFB (path_tracer.cu:491-554)",
                  "launch_schedule": ("one launch per frame" if args.pipe_sets == 1 else
                                      f"pipe_sets={args.pipe_sets}" if args.pipe_sets > 1 else "auto"),
                  "lanes_per_pixel": args.lanes_per_pixel or "auto",
                  "variant": "wavefront (k_wf_logic + k_wf_trace)" if args.wavefront else "megakernel (k_trace)",
                  "parallelism": par}
        build = T.build_identity()
        n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
        roof = roofline(args, world, config, bytes_step, step_s, nl / K, avg_launch_ms, build, n_cu)
        out = {
            # BASELINE.json's metric, naming the workload actually run (C2 by default)
            "metric": f"Mrays/s at {W}x{H}x{args.spp}spp ({args.scene}.gltf, {args.depth} bounces"
                      + (", env IS" if args.env_is else "") + "); achieved GB/s vs peak",
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(step_s * 1e3, 3),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": data_note(args),
            "config": config,
            "msamples_per_s": round(tot["samples"] / elapsed / 1e6, 2),
            "rays_per_sample": round(rays / max(tot["samples"], 1), 4),
            # rays = reference-equivalent traverseBVH calls; of them, the direct probes
            # resolved exactly in the shading pass without a BVH walk are local_rays
            "gpu_traversals": int(tot["traversals"] - tot["local_rays"]),
            "local_rays": int(tot["local_rays"]),
            "bvh_traversals_per_s_M": round((tot["traversals"] - tot["local_rays"]) / elapsed / 1e6, 2),
            "visits_per_ray": {k: round(l_tot[k] / max(l_tot["traversals"], 1), 3)
                               for k in ("wide_visits", "internal_visits", "leaf_tests")},
            "roofline": roof,
            "phases_ms_per_step": {"scene_build": round(sum(build_ms) / K, 3),
                                   "tree_wait": round(l_tot["tree_wait_ms"] / K, 3),
                                   "rng_init": round(l_tot["rng_init_ms"] / K, 3),
                                   "trace": round(l_tot["trace_ms"] / K, 3),
                                   "resolve": round(l_tot["resolve_ms"] / K, 3)},
            "build": build,
            "build_threads": build_threads,
            "async_build": int(args.async_build),
        }
        if ranks > 1 or deal_info:
            out["deal"] = deal_info or {"kind": "interleaved"}
        if per_rank_ms:
            out["per_rank_ms"] = per_rank_ms
            out["emulate_run_ms"] = run_ms
        if weak is not None:
            out["weak"] = weak
        if tolerance is not None:
            tolerance["vs_exact"] = round(tolerance["value"] / value, 4)
            out["tolerance_mode"] = tolerance
        if verified is not None:
            # the assembled frame(s) must equal one GPU rendering every row (the
            # RNG subsequence is the global pixel index, path_tracer.cu:39,320)
            out["gather_verified"] = verified
        if world == 1 and not emulate and args.cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
