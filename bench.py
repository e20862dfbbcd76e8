#!/usr/bin/env python3
"""Headline benchmark: Mpixels/s at 1920x1080, 2000 geodesic steps, default
scene (BASELINE.json `metric`, config 3), curved mode, noise mask off.

One step = one full frame: every rank renders its block-cyclic share of the
frame's rows (8-row blocks, block b -> rank b % N) with the gfx950 kernel,
then the tiles are gathered to rank 0 (RCCL over xGMI with the default
"nccl" backend; "gloo" stages the tiles through host memory, which lets N
ranks share one GPU for a functional rehearsal of the distributed path).
`value` = frame pixels x K / (max over ranks of the timed span) - strong
scaling (the frame is fixed, the GPUs share it).

Inputs are resident in HBM before timing: the scene, the step table and the
reference's own textures (assets/textures: 2k skybox, 8k for the 7680x4320
still, uv_checker + cubemap array) unless --textures standin. The camera is
the app's default one, or the app's H-key flyby (--camera flyby: a new
hyperbolicTrajectory camera every frame).

Also reported (rank 0): the integrate kernel's roofline - executed FP32 FLOP
per launch from rocprofv3 counters (profiles/pmc_latest.json, matched to this
kernel source and config) over the same timed run's frame time - and the
reference's CPU press-R geodesic loop swept over a sample of the frame's
pixels on this host (cpu_baseline; oracle restatement, "port").

  python bench.py [--gpus N --steps K --warmup W]   (N > 1: spawns N ranks, launch_contract)
  torchrun --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

KERNEL_SRC = ROOT / "schwarzschild-raytracer_amd" / "csrc" / "kernels" / "geodesic.hip"
# the reference loop's cost per executed chord step in the
# default scene (integrator 71 + black hole 17 + six objects, all-miss) and
# per pixel - what the un-culled shader would execute, kept for reference.
FLOP_PER_STEP = 360.0
FLOP_PER_PIXEL = 150.0
# MI355X_MICROARCH.md: FP32 vector peak (1024 SIMDs x 2.4 GHz x 64 FLOP/cycle:
# one wave64 v_fma_f32 per 2 cycles) and HBM3E peak.
PEAK_FP32_TFLOPS = 157.3
PEAK_HBM_GBS = 8000.0
CLOCK_GHZ = 2.4
SIMDS = 1024
BLOCK_ROWS = 8
CRITICAL_CANDIDATES = 8  # 16-row bands timed alone for roofline.critical_path
MAX_HW_QUEUES = 32  # gpurun's cap on GPU_MAX_HW_QUEUES
# BASELINE.json configs: name -> (width, height, max_steps)
WORKLOADS = {
    "small": (640, 360, 1000),       # config 2
    "headline": (1920, 1080, 2000),  # config 3 (the metric)
    "4k": (3840, 2160, 4000),        # config 4
    "8k": (7680, 4320, 8000),        # config 5 (offline still)
}
MODES = {"curved": 0, "flat": 1, "half_width": 2, "half_height": 3}
FLYBY = (30.0, 10.0)  # src/main.cpp:409: hyperbolicTrajectory(30, 10, t)


HEADLINE_PX = 1920 * 1080
MAX_BATCH = 16  # the bench's cap (the library takes SR_MAX_BATCH = 32)


def headline_scale_1gpu(width, height, world):
    """One GPU and frames of the headline's scale (half to one headline frame
    of pixels): the shape measured at round 4's kernel (below)."""
    return world == 1 and HEADLINE_PX // 2 <= width * height <= HEADLINE_PX


def frames_per_launch(width, height, world, steps=None):
    """Default frames per launch (sr_render_blocks_batch): a rank's share of B
    frames, B chosen so that one launch carries about eight headline frames'
    worth of pixels, 1..16. A rank holding 1/N of a frame then runs launches
    as large as a whole frame's: its share alone is latency-bound (the photon
    ring's waves) and small concurrent launches fill the GPU badly. With a
    timed window of `steps` frames, at most half of it per launch: two
    launches in flight overlap each other's ring-wave tails, one cannot
    (profiles/r02/s3_batch_*.jsonl, s12_batch_k20.jsonl: over
    20 frames, 8 / 10 / 10 / 10 frames per launch at N = 1 / 2 / 4 / 8 are
    within 0.5 % of the best measured). One GPU at the headline's scale: 16
    frames per launch (two launches in flight, launches_in_flight), and over
    a short window up to all but four of its frames in the first launch (the
    second overlaps its tail): at round 4's kernel 16 x 2 renders 1.2 % more
    frames per second than 8 x 3 over 96 frames and 1.0 % more over the
    driver's 20 (profiles/r04/s31_shape_96.jsonl, s32_shape_20.jsonl)."""
    if headline_scale_1gpu(width, height, world):
        b = MAX_BATCH
        if steps:
            b = max(1, min(b, max(-(-steps // 2), steps - 4)))
        return b
    b = max(1, min(MAX_BATCH, round(8 * HEADLINE_PX * world / (width * height))))
    if steps:
        b = max(1, min(b, -(-steps // 2)))
    return b


def launches_in_flight(batch, width=0, height=0, world=0):
    """Default launches in flight per GPU (each on its own context and stream):
    3 for batched launches, 4 for single frames; 2 for one
    GPU's 12 or more headline-scale frames per launch (frames_per_launch)."""
    if batch >= 12 and headline_scale_1gpu(width, height, world):
        return 2
    return 3 if batch > 1 else 4


def hw_queues_needed(launches, world, backend):
    """Hardware queues a rank wants: one per in-flight launch's stream, plus
    the collective's internal streams (RCCL) and the default stream; at
    least 8 (the setting every round-1 measurement ran with)."""
    return max(8, launches + (2 if world > 1 and backend == "nccl" else 0) + 1)


def kernel_sha() -> str:
    return hashlib.sha256(KERNEL_SRC.read_bytes()).hexdigest()[:16]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=96,
                    help="timed frames (96: twelve 8-frame launches, the pipeline in steady state rather than one fill)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="headline",
                    help="BASELINE.json config (width x height / steps); --width/--height/--max-steps override")
    ap.add_argument("--width", type=int, default=0)
    ap.add_argument("--height", type=int, default=0)
    ap.add_argument("--max-steps", type=int, default=0)
    ap.add_argument("--mode", choices=["curved", "flat", "half_width", "half_height"], default="curved",
                    help="raytrace_type (frag:865-878); the split modes use --curved-percentage")
    ap.add_argument("--curved-percentage", type=float, default=0.5)
    ap.add_argument("--percent-black", type=float, default=-1.0,
                    help="noise mask (frag:839-841, 879); the app runs 0.75, the headline -1 (off)")
    ap.add_argument("--camera", choices=["static", "flyby"], default="static",
                    help="static: the app's default camera; flyby: the H-key hyperbolic trajectory, a new camera "
                         "every frame (src/main.cpp:404-410)")
    ap.add_argument("--textures", choices=["auto", "assets", "standin"], default="auto",
                    help="assets: the reference's own textures (assets/textures); standin: procedural ones of the "
                         "same shapes; auto: assets when present")
    ap.add_argument("--skybox", choices=["auto", "2k", "8k"], default="auto",
                    help="BACKGROUND_TEXTURE_QUALITY (src/main.cpp:57-63); auto: 8k for the 8k still, else 2k")
    ap.add_argument("--no-cull", action="store_true", help="exhaustive per-object tests (reference loop)")
    ap.add_argument("--scene", choices=["default", "stress"], default="default",
                    help="default: the app's scene (src/main.cpp:222-268); stress: every capacity of the uniform "
                         "block filled (scenes.scene_stress: 3 of each primitive, 10 materials, 4 lights)")
    ap.add_argument("--test-ray", choices=["off", "on"], default="off",
                    help="the press-R overlay (frag:760-803, src/main.cpp:375-391): a 1000-point test-ray polyline "
                         "drawn into every frame (scenes.test_ray_overlay)")
    ap.add_argument("--inflight", type=int, default=0,
                    help="launches in flight per GPU, each on its own context and stream (0: 3 for batched "
                         "launches, 4 for single frames)")
    ap.add_argument("--batch", type=int, default=0,
                    help="frames per launch, 1..16 (sr_render_blocks_batch; 0: about eight headline frames' worth "
                         "of pixels of this rank's share per launch, at most half of --steps)")
    ap.add_argument("--split", default="0",
                    help="split tiles MAX_TILES[:LANES[:MIN_STEPS]] (sr_set_split; 0: off)")
    ap.add_argument("--stream-priority", choices=["off", "lead"], default="off",
                    help="lead: the first context's stream at high priority, the others at normal priority "
                         "(the hardware dispatches the leading launch's workgroups first; the others fill in)")
    ap.add_argument("--balance", choices=["auto", "cost", "cyclic"], default="auto",
                    help="N > 1: cost: each rank renders an equal number of 8-row blocks of about equal cost "
                         "(dist.balanced_blocks over the frame's step map, sr_render_block_list); cyclic: block b "
                         "on rank b %% N; auto: cost for the static camera (every frame is the priced one), cyclic "
                         "for the flyby (block costs drift between frames by more than priced lists gain, "
                         "dist.REPRICE_MARGIN)")
    ap.add_argument("--reprice", type=int, default=-1,
                    help="N > 1, --balance cost: re-price the block lists every this many launches from a "
                         "quarter-resolution cost map of the launch's camera (rank 0, broadcast; the priced "
                         "lists only when they beat cyclic rows by dist.REPRICE_MARGIN, else cyclic rows); -1: "
                         "every launches-in-flight launches with --camera flyby, else never; 0: never")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="nccl: RCCL gather of device tiles over xGMI (one GPU per rank); gloo: tiles staged "
                         "through host memory (ranks may share a GPU)")
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--critical-path", choices=["on", "off"], default="on",
                    help="time the slowest row bands alone (extra launches of the same kernel; off for rocprof)")
    ap.add_argument("--reference-loop", choices=["on", "off"], default="on",
                    help="time one un-culled frame (the reference's per-step all-object loop) for "
                         "roofline.speedup_vs_reference_loop")
    ap.add_argument("--cpu-sample-rows", type=int, default=0,
                    help="rows of the frame swept on the CPU for `value` (0 = every row: the full frame)")
    ap.add_argument("--single-frame", choices=["on", "off"], default="on",
                    help="also time single-frame launches (N = 1): one frame alone, and 4 in flight")
    ap.add_argument("--single-split", default="0",
                    help="split tiles for the latency figure of one frame alone: max_tiles[:lanes[:min_steps]] "
                         "(0 = off, the default since the black hole's crossing change: every split setting "
                         "measured 2-8 %% slower alone, profiles/r05/s32; the costliest tiles' rays in sparse "
                         "waves, DESIGN.md §6)")
    ap.add_argument("--dump-frames", default="",
                    help="directory: rank 0 saves every timed frame as assembled (frame_<f>.npy), for the "
                         "multi-rank parity test; copies are taken after the timed region")
    ap.add_argument("--traffic-json", default="",
                    help="HBM traffic record (default profiles/traffic_latest[_<variant>].json)")
    ap.add_argument("--pmc-json", default="",
                    help="PMC FLOP record (default profiles/pmc_latest[_<variant>].json)")
    return ap.parse_args()


def free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv: list[str], grace_s: float = 30.0) -> int:
    """`bench.py --gpus N` (N > 1) started without a launcher: run N rank
    processes of this script, one per GPU, with the env:// rendezvous
    torch.distributed.run would give them (RANK, LOCAL_RANK, WORLD_SIZE,
    LOCAL_WORLD_SIZE, MASTER_ADDR 127.0.0.1, a free MASTER_PORT). This parent
    imports neither torch nor HIP. The ranks share its stdout, so rank 0's JSON
    line is the run's line. Returns the first non-zero exit status (in the
    order the ranks failed), else 0; once a rank has failed the others get
    `grace_s` to finish before they are terminated (they would otherwise wait
    in a collective for the dead rank)."""
    # free_port() closes its socket before rank 0's store binds the port, so
    # another process can take it in between: rank 0 then exits with
    # EXIT_PORT_TAKEN (main) and the ranks are started again on a new port
    for attempt in range(PORT_ATTEMPTS):
        rc = _run_ranks(n, argv, free_port(), grace_s)
        if rc != EXIT_PORT_TAKEN:
            return rc
        print(f"bench: rendezvous port taken (attempt {attempt + 1}), new port", file=sys.stderr)
    return rc


EXIT_PORT_TAKEN = 98  # errno EADDRINUSE: rank 0's rendezvous store could not bind MASTER_PORT
PORT_ATTEMPTS = 3


def _run_ranks(n: int, argv: list[str], port: int, grace_s: float) -> int:
    import signal

    script = str(Path(__file__).resolve())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SR_BENCH_SPAWNED="1")
        procs.append(subprocess.Popen([sys.executable, script] + argv, env=env))

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                p.kill()

    old = signal.signal(signal.SIGTERM, lambda *a: (stop(), sys.exit(143)))
    first_bad, failed_at = 0, None
    try:
        while any(p.poll() is None for p in procs):
            for p in procs:
                rc = p.poll()
                if rc not in (None, 0) and first_bad == 0:
                    first_bad, failed_at = rc, time.monotonic()
                    print(f"bench: rank {procs.index(p)} exited with status {rc}", file=sys.stderr)
                    if rc == EXIT_PORT_TAKEN:  # the others wait on a store that never came up
                        failed_at -= grace_s
            if failed_at is not None and time.monotonic() - failed_at > grace_s:
                stop()
                break
            time.sleep(0.05)
        for p in procs:
            rc = p.wait()
            if rc != 0 and first_bad == 0:
                first_bad = rc
    finally:
        stop()
        signal.signal(signal.SIGTERM, old)
    return 1 if first_bad < 0 else first_bad  # a signal-killed rank (negative rc) is a failure too


def port_taken(e: BaseException) -> bool:
    """Whether an init_process_group failure is the store's bind of a port
    another process holds (EADDRINUSE)."""
    msg = str(e).lower()
    return "address already in use" in msg or "eaddrinuse" in msg or "errno: 98" in msg


def launch_contract(args) -> None:
    """The driver's launch shapes: `bench.py --gpus N` under
    torch.distributed.run (WORLD_SIZE set by the launcher: it must equal N),
    or alone (N > 1: spawn_ranks; N = 1: this process renders)."""
    if args.gpus < 1:
        raise SystemExit("bench: --gpus must be >= 1")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if int(env_world) != args.gpus:
            raise SystemExit(f"bench: WORLD_SIZE={env_world} from the launcher but --gpus {args.gpus}: "
                             "run one rank per GPU (--nproc-per-node equal to --gpus)")
        return
    if args.gpus > 1:
        sys.stdout.flush()
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))


def main():
    args = parse()
    launch_contract(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    W0, H0, N0 = WORKLOADS[args.workload]
    W, H, N = args.width or W0, args.height or H0, args.max_steps or N0
    B = args.batch if args.batch > 0 else frames_per_launch(W, H, world, args.steps)
    if not 1 <= B <= MAX_BATCH:
        raise SystemExit(f"bench: --batch must be 1..{MAX_BATCH}")
    F = args.inflight if args.inflight > 0 else launches_in_flight(B, W, H, world)
    split = [int(x) for x in args.split.split(":")] + [16, 1][len(args.split.split(":")) - 1:]
    # every in-flight frame's stream needs a hardware queue of its own (HIP's
    # default is 4 per process); must be set before the HIP runtime starts.
    # Under a profiler whose preloaded library has already started HIP the
    # in-process value is ignored: set it on the command line there.
    need = hw_queues_needed(F, world, args.dist_backend)
    if need > MAX_HW_QUEUES:
        F = MAX_HW_QUEUES - (need - F)
        print(f"bench: clamping frames in flight to {F} ({MAX_HW_QUEUES} hardware queues)", file=sys.stderr)
        need = MAX_HW_QUEUES
    have = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
    if have < need:
        os.environ["GPU_MAX_HW_QUEUES"] = str(need)
    import numpy as np
    import torch
    import torch.distributed as dist

    import srpkg

    pkg = srpkg.load_package()
    abi, sc = pkg.abi, pkg.scenes
    ndev_seen = torch.cuda.device_count()  # counts devices without initialising HIP
    if distributed and args.dist_backend == "nccl":
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
        if ndev_seen < local_world:
            # RCCL needs a GPU per rank: two ranks on one device hang or fail in init
            raise SystemExit(f"bench: --dist-backend nccl needs one GPU per rank: {local_world} local ranks but "
                             f"{ndev_seen} visible device(s) (use --dist-backend gloo to rehearse on fewer GPUs)")
    ndev = max(1, ndev_seen)
    dev = torch.device("cuda", local % ndev)
    if distributed:
        try:
            if args.dist_backend == "nccl":
                torch.cuda.set_device(dev)
                dist.init_process_group("nccl", device_id=dev)
            else:
                dist.init_process_group("gloo")
        except Exception as e:
            if port_taken(e) and os.environ.get("SR_BENCH_SPAWNED") == "1" and rank == 0:
                print(f"bench: rank 0 could not bind MASTER_PORT: {e}", file=sys.stderr)
                sys.exit(EXIT_PORT_TAKEN)  # spawn_ranks retries on a new port
            raise

    # ---- inputs resident in HBM ---------------------------------------------------
    scene = sc.scene_stress() if args.scene == "stress" else sc.scene_default(textured=True)
    test_ray = sc.test_ray_overlay() if args.test_ray == "on" else None
    params = abi.default_params(max_steps=N, percent_black=args.percent_black, raytrace_type=MODES[args.mode],
                                curved_percentage=args.curved_percentage)
    quality = args.skybox if args.skybox != "auto" else ("8k" if (W, H) == WORKLOADS["8k"][:2] else "2k")
    use_assets = args.textures == "assets" or (args.textures == "auto" and pkg.assets.available())
    if use_assets:
        skybox = pkg.assets.skybox(quality)
        arr, _, _ = pkg.assets.texture_array()
    else:
        skybox = sc.skybox(*((8192, 4096) if quality == "8k" else (2048, 1024)))
        arr, _, _ = sc.default_texture_array()
    # Cameras: frame f of the run (warmup + timed) uses cams[f].
    warm = max(args.warmup, F * B)  # every context learns its launch order
    n_frames = warm + args.steps
    if args.camera == "flyby":
        cams = [abi.camera_flyby((f + 0.5) / n_frames, *FLYBY) for f in range(n_frames)]
    else:
        cams = [abi.default_camera()] * n_frames
    # Launches in flight, B frames per launch: a frame's time is bounded by
    # the latency of its longest rays' waves, which a share of
    # 1/N of the rows does not shorten. One launch renders this rank's rows
    # of B consecutive frames (sr_render_blocks_batch, a camera per frame),
    # and F launches on their own contexts and streams fill the SIMDs those
    # waves leave idle. Launch j renders on context j % F; its tiles are
    # gathered to rank 0 on that context's stream (nccl, one collective per
    # launch), or through host memory once it is done (gloo).
    D = pkg.dist
    gloo = distributed and args.dist_backend == "gloo"
    ctxs = []
    def new_renderer():
        """a context with the run's inputs resident (scene, textures, test ray)"""
        rk = pkg.Renderer(dev.index)
        rk.set_scene(scene)
        rk.set_background(skybox)
        rk.set_texture_array(arr)
        rk.set_culling(not args.no_cull)
        if test_ray is not None:
            rk.set_test_ray(test_ray)
        return rk

    for k in range(F):
        rk = new_renderer()
        rk.set_split(split[0], split[1], split[2])
        tile_k = torch.zeros((B, D.tile_rows(world, H, BLOCK_ROWS), W, 4), dtype=torch.uint8, device=dev)
        host_k = torch.zeros(tuple(tile_k.shape), dtype=torch.uint8).pin_memory() if gloo else None
        gather_k = D.FrameGather(host_k if gloo else tile_k, world, rank, H, BLOCK_ROWS)
        if args.stream_priority == "lead":
            lo, hi = torch.cuda.Stream.priority_range()  # (lowest, highest): lower numbers run first
            s_k = torch.cuda.Stream(dev, priority=hi if k == 0 else lo)
        else:
            s_k = torch.cuda.current_stream(dev) if k == 0 else torch.cuda.Stream(dev)
        ctxs.append((rk, tile_k, gather_k, s_k, host_k))
    r, tile, _, stream, _ = ctxs[0]

    frames = {}  # --dump-frames: frame index -> assembled frame (rank 0), timed frames only
    dump_from = [1 << 30]
    last = [None]  # (first frame, assembled frames) of the last gathered launch, rank 0 (parity check)

    def keep(first, batch):
        if batch is None:
            return
        # no copy: FrameGather reuses its frame buffer at its NEXT call, and the
        # parity check reads this (the last launch's) before any further launch
        # (a copy here, in the timed region, cost ~7 % of the headline: s2)
        last[0] = (first, batch)
        if args.dump_frames:
            for i in range(batch.shape[0]):
                if first + i >= dump_from[0]:
                    frames[first + i] = batch[i].clone()  # on the launch's stream (nccl) or host (gloo)

    lists = [None]  # balanced_blocks lists (N > 1, --balance cost), set below from the step map
    sched = [None]  # dist.ListSchedule: the lists each context's launches render (re-pricing changes them)
    rp = {"every": 0, "pricer": None, "stream": None, "choices": []}  # flyby re-pricing (set below)

    def render(rk, first, n, out, s_k, lst=None):
        """frames first .. first + n - 1 of this rank's share into out[:n]"""
        lst = lst if lst is not None else lists[0]
        if lst is not None:
            rk.render_block_list(cams[first:first + n], params, W, H, BLOCK_ROWS, lst[rank], out=out[:n],
                                 stream=s_k)
        elif n == 1:
            rk.render_blocks(cams[first], params, W, H, BLOCK_ROWS, rank, world, out=out[0], stream=s_k)
        else:
            rk.render_blocks_batch(cams[first:first + n], params, W, H, BLOCK_ROWS, rank, world, out=out[:n],
                                   stream=s_k)

    gtime = {"on": False, "events": [], "host_s": 0.0}  # the timed launches' gathers (N > 1)

    def reprice(cam):
        """Lists for a moved camera (collective): rank 0 prices the blocks
        from a quarter-resolution cost map of `cam` on its own context and
        stream (the launches in flight run on), every rank gets its lists."""
        obj = [None]
        if rank == 0:
            wl, hl = max(8, W // 4), max(8, H // 4)
            wc = rp["pricer"].wave_costs(cam, params, wl, hl, stream=rp["stream"])
            rp["stream"].synchronize()
            # a quarter-resolution 8-row block spans four full-resolution ones
            cl = np.repeat(D.block_costs(wc.cpu()), 4)[:D.nblocks(H, BLOCK_ROWS)]
            lst, rp["last_choice"] = D.choose_lists(D.balanced_blocks(cl, world), cl, world, H, BLOCK_ROWS)
            rp["choices"].append(rp["last_choice"])
            obj = [lst]
        dist.broadcast_object_list(obj, src=0, device=None if gloo else dev)
        return obj[0]

    def launch(j, first, n):
        rk, tile_k, gather_k, s_k, host_k = ctxs[j % F]
        with torch.cuda.stream(s_k):
            lst = None
            if sched[0] is not None:
                lst, changed = sched[0].adopt(j, reprice(cams[first]) if sched[0].due(first) else None)
                if changed:
                    gather_k.set_lists(lst)
            render(rk, first, n, tile_k, s_k, lst)
            if gloo:
                host_k[:n].copy_(tile_k[:n], non_blocking=True)
                return
            if gtime["on"] and distributed:  # HIP events around the RCCL gather on the launch's stream
                e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                e[0].record(s_k)
                res = gather_k(n)
                e[1].record(s_k)
                gtime["events"].append(e)
                keep(first, res)
                return
            keep(first, gather_k(n))  # the assembled frames on rank 0 (RCCL gather for N > 1)

    def complete(j, first, n):  # gloo: the launch's host tiles are gathered once its render is done
        if gloo:
            _, _, gather_k, s_k, _ = ctxs[j % F]
            s_k.synchronize()
            t = time.perf_counter()
            res = gather_k(n)
            if gtime["on"]:
                gtime["host_s"] += time.perf_counter() - t
            keep(first, res)

    def run_frames(first, count):
        """frames first .. first + count - 1 in launches of B (the last takes the rest), F in flight"""
        work = [(j, f, min(B, first + count - f)) for j, f in enumerate(range(first, first + count, B))]
        for i, w in enumerate(work):
            launch(*w)
            if i >= F - 1:
                complete(*work[i - F + 1])
        for w in work[max(0, len(work) - F + 1):]:
            complete(*w)

    def sync_all():
        for c in ctxs:
            c[3].synchronize()

    # executed steps of this rank's rows (untimed; the debug variant of the kernel)
    _, _, steps_full = r.render_debug(cams[0], params, W, H)
    torch.cuda.synchronize(dev)
    balance = None
    balance_used = args.balance if args.balance != "auto" else ("cost" if args.camera == "static" else "cyclic")
    if distributed and balance_used == "cost":
        # rank 0 prices the blocks from the first frame's per-wave steps and
        # budget events and sends every rank the same lists (a rank whose own
        # cost map differed would otherwise render rows rank 0 does not expect)
        obj = [None]
        if rank == 0:
            costs = D.block_costs(r.wave_costs(cams[0], params, W, H, stream=stream))
            lst = D.balanced_blocks(costs, world)
            loads = [sum(costs[b] for b in l if b >= 0) for l in lst]
            cyc = [sum(costs[b] for b in D.blocks_of(k, world, H, BLOCK_ROWS)) for k in range(world)]
            obj = [(lst, {"max_over_mean": round(max(loads) / (sum(loads) / world), 4),
                          "cyclic_max_over_mean": round(max(cyc) / (sum(cyc) / world), 4),
                          "lists_from": "rank 0 (broadcast)"})]
        dist.broadcast_object_list(obj, src=0, device=None if gloo else dev)
        lists[0], balance = obj[0]
        for c in ctxs:
            c[2].set_lists(lists[0])
        rows_mine = D.rows_of_list(lists[0][rank], H, BLOCK_ROWS)
        # a moving camera: re-price every `every` launches
        rp["every"] = args.reprice if args.reprice >= 0 else (F if args.camera == "flyby" else 0)
        sched[0] = D.ListSchedule(lists[0], F, rp["every"], B)
        if rp["every"] and rank == 0:
            rp["pricer"] = new_renderer()
            rp["stream"] = torch.cuda.Stream(dev)
    else:
        rows_mine = D.rows_of(rank, world, H, BLOCK_ROWS)
    sigma_steps_frame = int(steps_full.sum().item())
    sigma_steps_mine = int(steps_full[rows_mine].sum().item())
    # candidate critical bands: the 16-row bands of workgroup tiles holding the
    # frame's longest rays (the slowest of them is timed below)
    band_max = steps_full.max(dim=1).values[: H // 16 * 16].view(-1, 16).max(dim=1).values
    band_rows = [int(b) * 16 for b in band_max.argsort(descending=True)[:CRITICAL_CANDIDATES].tolist()] or [0]
    del steps_full, band_max

    run_frames(0, warm)
    sync_all()

    # ---- the timed region: K frames in launches of B, F in flight, per-kernel
    # HIP events on every context's stream (integrate / shade / resume of each launch)
    per_ctx = -(-args.steps // (B * F)) + 1
    dump_from[0] = warm
    for c in ctxs:
        c[0].set_timing(per_ctx)
    if distributed:
        dist.barrier()
    sync_all()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    gtime["on"] = True
    run_frames(warm, args.steps)
    sync_all()
    torch.cuda.synchronize(dev)
    t_mine = time.perf_counter() - t0  # this rank's own span, before waiting for the others
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    gtime["on"] = False
    # parity of the last timed frame (rank 0 holds it assembled), before any
    # further launch reuses its context's tile
    parity = None
    if rank == 0 and last[0] is not None:
        first, batch = last[0]
        parity = frame_parity(args, W, H, N, quality, use_assets, batch[-1], first + batch.shape[0] - 1)
    ktimes = np.concatenate([c[0].kernel_times(per_ctx) for c in ctxs], axis=0)
    # frames of each row of ktimes: launch j of the window ran on context j % F
    # (run_frames), and each context lists its own launches in order
    sizes = [min(B, args.steps - f) for f in range(0, args.steps, B)]
    launch_frames = np.array([sizes[j] for k in range(len(ctxs)) for j in range(k, len(sizes), F)], dtype=np.int64)
    assert launch_frames.size == ktimes.shape[0], (launch_frames.size, ktimes.shape)
    if args.dump_frames and rank == 0:
        Path(args.dump_frames).mkdir(parents=True, exist_ok=True)
        for f, fr in frames.items():
            np.save(Path(args.dump_frames) / f"frame_{f}.npy", fr.cpu().numpy())
        frames.clear()
    for c in ctxs:
        c[0].set_timing(0)

    # frame latency (untimed for `value`): one launch of B frames alone on
    # context 0; every frame of it is done when the launch is
    lat_launches = 5
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for _ in range(lat_launches):
        render(r, warm, min(B, args.steps), tile, stream)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    latency_ms = ev0.elapsed_time(ev1) / lat_launches

    # Single-frame launches (untimed for `value`; the reference draws one frame
    # per loop iteration, src/main.cpp:318-319, camera re-uploaded each time,
    # :429): one frame alone (B = 1, F = 1: the interactive latency) and
    # single-frame launches with 4 in flight (B = 1, F = 4).
    single = None
    if world == 1 and args.single_frame == "on":
        single = single_frames(new_renderer, ctxs, cams, params, W, H, dev, args.single_split, render, warm,
                               restore=split)

    # the reference's loop: one un-culled frame against one culled frame, alone
    speedup_ref = None
    if args.reference_loop == "on" and not args.no_cull and rank == 0:
        def alone_integrate_ms(cull):
            r.set_culling(cull)
            r.set_timing(2)
            for _ in range(2):
                r.render_blocks(cams[0], params, W, H, BLOCK_ROWS, rank, world, out=tile[0], stream=stream)
            torch.cuda.synchronize(dev)
            t = float(r.kernel_times(2)[-1, 0])
            r.set_timing(0)
            return t
        culled = alone_integrate_ms(True)
        unculled = alone_integrate_ms(False)
        r.set_culling(True)
        speedup_ref = {"culled_ms": round(culled, 4), "reference_loop_ms": round(unculled, 4),
                       "speedup": round(unculled / culled, 2)}

    if balance is not None and rp["every"]:
        balance["reprice_every_launches"] = rp["every"]
        balance["repriced"] = sched[0].count
        if rank == 0:
            balance["reprice_choices"] = rp["choices"]
    last_camera = None
    if distributed and args.camera == "flyby" and rank == 0:
        # how even the lists in use (and the frame-0 lists, cyclic rows) are on
        # the last timed camera, by its full-resolution cost map (untimed)
        cost_last = D.block_costs(r.wave_costs(cams[warm + args.steps - 1], params, W, H, stream=stream).cpu())
        cyclic_lists = [D.blocks_of(k, world, H, BLOCK_ROWS) for k in range(world)]
        in_use = (sched[0].ctx[(len(range(warm, warm + args.steps, B)) - 1) % F] if sched[0] is not None
                  else lists[0] if lists[0] is not None else cyclic_lists)
        last_camera = {"lists_in_use": round(D.max_over_mean(in_use, cost_last), 4),
                       "cyclic": round(D.max_over_mean(cyclic_lists, cost_last), 4)}
        if lists[0] is not None:
            last_camera["frame0_lists"] = round(D.max_over_mean(lists[0], cost_last), 4)
    ranks = None
    if distributed:  # max over ranks (RCCL reduces device tensors, gloo host ones)
        t = torch.tensor([elapsed, latency_ms], dtype=torch.float64, device=None if gloo else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, latency_ms = float(t[0]), float(t[1])
        # what each rank did, so that an N-GPU line documents itself
        gms = gtime["host_s"] * 1e3 + sum(a.elapsed_time(b) for a, b in gtime["events"])
        props = torch.cuda.get_device_properties(dev)
        mine = {"rank": rank, "world_size": dist.get_world_size(), "local_rank": local, "device": dev.index,
                "device_name": props.name, "pci_bus_id": getattr(props, "pci_bus_id", None),
                "visible_devices": os.environ.get("HIP_VISIBLE_DEVICES", os.environ.get("CUDA_VISIBLE_DEVICES")),
                "rows": len(rows_mine), "share_ms_per_frame": round(t_mine * 1e3 / args.steps, 4),
                "integrate_kernel_ms": round(float(ktimes[:, 0].mean()), 4),
                "gather_ms_per_frame": round(gms / args.steps, 4),
                "gather": "host-staged gloo" if gloo else "RCCL gather, HIP events on the launch streams"}
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)

    ms_per_step = elapsed * 1e3 / args.steps
    mpix_s = W * H * args.steps / elapsed / 1e6

    # Critical path (untimed, after the timed regions): that band rendered on
    # its own (~120 workgroups, under one wave per SIMD), on a second context
    # so the frame's launch-order state stays untouched. Its time is the
    # slowest waves' latency without contention.
    critical = None
    if rank == 0 and world == 1 and args.critical_path == "on":
        rb = new_renderer()

        def band_time(band, reps):
            for _ in range(2):
                rb.render(cams[0], params, W, H, *band, stream=stream)
            times = []
            for _ in range(reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                rb.render(cams[0], params, W, H, *band, stream=stream)
                e1.record(stream)
                torch.cuda.synchronize(dev)
                times.append(e0.elapsed_time(e1))
            return sorted(times)[len(times) // 2]

        # the longest rays' band is not always the slowest (events differ):
        # time the candidates once, then the slowest of them five times
        cands = [(b, min(H, b + 16)) for b in band_rows]
        band = max(cands, key=lambda c: band_time(c, 1))
        band_ms = band_time(band, 5)
        rb.close()
        critical = {"band_rows": list(band), "band_ms": round(band_ms, 4),
                    "frac_of_frame_latency": round(band_ms / latency_ms, 3)}

    if rank == 0:
        roofline = make_roofline(args, W, H, N, world, F, B, ms_per_step, ktimes, launch_frames,
                                 latency_ms, sigma_steps_frame, sigma_steps_mine, len(rows_mine), critical,
                                 speedup_ref)
        cpu = None
        if args.cpu_baseline == "auto" and world == 1:
            cpu = cpu_baseline(cams[0], W, H, N, args.cpu_sample_rows)
        tex_desc = (f"the reference's assets/textures ({quality} skybox, uv_checker, cubemap; decoded to stb_image's bytes)"
                    if use_assets else f"procedural stand-in textures ({quality} skybox)")
        line = {
            "metric": ("Mpixels/s at 1920x1080, 2000 geodesic steps; 1/2/4/8 MI355X"
                       if (W, H, N) == WORKLOADS["headline"] else f"Mpixels/s at {W}x{H}, {N} geodesic steps"),
            "value": round(mpix_s, 3),
            "unit": "Mpixels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": ("synthetic: " + ("the max-capacity scene (scenes.scene_stress: 21 objects, 10 materials, 4 lights)"
                                      if args.scene == "stress" else "default scene of src/main.cpp:222-268")
                     + (", the press-R overlay (scenes.test_ray_overlay, 1000 points)" if test_ray is not None else "")
                     + f", {tex_desc}"),
            "config": {
                "workload": (f"{W}x{H} {args.mode}-mode frame"
                             + (f" (curved_percentage {args.curved_percentage})" if args.mode.startswith("half") else "")
                             + f", {N} geodesic steps, {args.scene} scene"
                             + (", test-ray overlay" if test_ray is not None else "") + ", percent_black "
                             + ("off" if args.percent_black < 0 else str(args.percent_black))
                             + (", flyby camera (a new camera every frame)" if args.camera == "flyby" else "")),
                "width": W,
                "height": H,
                "max_steps": N,
                "camera": args.camera,
                "textures": "assets" if use_assets else "standin",
                "skybox": quality,
                "tiling": ((f"cost-balanced {BLOCK_ROWS}-row blocks over {world} ranks (per-wave steps and events of "
                            "the first frame), " if balance else f"block-cyclic {BLOCK_ROWS}-row bands over {world} rank(s), ")
                           + ("RCCL gather to rank 0" if not gloo else "gloo gather of host-staged tiles to rank 0")),
                "balance": balance,
                "balance_policy": {"requested": args.balance, "used": balance_used if distributed else None},
                "last_camera_max_over_mean": last_camera,
                "dist_backend": args.dist_backend if distributed else None,
                "launches_in_flight": F,
                "stream_priority": args.stream_priority,
                "frames_per_launch": B,
                "frames_in_flight": F * B,
                # the timed window's launches (frames each): a window that is
                # not a multiple of B ends with a shorter launch
                "launch_sizes": [min(B, args.steps - f) for f in range(0, args.steps, B)],
                "split_tiles": args.split,
                "gpu_max_hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
                "frame_latency_ms": round(latency_ms, 4),
                "single_frame": single,
                "culling": not args.no_cull,
                "world_size": world,
                "ranks": ranks,
            },
            "roofline": roofline,
            "cpu_baseline": cpu,
            "parity": parity,
        }
        print(json.dumps(line), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()
    for c in ctxs:
        c[0].close()
    if rp["pricer"] is not None:
        rp["pricer"].close()


def single_frames(new_renderer, ctxs, cams, params, W, H, dev, split_arg, render, first,
                  restore=(0, 16, 1), frames=20, alone_reps=15, inflight=4):
    """Single-frame launches (sr_render_blocks of the whole frame): `alone` =
    one frame at a time, each waited for (median of alone_reps; HIP events on
    the context's stream), `inflight` = `frames` frames in launches of one,
    `inflight` contexts and streams round robin, no host wait between them
    (wall clock around the sequence, synchronised on both sides). Both on
    contexts that have learned the frame's launch order. split_arg: split
    tiles (sr_set_split) on these contexts for the measurement."""
    import statistics

    import torch

    split = [int(x) for x in split_arg.split(":")] + [16, 1][len(split_arg.split(":")) - 1:]
    pool = [(c[0], c[1], c[3]) for c in ctxs[:inflight]]
    extra = []
    while len(pool) < inflight:
        rk = new_renderer()
        extra.append(rk)
        pool.append((rk, torch.zeros((1,) + tuple(ctxs[0][1].shape[1:]), dtype=torch.uint8, device=dev),
                     torch.cuda.Stream(dev)))
    n_cam = len(cams)

    def learn(sp):  # each context learns the single-frame launch order (and split tiles) first
        for rk, _, _ in pool:
            rk.set_split(*sp)
        for k, (rk, tile_k, s_k) in enumerate(pool):
            with torch.cuda.stream(s_k):
                for j in range(2):
                    render(rk, (first + k + j) % n_cam, 1, tile_k, s_k)
        for _, _, s_k in pool:
            s_k.synchronize()

    def configure(k, sp, latency):  # context k of the pool: split tiles, latency mode, launch order learned
        rk, tile_k, s_k = pool[k]
        rk.set_split(*sp)
        rk.set_latency_mode(latency)
        with torch.cuda.stream(s_k):
            for j in range(2):
                render(rk, (first + k + j) % n_cam, 1, tile_k, s_k)
        s_k.synchronize()

    def time_one(k, j):
        rk, tile_k, s_k = pool[k]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(s_k):
            e0.record(s_k)
            render(rk, (first + j) % n_cam, 1, tile_k, s_k)
            e1.record(s_k)
        s_k.synchronize()
        return e0.elapsed_time(e1)

    # one frame at a time on three contexts of the pool: split tiles (the
    # frame's costliest tiles' rays in sparse waves), the default launch, and
    # the latency mode (sr_set_latency_mode: a 2-step fast loop) without split
    # tiles (with them it measured slower: s8). The three are timed round
    # robin, so drift in the GPU's state over the measurement (clocks, the
    # pipeline run before it) reaches all three alike.
    configure(0, split, False)
    configure(1, (0, 16, 1), False)
    configure(2, (0, 16, 1), True)
    times = [[], [], []]
    for j in range(alone_reps):
        for k in range(3):
            times[k].append(time_one(k, j))
    alone, alone_unsplit, alone_latency = (statistics.median(t) for t in times)
    for rk, _, _ in pool:
        rk.set_latency_mode(False)
    learn((0, 16, 1))  # the in-flight launches below: default launches on every context
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for j in range(frames):
        rk, tile_k, s_k = pool[j % inflight]
        with torch.cuda.stream(s_k):
            render(rk, (first + j) % n_cam, 1, tile_k, s_k)
    for _, _, s_k in pool:
        s_k.synchronize()
    torch.cuda.synchronize(dev)
    per = (time.perf_counter() - t0) * 1e3 / frames
    for rk, _, _ in pool:
        rk.set_split(*restore)
    for rk in extra:
        rk.close()
    return {
        "alone": {"frames_per_launch": 1, "launches_in_flight": 1, "ms_per_frame": round(alone, 4),
                  "mpix_s": round(W * H / alone / 1e3, 3), "runs": alone_reps, "stat": "median, HIP events, round robin with the two below",
                  "split_tiles": split_arg, "latency_mode": False},
        "alone_default": {"ms_per_frame": round(alone_unsplit, 4), "mpix_s": round(W * H / alone_unsplit / 1e3, 3),
                          "split_tiles": "0", "latency_mode": False},
        "alone_latency_mode": {"ms_per_frame": round(alone_latency, 4),
                               "mpix_s": round(W * H / alone_latency / 1e3, 3), "split_tiles": "0",
                               "latency_mode": True},
        "inflight": {"frames_per_launch": 1, "launches_in_flight": inflight, "ms_per_frame": round(per, 4),
                     "mpix_s": round(W * H / per / 1e3, 3), "frames": frames, "stat": "wall clock",
                     "split_tiles": "0"},
    }


FRAME_HASHES = ROOT / "tests" / "golden" / "frame_hashes.npz"


def frame_parity(args, W, H, N, quality, use_assets, frame, index):
    """One timed frame against the oracle's frame (tests/golden/frame_hashes.npz,
    made by tests/golden/make_frame_hashes.py in the build container): sha256
    of every RGBA8 row equal, and the frame hash over them. Only the inputs the
    fixture was made with (the app's static camera, the reference's textures,
    curved mode, noise mask off) have one."""
    import numpy as np

    fr = frame.cpu().numpy() if hasattr(frame, "cpu") else np.asarray(frame)
    fr = np.ascontiguousarray(fr[:H])
    rows_sha = np.stack([np.frombuffer(hashlib.sha256(fr[y].tobytes()).digest(), dtype=np.uint8) for y in range(H)])
    digest = hashlib.sha256(rows_sha.tobytes()).hexdigest()
    out = {"frame": index, "frame_sha": digest[:16], "frame_sha_match": None}
    if not (args.camera == "static" and use_assets and args.mode == "curved" and args.percent_black < 0):
        out["reason"] = "no oracle fixture for these inputs"
        return out
    variant = scene_variant(args)
    if args.scene == "stress" and args.test_ray == "on":
        out["reason"] = "no oracle fixture for the stress scene with the test ray"
        return out
    if not FRAME_HASHES.exists():
        out["reason"] = "tests/golden/frame_hashes.npz missing"
        return out
    with np.load(FRAME_HASHES) as z:
        for cfg in sorted({k.split("/")[0] for k in z.files}):
            if f"{cfg}/config" not in z.files or tuple(int(v) for v in z[f"{cfg}/config"]) != (W, H, N):
                continue
            if (bytes(z[f"{cfg}/variant"]).decode() if f"{cfg}/variant" in z.files else "default") != variant:
                continue
            if bytes(z[f"{cfg}/skybox"]).decode() != quality:
                continue
            rows = z[f"{cfg}/rows"]
            ok = bool(np.array_equal(rows_sha[rows], z[f"{cfg}/rgba_sha"]))
            out.update(fixture=f"tests/golden/frame_hashes.npz {cfg}", rows_compared=int(len(rows)),
                       rows_differing=int((rows_sha[rows] != z[f"{cfg}/rgba_sha"]).any(-1).sum()))
            if f"{cfg}/frame_sha" in z.files:
                ok = ok and digest == bytes(z[f"{cfg}/frame_sha"]).hex()
            out["frame_sha_match"] = ok
            return out
    out["reason"] = "no oracle fixture for this size"
    return out


def scene_variant(args) -> str:
    """The scene variant a bench line, its frame-hash fixture and its counter
    records are keyed by: default, stress (--scene stress) or testray (--test-ray on)."""
    return "stress" if args.scene == "stress" else ("testray" if args.test_ray == "on" else "default")


def counter_variant(args) -> str:
    """The key of a line's PMC / traffic records: the scene variant, plus any
    option that changes the integrate kernel's work per frame (mode, noise
    mask, no culling, a moving camera). Only the lines the roofline sessions
    measure (default, stress, testray) find records; the others print
    `frac` null instead of another workload's counters."""
    v = scene_variant(args)
    mods = []
    if getattr(args, "mode", "curved") != "curved":
        mods.append(args.mode)
    if getattr(args, "percent_black", -1.0) >= 0.0:
        mods.append("noise")
    if getattr(args, "no_cull", False):
        mods.append("nocull")
    if getattr(args, "camera", "static") != "static":
        mods.append(args.camera)
    return "_".join([v] + mods) if mods else v


def profile_record(path: str, kind: str, variant: str) -> Path:
    """--pmc-json / --traffic-json, or profiles/<kind>_latest[_<variant>].json."""
    if path:
        return Path(path)
    return ROOT / "profiles" / (f"{kind}_latest.json" if variant == "default" else f"{kind}_latest_{variant}.json")


def load_matching(path, W, H, N, world, variant="default"):
    """A profiles/*.json record if it was measured on this config, scene variant and kernel source."""
    p = Path(path)
    if not p.exists():
        return None
    try:
        rec = json.loads(p.read_text())
    except Exception:  # noqa: BLE001
        return None
    if (rec.get("width"), rec.get("height"), rec.get("max_steps")) != (W, H, N):
        return None
    if rec.get("kernel_sha") not in (None, kernel_sha()):
        return None
    if rec.get("variant", "default") != variant:
        return None
    return rec


def launch_accounting(ktimes, launch_frames, ms_per_step):
    """Kernel time of the timed window's launches, which need not be equal
    (20 frames in launches of 16 are [16, 4]): per integrate launch
    (`kernel_ms`, the plain mean rocprofv3 --stats reports), per launch size,
    per frame (total duration / frames), and `overlap` = total integrate
    duration / the window (frames x ms_per_step): the mean number of
    integrate launches in flight. ktimes: [launches, 3] ms (integrate, shade,
    resume); launch_frames: frames of each launch."""
    import numpy as np

    kt = np.asarray(ktimes, dtype=np.float64).reshape(-1, 3)
    lf = np.asarray(launch_frames, dtype=np.int64).reshape(-1)
    assert kt.shape[0] == lf.size and lf.size > 0
    window_ms = float(lf.sum()) * ms_per_step
    by_size = {str(int(b)): round(float(kt[lf == b, 0].mean()), 4) for b in sorted(set(lf.tolist()), reverse=True)}
    return {
        "kernel_ms": round(float(kt[:, 0].mean()), 4),
        "kernel_ms_by_launch_frames": by_size,
        "kernel_ms_per_frame": round(float(kt[:, 0].sum() / lf.sum()), 4),
        "launch_frames": lf.tolist(),
        "overlap": round(float(kt[:, 0].sum()) / window_ms, 3),
        "pipeline_ms_per_frame": {"integrate": round(float(kt[:, 0].sum() / lf.sum()), 4),
                                  "shade": round(float(kt[:, 1].sum() / lf.sum()), 4),
                                  "resume": round(float(kt[:, 2].sum() / lf.sum()), 4)},
    }


def make_roofline(args, W, H, N, world, F, B, ms_per_step, ktimes, launch_frames, latency_ms,
                  sigma_steps_frame, sigma_steps_mine, rows_mine, critical, speedup_ref):
    """Roofline of the dominant kernel (sr_integrate_kernel: ray generation,
    the step loop and every intersection test), on rank 0's launches.

    The path is FP32-VALU bound (no contraction for MFMA, ~4 B of compulsory
    HBM traffic per pixel). `achieved` is the FP32 work the kernel EXECUTES:
    the FLOP per frame counted by the hardware (SQ_INSTS_VALU_FLOPS_FP32 +
    _TRANS per integrate dispatch over the dispatch's B frames, rocprofv3
    --pmc on this kernel source and config, calibrated by
    tools/microbench/flops_calib.hip: profiles/pmc_latest.json) times the
    frames per second of this run, so `frac` is utilisation of the FP32 peak. `kernel_ms` is the same run's mean
    integrate-launch duration (HIP events on each launch's stream): it is
    what the rocprofv3 --stats summary of this command reports; launches of
    unequal size are also reported per size and per frame, and `overlap` is
    the total integrate duration over the timed window (launch_accounting)."""
    variant = counter_variant(args)
    pmc = load_matching(profile_record(args.pmc_json, "pmc", variant), W, H, N, world, variant)
    share = sigma_steps_mine / max(1, sigma_steps_frame)  # rank 0's share of the frame's steps
    executed = None
    achieved = None
    valu_issue = None
    per_frame = (pmc or {}).get("frames_per_launch", 1)
    if pmc and pmc.get("flop_per_launch"):
        executed = pmc["flop_per_launch"] / per_frame * share  # per frame of this rank's share
        achieved = executed / (ms_per_step * 1e-3) / 1e12
        if pmc.get("valu_insts_per_launch"):
            # wave64 VALU instructions x 2 cycles on a SIMD-32 over the SIMD-cycles at 2.4 GHz
            valu_issue = (pmc["valu_insts_per_launch"] / per_frame * share * 2.0
                          / (SIMDS * CLOCK_GHZ * 1e9 * ms_per_step * 1e-3))
    traffic = None
    tr = load_matching(profile_record(args.traffic_json, "traffic", variant), W, H, N, world, variant)
    if tr and world == 1:
        traffic = tr.get("hbm_bytes_per_frame", tr.get("hbm_bytes_per_launch"))
    hbm_bytes = rows_mine * W * 4  # compulsory RGBA8 store; textures stay cache resident
    ref_flop = sigma_steps_mine * FLOP_PER_STEP + rows_mine * W * FLOP_PER_PIXEL
    return {
        "bound": "valu",
        "kernel": "sr_integrate_kernel",
        "achieved": None if achieved is None else round(achieved, 3),
        "peak": PEAK_FP32_TFLOPS,
        "unit": "TFLOP/s",
        "frac": None if achieved is None else round(achieved / PEAK_FP32_TFLOPS, 4),
        "traffic": traffic,
        "executed_flop_per_frame": None if executed is None else round(executed),
        "valu_issue_frac": None if valu_issue is None else round(valu_issue, 4),
        **launch_accounting(ktimes, launch_frames, ms_per_step),
        "launches_in_flight": F,
        "frames_per_launch": B,
        # this rank's executed ray-steps of one frame (the debug render of the
        # first camera), and of one launch of B frames (static camera: B times
        # that; a flyby's frames differ, so none)
        "steps_per_frame": sigma_steps_mine,
        "steps_per_launch": sigma_steps_mine * B if args.camera == "static" else None,
        "mean_steps_per_pixel": round(sigma_steps_frame / (W * H), 2),
        "pmc_source": None if not pmc else pmc.get("source"),
        # the un-culled reference loop (360 FLOP per step) and the
        # measured speed-up of the culled kernel over it; not utilisation
        "reference_loop": {"flop_per_frame": ref_flop, **(speedup_ref or {})},
        "critical_path": critical,
        "hbm": {
            "achieved": round(hbm_bytes / (ms_per_step * 1e-3) / 1e9, 3),
            "peak": PEAK_HBM_GBS,
            "unit": "GB/s",
            "frac": round(hbm_bytes / (ms_per_step * 1e-3) / 1e9 / PEAK_HBM_GBS, 6),
            "algorithmic_bytes": hbm_bytes,
        },
    }


def cgroup_cpus():
    """CPUs the cgroup's quota grants (cgroup v2 cpu.max, v1 cfs quota), or None."""
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            return max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    try:
        q = int(Path("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read_text())
        per = int(Path("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read_text())
        if q > 0:
            return max(1, q // per)
    except (OSError, ValueError):
        pass
    return None


def host_cpu():
    """(threads, basis): every thread sched_getaffinity allows this process,
    bounded by the cgroup's CPU quota when one is set (more threads than the
    quota only time-slice), plus nproc and the CPU model for the line."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = nproc
    quota = cgroup_cpus()
    threads = min(aff, quota) if quota else aff
    model = "unknown"
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                model = line.split(":", 1)[1].strip()
                break
    except Exception:  # noqa: BLE001
        pass
    return {"threads": threads, "affinity": aff, "cgroup_cpus": quota, "nproc": nproc, "model": model,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


# BASELINE.json config 1: one press-R ray of 2000 steps from the app's camera
# position (src/main.cpp:222), the directions SURVEY.md Appendix B timed
PRESSR_RAYS = (((0.0, 2.0, 15.0), (1.0, -2.0, -15.0)), ((0.0, 2.0, 15.0), (3.0, -2.0, -15.0)))
# the other sweeps of BASELINE.md §3: (name, width, height, max_steps)
CPU_SWEEPS = (("640x360/1000", 640, 360, 1000), ("1920x1080/2000", 1920, 1080, 2000),
              ("3840x2160/4000", 3840, 2160, 4000))


def cpu_baseline(cam, W, H, N, sample_rows, budget_s=2.5, sweeps=CPU_SWEEPS, rays=PRESSR_RAYS):
    """The reference's press-R CPU geodesic (src/main.cpp:73-124, double
    temporaries, a std::vector per ray) on this host, the
    oracle's restatement of it ("port"; the reference app needs glm and GLFW,
    absent here):
      - value: swept over every row of this frame (every pixel's camera
        ray, N steps; BASELINE.md §3 "wall time over the full frame"), all
        threads of host_cpu(), -O2, median of 3 (sample_rows > 0: that many
        rows around the centre instead, labelled as a sample);
      - O0: the same at -O0 (the reference's CMake default build), on a
        quarter of those rows (a sample, labelled);
      - configs: config 1 (one ray at N = 2000, microseconds per ray on one
        thread) and the 640x360 / 1000, 1920x1080 / 2000 and 3840x2160 / 4000
        sweeps: the full frame where it fits the time budget, else a row
        sample around the frame centre (labelled);
      - like_for_like: the reference shader itself (with scene intersection
        and shading) on SwiftShader in the survey container, BASELINE.md §2,
        quoted as context (it is not run here: the shader lives in the
        reference, which does not travel to the GPU box)."""
    import statistics

    import numpy as np

    import srpkg

    oracle = srpkg.load_oracle()
    hc = host_cpu()
    threads = hc["threads"]

    def rows_for(w, h, n, target_s):
        t = time.perf_counter()  # calibrate on 8 rows through the centre
        oracle.pressr_sweep(cam, w, h, n, 2, h // 2 - 4, h // 2 + 4, threads)
        dt = max(time.perf_counter() - t, 1e-3)
        return int(min(h, max(8, 8 * target_s / dt)))

    def rate(fn, w, h, n, rows):
        y0 = max(0, h // 2 - rows // 2)  # rows [y0, y1) around the frame centre
        y1 = min(h, y0 + rows)
        runs, pts = [], 0
        for _ in range(3):
            t = time.perf_counter()
            pts = fn(cam, w, h, n, 2, y0, y1, threads)
            runs.append(time.perf_counter() - t)
        dt = statistics.median(runs)
        return (y1 - y0) * w / dt / 1e6, y0, y1, pts, dt

    if sample_rows <= 0:
        sample_rows = H  # the full frame
    v2, y0, y1, pts, dt = rate(oracle.pressr_sweep, W, H, N, sample_rows)
    full = (y0, y1) == (0, H)
    o0 = None
    if hasattr(oracle, "pressr_sweep_O0"):
        try:
            v0, a0, b0, _, d0 = rate(oracle.pressr_sweep_O0, W, H, N, max(8, sample_rows // 4))
            o0 = {"value": round(v0, 4), "sample": f"rows [{a0},{b0}) x {W} px, median {d0:.2f} s"}
        except (FileNotFoundError, OSError):
            o0 = None
    configs = {}
    for pos, fwd in rays:  # config 1: microseconds per ray, one thread
        v = np.array(fwd, dtype=np.float32)
        v = (v * np.float32(1.0 / np.sqrt(np.float32(np.dot(v, v))))).tolist()
        n_pts = oracle.pressr_ray_repeat(pos, v, 2000, 2, 1)
        reps = 50
        while True:
            t = time.perf_counter()
            oracle.pressr_ray_repeat(pos, v, 2000, 2, reps)
            el = time.perf_counter() - t
            if el > 0.3 or reps > 1 << 22:
                break
            reps *= 4
        configs[f"config1 dir {fwd}"] = {"value": round(el / reps * 1e6, 3), "unit": "us/ray", "cores": 1,
                                         "points": n_pts, "sample": f"{reps} traces, N = 2000, pos {pos}"}
    for name, w, h, n in sweeps:
        if (w, h, n) == (W, H, N):
            configs[name] = {"value": round(v2, 4), "unit": "Mpixels/s", "cores": threads, "same_as": "value"}
            continue
        rv, a, b, p_, d = rate(oracle.pressr_sweep, w, h, n, rows_for(w, h, n, budget_s))
        configs[name] = {"value": round(rv, 4), "unit": "Mpixels/s", "cores": threads,
                         "sample": ("full frame" if (a, b) == (0, h) else f"sample: rows [{a},{b}) of {h}")
                         + f" x {w} px, {p_} points, median of 3 runs {d:.2f} s"}
    return {
        "value": round(v2, 4),
        "unit": "Mpixels/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"full frame: press-R loop (src/main.cpp:73-124) over all {H} rows x {W} px of the {W}x{H} frame, "
                   if full else
                   f"sample: press-R loop (src/main.cpp:73-124) over rows [{y0},{y1}) x {W} px of the {W}x{H} frame, ")
                  + f"{N} steps, {pts} points, median of 3 runs {dt:.2f} s, -O2, {threads} threads",
        "cores_basis": (f"sched_getaffinity allows {hc['affinity']} CPUs"
                        + (f", the cgroup quota {hc['cgroup_cpus']}" if hc["cgroup_cpus"] else ", no cgroup quota")
                        + f"; nproc {hc['nproc']}"),
        "nproc": hc["nproc"],
        "cpu_model": hc["model"],
        "O0": o0,
        "configs": configs,
        "note": "integrator only: the press-R loop does no scene intersection or shading (BASELINE.md §3)",
        "like_for_like": {"value": 0.00225, "unit": "Mpixels/s", "cores": 8,
                          "what": "the reference shader (assets/shaders/black_hole.frag, with intersection and "
                                  "shading) on SwiftShader 4.1, 1920x1080 / 2000 steps, 922 s per frame",
                          "where": "survey container, 8-core Xeon (BASELINE.md §2, SURVEY App. A); quoted as "
                                   "context, not run on this host"},
    }


if __name__ == "__main__":
    main()
