#!/usr/bin/env python3
"""Headline benchmark: Mpixels/s at 1920x1080, 2000 geodesic steps, default
scene (BASELINE.json `metric`, config 3), curved mode, noise mask off.

One step = one full frame: every rank renders its block-cyclic share of the
frame's rows (8-row blocks, block b -> rank b % N) with the gfx950 kernel,
then the tiles are gathered to rank 0 over RCCL (torch.distributed "nccl").
`value` = frame pixels x K / (max over ranks of the timed span) — strong
scaling (the frame is fixed, the GPUs share it).

Inputs are resident in HBM before timing (scene, textures, step table).
Also reported: the kernel's roofline (algorithmic FLOP/s from the executed
step count, SURVEY §8d cost model, HIP events on the render stream) and the
reference's CPU press-R geodesic loop swept over a sample of the frame's
pixels on this host (cpu_baseline; oracle restatement, "port").

  python bench.py [--gpus N --steps K --warmup W]
  torchrun --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

# algorithmic cost per executed chord step in the default
# scene (integrator 71 + black hole 17 + six objects, all-miss) and per pixel.
FLOP_PER_STEP = 360.0
FLOP_PER_PIXEL = 150.0
FLOP_PER_PIXEL_INTEGRATE = 100.0  # ray generation (P3, ~40) + orbital seed (P6, ~60); lighting is the shade kernel's
# MI355X_MICROARCH.md: FP32 vector peak (packed FMA) and HBM3E peak.
PEAK_FP32_TFLOPS = 157.3
PEAK_FP32_UNPACKED_TFLOPS = 78.6
PEAK_HBM_GBS = 8000.0
BLOCK_ROWS = 8
CRITICAL_CANDIDATES = 8  # 16-row bands timed alone for roofline.critical_path
# BASELINE.json configs: name -> (width, height, max_steps)
WORKLOADS = {
    "small": (640, 360, 1000),       # config 2
    "headline": (1920, 1080, 2000),  # config 3 (the metric)
    "4k": (3840, 2160, 4000),        # config 4
    "8k": (7680, 4320, 8000),        # config 5 (offline still)
}
MODES = {"curved": 0, "flat": 1, "half_width": 2, "half_height": 3}


def frames_in_flight(width, height, world):
    """Default frames in flight per GPU: 4 while a rank holds at least a
    quarter of a 1080p frame, 6 below that."""
    return 4 if width * height / world >= 1920 * 1080 / 4 else 6


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
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
    ap.add_argument("--no-cull", action="store_true", help="exhaustive per-object tests (reference loop)")
    ap.add_argument("--inflight", type=int, default=0,
                    help="frames in flight per GPU, each on its own context and stream (0: 4, or 6 when the rank holds under a quarter of a 1080p frame)")
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--critical-path", choices=["on", "off"], default="on",
                    help="time the slowest row bands alone (extra launches of the same kernel; off for rocprof stats)")
    ap.add_argument("--cpu-sample-rows", type=int, default=0, help="rows of the frame swept on the CPU (0 = auto)")
    ap.add_argument("--traffic-json", default=str(ROOT / "profiles" / "traffic_latest.json"))
    ap.add_argument("--pmc-json", default=str(ROOT / "profiles" / "pmc_latest.json"))
    return ap.parse_args()


def main():
    args = parse()
    # every in-flight frame's stream needs a hardware queue of its own (HIP's
    # default is 4 per process); must be set before the HIP runtime starts
    if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 8:
        os.environ["GPU_MAX_HW_QUEUES"] = "8"
    import numpy as np
    import torch
    import torch.distributed as dist

    import srpkg

    pkg = srpkg.load_package()
    abi, sc = pkg.abi, pkg.scenes

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    if distributed:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    W0, H0, N0 = WORKLOADS[args.workload]
    W, H, N = args.width or W0, args.height or H0, args.max_steps or N0

    # ---- inputs resident in HBM ---------------------------------------------------
    scene = sc.scene_default(textured=True)
    cam = abi.default_camera()
    params = abi.default_params(max_steps=N, percent_black=args.percent_black, raytrace_type=MODES[args.mode],
                                curved_percentage=args.curved_percentage)
    # Frames in flight: a frame's time is bounded by the latency of its
    # longest rays' waves, which a share of 1/N of the rows
    # does not shorten; independent frames on their own contexts and streams
    # fill the SIMDs those waves leave idle. Step f renders frame f on context
    # f % F and gathers it to rank 0 on that context's stream.
    # (measured with tools/inflight.py --shard, profiles/r01/s12_inflight_shards.txt:
    # one rank's share of an 8-GPU frame takes 1.60 ms alone, 0.34 ms per frame
    # with 6 in flight; of a 2-GPU frame 0.83 ms with 2, 0.76 ms with 4).
    # What matters is the rank's pixel count: 4 in flight while a rank holds at
    # least a quarter of a 1080p frame, 6 below that (an 8-GPU share, config 2).
    # Re-measured at N = 1 (profiles/r01/s18_inflight_headline.jsonl): 2 / 3 /
    # 4 / 6 in flight give 1.44 / 1.41 / 1.41 / 1.41 ms per frame.
    F = args.inflight if args.inflight > 0 else frames_in_flight(W, H, world)
    skybox = sc.skybox(2048, 1024)
    arr, _, _ = sc.default_texture_array()
    D = pkg.dist
    ctxs = []
    for k in range(F):
        rk = pkg.Renderer(local)
        rk.set_scene(scene)
        rk.set_background(skybox)
        rk.set_texture_array(arr)
        rk.set_culling(not args.no_cull)
        tile_k = torch.zeros((D.tile_rows(world, H, BLOCK_ROWS), W, 4), dtype=torch.uint8, device=dev)
        ctxs.append((rk, tile_k, D.FrameGather(tile_k, world, rank, H, BLOCK_ROWS),
                     torch.cuda.current_stream(dev) if k == 0 else torch.cuda.Stream(dev)))
    r, tile, gather, stream = ctxs[0]

    def render_tile():
        r.render_blocks(cam, params, W, H, BLOCK_ROWS, rank, world, out=tile, stream=stream)

    def step(f=0):
        rk, tile_k, gather_k, s_k = ctxs[f % F]
        with torch.cuda.stream(s_k):
            rk.render_blocks(cam, params, W, H, BLOCK_ROWS, rank, world, out=tile_k, stream=s_k)
            return gather_k()  # the assembled frame on rank 0 (RCCL gather for N > 1)

    def sync_all():
        for _, _, _, s_k in ctxs:
            s_k.synchronize()

    # executed steps of this rank's rows (untimed; the debug variant of the kernel)
    rows_mine = D.rows_of(rank, world, H, BLOCK_ROWS)
    _, _, steps_full = r.render_debug(cam, params, W, H)
    torch.cuda.synchronize(dev)
    sigma_steps_frame = int(steps_full.sum().item())
    sigma_steps_mine = int(steps_full[rows_mine].sum().item())
    # candidate critical bands: the 16-row bands of workgroup tiles holding the
    # frame's longest rays (the slowest of them is timed below)
    band_max = steps_full.max(dim=1).values[: H // 16 * 16].view(-1, 16).max(dim=1).values
    band_rows = [int(b) * 16 for b in band_max.argsort(descending=True)[:CRITICAL_CANDIDATES].tolist()] or [0]
    del steps_full, band_max

    for f in range(max(args.warmup, F)):  # every context learns its launch order
        step(f)
    sync_all()

    # kernel-only timing with HIP events on the render stream (separate loop
    # so the gather does not sit between the events); the library records
    # per-kernel events (integrate / shade / resume) for the same frames
    r.set_timing(args.steps)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for _ in range(args.steps):
        render_tile()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    kernel_ms = ev0.elapsed_time(ev1) / args.steps
    ktimes = r.kernel_times(args.steps)
    r.set_timing(0)
    integrate_ms, shade_ms, resume_ms = (float(x) for x in ktimes.mean(axis=0))

    if distributed:
        dist.barrier()
    sync_all()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for f in range(args.steps):
        step(f)
    sync_all()
    torch.cuda.synchronize(dev)
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        k = torch.tensor([kernel_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(k, op=dist.ReduceOp.MAX)
        kernel_ms_max = float(k.item())
    else:
        kernel_ms_max = kernel_ms

    ms_per_step = elapsed * 1e3 / args.steps
    mpix_s = W * H * args.steps / elapsed / 1e6

    # Critical path (untimed, after the timed regions): that band rendered on
    # its own (~120 workgroups, under one wave per SIMD), on a second context
    # so the frame's launch-order state stays untouched. Its time is the
    # slowest waves' latency without contention.
    critical = None
    if rank == 0 and world == 1 and args.critical_path == "on":
        rb = pkg.Renderer(local)
        rb.set_scene(scene)
        rb.set_background(skybox)
        rb.set_texture_array(arr)
        rb.set_culling(not args.no_cull)

        def band_time(band, reps):
            for _ in range(2):
                rb.render(cam, params, W, H, *band, stream=stream)
            times = []
            for _ in range(reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                rb.render(cam, params, W, H, *band, stream=stream)
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
                    "frac_of_frame": round(band_ms / kernel_ms, 3)}

    if rank == 0:
        # roofline of the dominant kernel (sr_integrate_kernel: ray generation,
        # the step loop and every intersection test), on rank 0's launch
        flop = sigma_steps_mine * FLOP_PER_STEP + len(rows_mine) * W * FLOP_PER_PIXEL_INTEGRATE
        achieved_tflops = flop / (integrate_ms * 1e-3) / 1e12
        frame_flop = sigma_steps_mine * FLOP_PER_STEP + len(rows_mine) * W * FLOP_PER_PIXEL
        hbm_bytes = len(rows_mine) * W * 4  # compulsory RGBA8 store; textures stay cache resident
        traffic = None
        tj = Path(args.traffic_json)
        if tj.exists():
            try:
                rec = json.loads(tj.read_text())
                if rec.get("width") == W and rec.get("height") == H and rec.get("max_steps") == N and world == 1:
                    traffic = rec.get("hbm_bytes_per_launch")
            except Exception:  # noqa: BLE001
                traffic = None
        pmc = None
        pj = Path(args.pmc_json)
        if pj.exists():
            try:
                rec = json.loads(pj.read_text())
                if rec.get("width") == W and rec.get("height") == H and rec.get("max_steps") == N and world == 1:
                    pmc = {k: rec[k] for k in ("valu_busy", "salu_per_valu", "source") if k in rec}
            except Exception:  # noqa: BLE001
                pmc = None
        roofline = {
            "bound": "valu",
            "kernel": "sr_integrate_kernel",
            "achieved": round(achieved_tflops, 3),
            "peak": PEAK_FP32_TFLOPS,
            "unit": "TFLOP/s",
            "frac": round(achieved_tflops / PEAK_FP32_TFLOPS, 4),
            "traffic": traffic,
            "frac_unpacked_peak": round(achieved_tflops / PEAK_FP32_UNPACKED_TFLOPS, 4),
            "kernel_ms": round(integrate_ms, 4),
            "flop_per_launch": flop,
            "steps_per_launch": sigma_steps_mine,
            "mean_steps_per_pixel": round(sigma_steps_frame / (W * H), 2),
            "pipeline_ms": {"integrate": round(integrate_ms, 4), "shade": round(shade_ms, 4),
                            "resume": round(resume_ms, 4), "frame_events": round(kernel_ms, 4)},
            "frame": {
                "achieved": round(frame_flop / (kernel_ms * 1e-3) / 1e12, 3),
                "unit": "TFLOP/s",
                "flop_per_frame": frame_flop,
                "frac": round(frame_flop / (kernel_ms * 1e-3) / 1e12 / PEAK_FP32_TFLOPS, 4),
            },
            # algorithmic = the reference loop's work; culling
            # executes a fraction of it, so frac can approach or pass 1. The
            # frame is bounded by the latency of its longest rays' waves:
            # critical_path = their band alone; pmc = executed VALU issue
            # (profiles/pmc_latest.json, same config)
            "critical_path": critical,
            "pmc": pmc,
            "hbm": {
                "achieved": round(hbm_bytes / (kernel_ms * 1e-3) / 1e9, 3),
                "peak": PEAK_HBM_GBS,
                "unit": "GB/s",
                "frac": round(hbm_bytes / (kernel_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 6),
                "algorithmic_bytes": hbm_bytes,
            },
        }
        cpu = None
        if args.cpu_baseline == "auto" and world == 1:
            cpu = cpu_baseline(cam, W, H, N, args.cpu_sample_rows)
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
            "data": "synthetic (default scene of src/main.cpp:222-268, procedural stand-in textures)",
            "config": {
                "workload": (f"{W}x{H} {args.mode}-mode frame"
                             + (f" (curved_percentage {args.curved_percentage})" if args.mode.startswith("half") else "")
                             + f", {N} geodesic steps, default scene, percent_black "
                             + ("off" if args.percent_black < 0 else str(args.percent_black))),
                "width": W,
                "height": H,
                "max_steps": N,
                "tiling": f"block-cyclic {BLOCK_ROWS}-row bands over {world} rank(s), RCCL gather to rank 0",
                "frames_in_flight": F,
                "frame_latency_ms": round(kernel_ms_max, 4),
                "culling": not args.no_cull,
                "kernel_ms_max_over_ranks": round(kernel_ms_max, 4),
            },
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()
    for rk, _, _, _ in ctxs:
        rk.close()


def cpu_baseline(cam, W, H, N, sample_rows):
    """The reference's press-R CPU geodesic (src/main.cpp:73-124) swept over
    a bounded sample of the frame's pixels, all host cores (oracle port)."""
    import srpkg

    oracle = srpkg.load_oracle()
    threads = min(16, os.cpu_count() or 1)
    if sample_rows <= 0:
        # calibrate: time 8 rows, size the sample to ~10 s of work
        t = time.perf_counter()
        oracle.pressr_sweep(cam, W, H, N, 2, H // 2 - 4, H // 2 + 4, threads)
        dt = max(time.perf_counter() - t, 1e-3)
        sample_rows = int(min(H, max(8, 8 * 10.0 / dt)))
    # evenly spread bands: rows [y0, y0 + n) around the frame centre
    y0 = max(0, H // 2 - sample_rows // 2)
    y1 = min(H, y0 + sample_rows)
    t = time.perf_counter()
    pts = oracle.pressr_sweep(cam, W, H, N, 2, y0, y1, threads)
    dt = time.perf_counter() - t
    px = (y1 - y0) * W
    return {
        "value": round(px / dt / 1e6, 4),
        "unit": "Mpixels/s",
        "cores": threads,
        "kind": "port",
        "sample": f"press-R loop (src/main.cpp:73-124) over rows [{y0},{y1}) x {W} px of the {W}x{H} frame, "
                  f"{N} steps, {pts} points, {dt:.2f} s, -O2",
    }


if __name__ == "__main__":
    main()
