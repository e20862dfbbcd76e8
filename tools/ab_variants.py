#!/usr/bin/env python3
"""A/B timing of libsr variants in ONE process, interleaved rounds
(cdna_hip_programming.md §5.4 rule 24). Each variant .so is loaded privately
(RTLD_LOCAL) with its own context; the headline frame is rendered and the
kernel timed with HIP events on the torch stream. Also checks every variant's
frame is byte-identical to the first variant's.

  python tools/ab_variants.py lib/variants/libsr_a.so lib/variants/libsr_b.so [--rounds 5 --reps 3]
"""
import argparse
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--max-steps", type=int, default=2000)
    ap.add_argument("--camera", default="default")
    ap.add_argument("--scene", choices=["tex", "untex", "bh", "stress", "general"], default="tex",
                    help="stress: scenes.scene_stress (21 objects); general: an 8-object random scene (every object "
                         "in a budget slot, the general 8-slot / 3-cylinder instantiation)")
    ap.add_argument("--throughput", action="store_true",
                    help="bench.py's pipeline instead of single frames: --frames frames in launches of --batch "
                         "(sr_render_blocks_batch), --inflight launches in flight on their own contexts and streams")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--inflight", type=int, default=3)
    ap.add_argument("--frames", type=int, default=48)
    args = ap.parse_args()
    import torch

    import srpkg

    pkg = srpkg.load_package()
    abi, sc = pkg.abi, pkg.scenes
    if args.scene == "bh":
        scene = sc.scene_black_hole_only()
    elif args.scene == "stress":
        scene = sc.scene_stress()
    elif args.scene == "general":
        scene = sc.scene_random(7, n_objects=8, translucent=False, planes=False)
    else:
        scene = sc.scene_default(textured=args.scene == "tex")
    cam = abi.default_camera() if args.camera == "default" else sc.random_camera(int(args.camera))
    params = abi.default_params(max_steps=args.max_steps, percent_black=-1.0)
    bg = np.ascontiguousarray(sc.skybox(2048, 1024))
    arr, _, _ = sc.default_texture_array()
    W, H = args.width, args.height
    stream = torch.cuda.current_stream()
    sp = C.c_void_p(stream.cuda_stream)
    variants = []
    for path in args.libs:
        lib = C.CDLL(str(Path(path).resolve()), mode=C.RTLD_LOCAL)
        for name, (res, argt) in {**abi.SIGNATURES, **abi.EXTRA_SIGNATURES}.items():
            if not hasattr(lib, name):
                continue  # older variants predate some exports
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, argt
        ctx = C.c_void_p()
        abi.check(lib.sr_create(C.byref(ctx), 0), "sr_create")
        abi.check(lib.sr_set_scene(ctx, C.byref(scene)), "scene")
        abi.check(lib.sr_set_background(ctx, bg.ctypes.data, bg.shape[1], bg.shape[0], 3), "bg")
        abi.check(lib.sr_set_texture_array(ctx, arr.ctypes.data, arr.shape[2], arr.shape[1], arr.shape[0], arr.shape[3]), "arr")
        out = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
        variants.append((Path(path).name, lib, ctx, out))

    def launch(v):
        _, lib, ctx, out = v
        abi.check(lib.sr_render(ctx, C.byref(cam), C.byref(params), W, H, 0, H, C.c_void_p(out.data_ptr()), W * 4, sp), "render")

    for v in variants:
        launch(v)
    torch.cuda.synchronize()
    nsteps = {}
    for name, lib, ctx, out in variants:
        st = torch.empty((H, W), dtype=torch.int32, device="cuda")
        abi.check(lib.sr_render_debug(ctx, C.byref(cam), C.byref(params), W, H, 0, H, None, None,
                                      C.c_void_p(st.data_ptr()), sp), "debug")
        torch.cuda.synchronize()
        nsteps[name] = int(st.sum().item())
    if args.throughput:
        # per variant: inflight contexts, each with its stream and a B-frame output
        tp = []
        for name, lib, ctx0, _ in variants:
            ctxs = []
            for k in range(args.inflight):
                c = ctx0
                if k:
                    c = C.c_void_p()
                    abi.check(lib.sr_create(C.byref(c), 0), "sr_create")
                    abi.check(lib.sr_set_scene(c, C.byref(scene)), "scene")
                    abi.check(lib.sr_set_background(c, bg.ctypes.data, bg.shape[1], bg.shape[0], 3), "bg")
                    abi.check(lib.sr_set_texture_array(c, arr.ctypes.data, arr.shape[2], arr.shape[1], arr.shape[0],
                                                       arr.shape[3]), "arr")
                st = torch.cuda.Stream()
                o = torch.empty((args.batch, H, W, 4), dtype=torch.uint8, device="cuda")
                ctxs.append((c, st, o))
            tp.append((name, lib, ctxs))
        cams = (abi.Camera * args.batch)(*([cam] * args.batch))

        def run_tp(v):
            _, lib, ctxs = v
            for j in range(args.frames // args.batch):
                c, st, o = ctxs[j % len(ctxs)]
                abi.check(lib.sr_render_blocks_batch(c, cams, args.batch, C.byref(params), W, H, 8, 0, 1,
                                                     C.c_void_p(o.data_ptr()), W * 4, o[0].numel(),
                                                     C.c_void_p(st.cuda_stream)), "batch")
            torch.cuda.synchronize()

        for v in tp:
            run_tp(v)  # learn the launch orders
        ttimes = {v[0]: [] for v in tp}
        import time
        for _ in range(args.rounds):
            for v in tp:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                run_tp(v)
                ttimes[v[0]].append((time.perf_counter() - t0) * 1e3 / args.frames)
        tref = tp[0][2][0][2].cpu().numpy()
        res = {k: {"median_ms_per_frame": float(np.median(t)), "min_ms_per_frame": float(np.min(t)),
                   "mpix_s": W * H / (np.median(t) * 1e-3) / 1e6,
                   "identical": bool(np.array_equal(dict((v[0], v) for v in tp)[k][2][0][2].cpu().numpy(), tref))}
               for k, t in ttimes.items()}
        print(json.dumps({"throughput": res, "batch": args.batch, "inflight": args.inflight, "frames": args.frames},
                         indent=1))
        return
    ref = variants[0][3].cpu().numpy()
    same = {v[0]: bool(np.array_equal(v[3].cpu().numpy(), ref)) for v in variants}
    times = {v[0]: [] for v in variants}
    for _ in range(args.rounds):
        for v in variants:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.reps):
                launch(v)
            e1.record(stream)
            torch.cuda.synchronize()
            times[v[0]].append(e0.elapsed_time(e1) / args.reps)
    res = {k: {"median_ms": float(np.median(t)), "min_ms": float(np.min(t)),
               "mpix_s": W * H / (np.median(t) * 1e-3) / 1e6, "identical": same[k], "steps": nsteps[k],
               "ps_per_step": np.median(t) * 1e9 / nsteps[k]} for k, t in times.items()}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
