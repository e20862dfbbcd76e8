#!/usr/bin/env python3
"""Frames in flight on one GPU: F contexts, each on its own stream, render K
frames of the headline frame round-robin; prints frames/s and Mpix/s per F.
The frame's time is bounded by its longest rays' waves; with
several frames in flight the next frames' waves fill the SIMDs those leave idle.
  python tools/inflight.py [--frames 24] [--inflight 1 2 3 4]"""
import argparse
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=24)
    ap.add_argument("--inflight", type=int, nargs="+", default=[1, 2, 3, 4])
    ap.add_argument("--lib", default="", help="libsr variant to load (default: the package's)")
    ap.add_argument("--shard", type=int, nargs=2, default=[0, 1], metavar=("RANK", "N"),
                    help="render only this rank's block-cyclic share of an N-GPU frame (8-row blocks)")
    args = ap.parse_args()
    if args.lib:
        os.environ["SR_LIB"] = str(Path(args.lib).resolve())
    # as bench.py: every in-flight frame's stream gets a hardware queue
    if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 8:
        os.environ["GPU_MAX_HW_QUEUES"] = "8"
    import torch

    import srpkg

    pkg = srpkg.load_package()
    abi, sc = pkg.abi, pkg.scenes
    scene = sc.scene_default(textured=True)
    bg = sc.skybox(2048, 1024)
    arr, _, _ = sc.default_texture_array()
    cam = abi.default_camera()
    params = abi.default_params(max_steps=2000, percent_black=-1.0)
    W, H = 1920, 1080
    rank, world = args.shard
    D = pkg.dist
    rs, ss, outs = [], [], []
    for k in range(max(args.inflight)):
        r = pkg.Renderer(0)
        r.set_scene(scene)
        r.set_background(bg)
        r.set_texture_array(arr)
        rs.append(r)
        ss.append(torch.cuda.Stream())
        outs.append(torch.empty((D.tile_rows(world, H, 8), W, 4), dtype=torch.uint8, device="cuda"))
    for k in range(len(rs)):  # learn each context's launch order
        for _ in range(2):
            rs[k].render_blocks(cam, params, W, H, 8, rank, world, out=outs[k], stream=ss[k])
    torch.cuda.synchronize()
    for F in args.inflight:
        t0 = time.perf_counter()
        for f in range(args.frames):
            k = f % F
            rs[k].render_blocks(cam, params, W, H, 8, rank, world, out=outs[k], stream=ss[k])
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"shard {rank}/{world}, in flight {F}: {dt * 1e3 / args.frames:.4f} ms/frame "
              f"({W * H * args.frames / dt / 1e6:.1f} whole-frame Mpix/s if every rank kept this pace)", flush=True)
    for r in rs:
        r.close()


if __name__ == "__main__":
    main()
