#!/usr/bin/env python3
"""Times the render of a row band of the headline frame (1920x1080/2000,
default scene) with one libsr variant: with a band of one 16-row tile row
the grid is ~0.5 waves per SIMD, so the launch time is the slowest wave's
time without contention.
  python tools/time_rows.py LIB [--rows 704 720] [--reps 5]"""
import argparse
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--rows", type=int, nargs=2, action="append")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--scene", default="tex")
    args = ap.parse_args()
    os.environ["SR_LIB"] = str(Path(args.lib).resolve())
    import torch

    import srpkg

    pkg = srpkg.load_package()
    abi, sc = pkg.abi, pkg.scenes
    r = pkg.Renderer(0)
    r.set_scene(sc.scene_black_hole_only() if args.scene == "bh" else sc.scene_default(textured=args.scene == "tex"))
    r.set_background(sc.skybox(2048, 1024))
    arr, _, _ = sc.default_texture_array()
    r.set_texture_array(arr)
    cam = abi.default_camera()
    params = abi.default_params(max_steps=2000, percent_black=-1.0)
    for a, b in args.rows or [[704, 720]]:
        out = None
        for _ in range(2):
            out = r.render(cam, params, 1920, 1080, a, b, out=out)
        ts = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            out = r.render(cam, params, 1920, 1080, a, b, out=out)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        print(f"{Path(args.lib).name} rows [{a},{b}) scene {args.scene}: median {ts[len(ts) // 2]:.4f} ms min {ts[0]:.4f} ms")
    r.close()


if __name__ == "__main__":
    main()
