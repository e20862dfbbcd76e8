#!/usr/bin/env python3
"""Renders the headline frame N times through the C-ABI (for rocprofv3 runs).
  python tools/prof_frame.py [--frames 3] [--lib path] [--width 1920 --height 1080 --max-steps 2000]"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--max-steps", type=int, default=2000)
    ap.add_argument("--no-cull", action="store_true")
    ap.add_argument("--scene", default="tex", choices=["tex", "untex", "bh"])
    args = ap.parse_args()
    import torch

    import srpkg

    pkg = srpkg.load_package()
    abi, sc = pkg.abi, pkg.scenes
    r = pkg.Renderer(0)
    if args.scene == "bh":
        r.set_scene(sc.scene_black_hole_only())
    else:
        r.set_scene(sc.scene_default(textured=args.scene == "tex"))
    r.set_background(sc.skybox(2048, 1024))
    arr, _, _ = sc.default_texture_array()
    r.set_texture_array(arr)
    r.set_culling(not args.no_cull)
    cam = abi.default_camera()
    params = abi.default_params(max_steps=args.max_steps, percent_black=-1.0)
    out = None
    for _ in range(args.frames):
        out = r.render(cam, params, args.width, args.height, out=out)
    torch.cuda.synchronize()
    r.close()


if __name__ == "__main__":
    main()
