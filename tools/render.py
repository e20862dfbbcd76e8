#!/usr/bin/env python3
"""Render frames of the app's default scene on the GPU and write them as PNG
(sr_write_png): the offline counterpart of the reference's window present
(src/main.cpp:318-319, 432). A flyby renders N frames along the H-key
hyperbolic trajectory (src/main.cpp:404-410) in batched launches.

  python tools/render.py --out frame.png [--width 1920 --height 1080 --max-steps 2000]
  python tools/render.py --flyby 8 --out flyby_%02d.png
"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

MODES = {"curved": 0, "flat": 1, "half_width": 2, "half_height": 3}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True, help="PNG path (with %%d for --flyby frames)")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--max-steps", type=int, default=2000)
    ap.add_argument("--mode", choices=sorted(MODES), default="curved")
    ap.add_argument("--percent-black", type=float, default=-1.0)
    ap.add_argument("--crosshair", action="store_true")
    ap.add_argument("--textures", choices=["assets", "standin"], default="assets")
    ap.add_argument("--flyby", type=int, default=0, help="frames along the hyperbolic flyby (0: the default camera)")
    args = ap.parse_args()
    import torch

    import srpkg

    pkg = srpkg.load_package()
    abi, sc = pkg.abi, pkg.scenes
    r = pkg.Renderer(0)
    r.set_scene(sc.scene_default(textured=True))
    if args.textures == "assets":
        r.set_background(pkg.assets.skybox("8k" if args.width * args.height > 4096 * 2160 else "2k"))
        arr, _, _ = pkg.assets.texture_array()
    else:
        r.set_background(sc.skybox(2048, 1024))
        arr, _, _ = sc.default_texture_array()
    r.set_texture_array(arr)
    params = abi.default_params(max_steps=args.max_steps, percent_black=args.percent_black,
                                raytrace_type=MODES[args.mode])
    params.crosshair = 1 if args.crosshair else 0
    W, H = args.width, args.height
    if args.flyby <= 0:
        frame = r.render(abi.default_camera(), params, W, H)
        torch.cuda.synchronize()
        abi.write_png(args.out, frame.cpu().numpy())
        print(f"wrote {args.out}")
    else:
        n = args.flyby
        cams = [abi.camera_flyby((f + 0.5) / n, 30.0, 10.0) for f in range(n)]
        for first in range(0, n, 32):  # sr_render_blocks_batch takes up to 32 frames
            out, rows = r.render_blocks_batch(cams[first:first + 32], params, W, H, H, 0, 1)
            torch.cuda.synchronize()
            for k, fr in enumerate(out.cpu().numpy()):
                path = args.out % (first + k) if "%" in args.out else f"{Path(args.out).stem}_{first + k:03d}.png"
                abi.write_png(path, fr[:rows])
                print(f"wrote {path}")
    r.close()


if __name__ == "__main__":
    main()
