#!/usr/bin/env python3
"""One pixel's ray, step by step, from an SR_TRACE build (device printf of
the integrate kernel's slow-path steps, budget events, exact chords, and
fast-loop steps past u = 1e20), every other pixel masked off (SR_LANE_MASK):
  tools/build_variant.sh trace -DSR_LANE_MASK -DSR_TRACE
  python tools/trace_pixel.py schwarzschild-raytracer_amd/lib/variants/libsr_trace.so PX PY \\
      [--scene stress] [--size 640 360] [--steps 1000]
PY is the GL row (row 0 at the bottom), as in render_debug's arrays. The
oracle's side of the same ray: any printf of its step loop in a copy of
oracle/sr_oracle.c (round 6: the singularity ray)."""
import argparse
import ctypes as C
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("px", type=int)
    ap.add_argument("py", type=int)
    ap.add_argument("--scene", default="stress", choices=["default", "stress"])
    ap.add_argument("--size", type=int, nargs=2, default=[640, 360])
    ap.add_argument("--steps", type=int, default=1000)
    args = ap.parse_args()
    os.environ["SR_LIB"] = str(Path(args.lib).resolve())
    import srpkg
    import torch

    pkg = srpkg.load_package()
    abi, sc, A = pkg.abi, pkg.scenes, pkg.assets
    lib = abi.load()
    fn = lib.sr_debug_set_lane_mask
    fn.restype, fn.argtypes = C.c_int, [C.c_void_p]
    W, H = args.size
    r = pkg.Renderer(0)
    r.set_scene(sc.scene_stress() if args.scene == "stress" else sc.scene_default(textured=True))
    r.set_background(A.skybox("2k"))
    arr, _, _ = A.texture_array()
    r.set_texture_array(arr)
    params = abi.default_params(max_steps=args.steps, percent_black=-1.0)
    m = np.zeros((H, W), np.uint8)
    m[args.py, args.px] = 1
    dm = torch.from_numpy(m).cuda()
    abi.check(fn(dm.data_ptr()), "sr_debug_set_lane_mask")
    f, b, s = r.render_debug(abi.default_camera(), params, W, H)
    torch.cuda.synchronize()
    abi.check(fn(None), "sr_debug_set_lane_mask")
    print("RESULT steps", int(s[args.py, args.px]), "rgba8", b[args.py, args.px].tolist(),
          "frag", f[args.py, args.px].tolist(), flush=True)


if __name__ == "__main__":
    main()
