#!/usr/bin/env python3
"""One headline frame alone, kernel by kernel: the integrate, shade and
resume (+ order) durations of single-frame launches (HIP events on the
context's stream, sr_debug_kernel_times) beside the whole launch's time, to
see what follows the integrate kernel on a frame's critical path.
  python tools/frame_parts.py [--reps 15] [--lib path]"""
import argparse
import json
import os
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--lib", default="")
    args = ap.parse_args()
    if args.lib:
        os.environ["SR_LIB"] = str(Path(args.lib).resolve())
    import srpkg
    import torch

    pkg = srpkg.load_package()
    abi, sc, A = pkg.abi, pkg.scenes, pkg.assets
    W, H, N = 1920, 1080, 2000
    r = pkg.Renderer(0)
    r.set_scene(sc.scene_default(textured=True))
    r.set_background(A.skybox("2k"))
    arr, _, _ = A.texture_array()
    r.set_texture_array(arr)
    params = abi.default_params(max_steps=N, percent_black=-1.0)
    cam = abi.default_camera()
    s = torch.cuda.current_stream()
    for _ in range(3):  # the launch order learned
        r.render(cam, params, W, H)
    torch.cuda.synchronize()
    r.set_timing(args.reps)
    whole = []
    for _ in range(args.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        r.render(cam, params, W, H)
        e1.record(s)
        torch.cuda.synchronize()
        whole.append(e0.elapsed_time(e1))
    kt = r.kernel_times(args.reps)
    med = [statistics.median(kt[:, j].tolist()) for j in range(3)]
    out = {"frame_ms": round(statistics.median(whole), 4), "integrate_ms": round(med[0], 4),
           "shade_ms": round(med[1], 4), "resume_order_ms": round(med[2], 4),
           "after_integrate_ms": round(statistics.median(whole) - med[0], 4), "reps": args.reps}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
