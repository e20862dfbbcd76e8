#!/usr/bin/env python3
"""Latency bound of regrouping rays between waves, measured
with an SR_LANE_MASK build (tools/build_variant.sh lanemask -DSR_LANE_MASK):
masked pixels run no ray, so a band rendered with only some of its rays shows
how long those rays' waves take without the others.

For the headline frame's slowest 16-row bands and the whole frame, times the
render (median of --reps, HIP events) with these masks:
  all       every pixel (the production frame)
  ge<S>     only rays of at least S steps (the long rays in their own waves)
  lt<S>     only rays below S steps
  one       only the longest ray of each 8x8 wave tile
  onering   only the longest ray of each wave tile whose longest ray has >= 1000 steps

  python tools/lane_mask.py LIB [--bands 4] [--reps 5]
"""
import argparse
import ctypes as C
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--bands", type=int, default=4)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default="")
    ap.add_argument("--rows", type=int, nargs=2, action="append", help="extra bands [a, b) to time")
    ap.add_argument("--split", action="store_true",
                    help="also quadK (4x4 quads of each 8x8 wave tile) and subK (2x2 cells): the latency of a band "
                         "rendered as 16- or 4-lane waves is the max over K")
    ap.add_argument("--shard", type=int, nargs=2, action="append",
                    help="RANK WORLD: time that rank's block-cyclic share (8-row blocks, sr_render_blocks)")
    args = ap.parse_args()
    os.environ["SR_LIB"] = str(Path(args.lib).resolve())
    import torch

    import srpkg

    pkg = srpkg.load_package()
    abi, sc = pkg.abi, pkg.scenes
    lib = abi.load()
    fn = lib.sr_debug_set_lane_mask
    fn.restype, fn.argtypes = C.c_int, [C.c_void_p]
    W, H, N = 1920, 1080, 2000
    r = pkg.Renderer(0)
    r.set_scene(sc.scene_default(textured=True))
    r.set_background(sc.skybox(2048, 1024))
    arr, _, _ = sc.default_texture_array()
    r.set_texture_array(arr)
    cam = abi.default_camera()
    params = abi.default_params(max_steps=N, percent_black=-1.0)
    _, _, steps = r.render_debug(cam, params, W, H)
    torch.cuda.synchronize()
    steps = steps.cpu().numpy().astype(np.int64)

    # longest ray of each 8x8 wave tile (frame-aligned 16x16 workgroup tiles)
    Hp, Wp = (H + 7) // 8 * 8, (W + 7) // 8 * 8
    sp = np.full((Hp, Wp), -1, np.int64)
    sp[:H, :W] = steps
    tiles = sp.reshape(Hp // 8, 8, Wp // 8, 8).transpose(0, 2, 1, 3).reshape(Hp // 8, Wp // 8, 64)
    arg = tiles.argmax(-1)
    tmax = tiles.max(-1)
    one = np.zeros((Hp // 8, Wp // 8, 64), bool)
    np.put_along_axis(one, arg[..., None], True, axis=-1)
    one = one.reshape(Hp // 8, Wp // 8, 8, 8).transpose(0, 2, 1, 3).reshape(Hp, Wp)[:H, :W]
    ring = np.repeat(np.repeat(tmax >= 1000, 8, 0), 8, 1)[:H, :W]
    masks = {
        "all": np.ones((H, W), bool),
        "ge1000": steps >= 1000,
        "ge1500": steps >= 1500,
        "lt1000": steps < 1000,
        "ge500": steps >= 500,
        "lt500": steps < 500,
        "one": one,
        "onering": one & ring,
    }
    if args.split:
        yy, xx = np.mgrid[0:H, 0:W]
        for k in range(4):
            masks[f"quad{k}"] = ((xx % 8) // 4 + 2 * ((yy % 8) // 4)) == k
        for k in range(16):
            masks[f"sub{k}"] = ((xx % 8) // 2 + 4 * ((yy % 8) // 2)) == k
    band_max = steps.max(axis=1)[: H // 16 * 16].reshape(-1, 16).max(axis=1)
    bands = [(int(b) * 16, int(b) * 16 + 16) for b in np.argsort(-band_max)[: args.bands]]
    bands += [tuple(b) for b in (args.rows or [])] + [(0, H)]
    bands += [("shard", rk, wd) for rk, wd in (args.shard or [])]
    D = pkg.dist

    def render(band, out):
        if band[0] == "shard":
            _, rk, wd = band
            if out is None:
                out = torch.zeros((D.tile_rows(wd, H, 8), W, 4), dtype=torch.uint8, device="cuda")
            r.render_blocks(cam, params, W, H, 8, rk, wd, out=out)
            return out
        return r.render(cam, params, W, H, band[0], band[1], out=out)

    dev_mask = {k: torch.from_numpy(v.astype(np.uint8)).cuda() for k, v in masks.items()}
    res = {"kept": {k: int(v.sum()) for k, v in masks.items()}, "bands": {}}
    for band in bands:
        row = {}
        for k, m in dev_mask.items():
            torch.cuda.synchronize()
            abi.check(fn(m.data_ptr()), "set mask")
            out = None
            for _ in range(2):
                out = render(band, out)
            ts = []
            for _ in range(args.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                out = render(band, out)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            ts.sort()
            row[k] = round(ts[len(ts) // 2], 4)
        name = f"shard {band[1]}/{band[2]}" if band[0] == "shard" else f"rows {band[0]}-{band[1]}"
        if args.split:
            row["quad_max"] = max(row[f"quad{k}"] for k in range(4))
            row["sub_max"] = max(row[f"sub{k}"] for k in range(16))
            for k in list(row):
                if k[:3] in ("qua", "sub") and not k.endswith("max"):
                    del row[k]
        res["bands"][name] = row
        print(f"{name}: " + "  ".join(f"{k} {v:.3f}" for k, v in row.items()), flush=True)
    abi.check(fn(None), "clear mask")
    print(json.dumps(res))
    if args.out:
        Path(args.out).write_text(json.dumps(res) + "\n")


if __name__ == "__main__":
    main()
