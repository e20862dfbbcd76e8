#!/usr/bin/env python3
"""How well block lists priced from a cheap cost map balance the ranks of a
moving camera (bench.py --camera flyby --reprice; dist.balanced_blocks).

For the bench's N-rank flyby (its cameras, launch shape and re-price points)
this prices lists at every re-price camera from several cost maps of that
camera - the full-resolution map (the truth), a half- and a quarter-resolution
one (the coarse blocks' costs repeated over the full blocks they span, or
interpolated) - and scores each, and the frame-0 lists and block-cyclic rows,
by max/mean of the ranks' loads under the full-resolution map of the camera
the lists are used for (the next re-price camera, and the last one). Also the
GPU time of each map.
  python tools/reprice_eval.py [--world 8 --steps 20]"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    args = ap.parse_args()
    import torch

    import bench
    import srpkg

    pkg = srpkg.load_package()
    abi, sc, D = pkg.abi, pkg.scenes, pkg.dist
    W, H, N = bench.WORKLOADS["headline"]
    world = args.world
    B = bench.frames_per_launch(W, H, world, args.steps)
    F = bench.launches_in_flight(B, W, H, world)
    warm = max(args.warmup, F * B)
    n_frames = warm + args.steps
    cams = [abi.camera_flyby((f + 0.5) / n_frames, *bench.FLYBY) for f in range(n_frames)]
    params = abi.default_params(max_steps=N, percent_black=-1.0)
    r = pkg.Renderer(0)
    r.set_scene(sc.scene_default(textured=True))
    A = pkg.assets
    r.set_background(A.skybox("2k") if A.available() else sc.skybox(2048, 1024))
    r.set_texture_array(A.texture_array()[0] if A.available() else sc.default_texture_array()[0])
    nb = D.nblocks(H, bench.BLOCK_ROWS)

    def cost_map(cam, w, h):
        torch.cuda.synchronize()
        t = time.perf_counter()
        wc = r.wave_costs(cam, params, w, h)
        torch.cuda.synchronize()
        return D.block_costs(wc.cpu()), (time.perf_counter() - t) * 1e3

    def spread(cl, k, mode):
        if mode == "repeat":
            return np.repeat(cl, k)[:nb]
        centres = (np.arange(len(cl)) + 0.5) * k  # coarse block centres in full-block units
        return np.interp(np.arange(nb) + 0.5, centres, cl)

    def mom(lists, cost):
        loads = [sum(cost[b] for b in l if b >= 0) for l in lists]
        return round(max(loads) / (sum(loads) / world), 4)

    cyclic = [D.blocks_of(k, world, H, bench.BLOCK_ROWS) for k in range(world)]
    truth = {}

    def true_cost(f):
        if f not in truth:
            truth[f] = cost_map(cams[f], W, H)[0]
        return truth[f]

    frame0 = D.balanced_blocks(true_cost(0), world)
    # re-price points: every F launches (the bench's default with the flyby)
    firsts = list(range(0, n_frames, B))
    points = [f for j, f in enumerate(firsts) if j and (f // B) % F == 0]
    last = n_frames - 1
    rows = []
    for i, f in enumerate(points):
        use_until = points[i + 1] if i + 1 < len(points) else last
        targets = sorted({min(f + B * F - 1, last), use_until, last})
        est = {}
        c_full, t_full = cost_map(cams[f], W, H)
        est["full"] = (c_full, t_full)
        for name, div, k in (("half", 2, 2), ("quarter", 4, 4)):
            cl, t = cost_map(cams[f], max(8, W // div), max(8, H // div))
            est[name + "_repeat"] = (spread(cl, k, "repeat"), t)
            est[name + "_interp"] = (spread(cl, k, "interp"), t)
        row = {"reprice_frame": f, "targets": targets, "map_ms": {k: round(v[1], 3) for k, v in est.items()}}
        for tgt in targets:
            tc = true_cost(tgt)
            sc_ = {"frame0": mom(frame0, tc), "cyclic": mom(cyclic, tc)}
            for k, (c, _) in est.items():
                sc_[k] = mom(D.balanced_blocks(c, world), tc)
            row[f"at_{tgt}"] = sc_
        rows.append(row)
        print(json.dumps(row), flush=True)
    print(json.dumps({"world": world, "B": B, "F": F, "frames": n_frames, "points": points}))
    r.close()


if __name__ == "__main__":
    main()
