#!/usr/bin/env python3
"""Split-tile sweep (sr_set_split): for each setting
K:LANES:MIN_STEPS (K = 0: off) and each share of the headline frame, the
single-frame latency (one context alone) and the time per frame with F frames
in flight (F contexts on their own streams), frames byte-compared with the
unsplit render.
  python tools/split_sweep.py --split 0:16:1 64:16:1000 64:16:1000:L ... [--shard 0 1 --shard 0 8] [--inflight 4]
(a fourth field L: with the latency mode, sr_set_latency_mode)
Prints one JSON line per (setting, share)."""
import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--split", nargs="+", default=["0:16:1"])
    ap.add_argument("--shard", type=int, nargs=2, action="append", metavar=("RANK", "N"))
    ap.add_argument("--inflight", type=int, nargs="+", default=[4])
    ap.add_argument("--frames", type=int, default=24)
    ap.add_argument("--camera", choices=["static", "flyby"], default="static")
    ap.add_argument("--out", default="")
    ap.add_argument("--lib", default="", help="libsr variant to load (default: the package's)")
    ap.add_argument("--batch", type=int, nargs="+", default=[1], help="frames per launch (sr_render_blocks_batch)")
    ap.add_argument("--balance", choices=["cyclic", "cost"], default="cyclic",
                    help="rank shares: block-cyclic rows, or dist.balanced_blocks lists (sr_render_block_list)")
    args = ap.parse_args()
    if args.lib:
        os.environ["SR_LIB"] = str(Path(args.lib).resolve())
    need = max(8, max(args.inflight) + 1)  # a hardware queue per in-flight frame's stream (bench.py)
    if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < need:
        os.environ["GPU_MAX_HW_QUEUES"] = str(need)
    import numpy as np
    import torch

    import srpkg

    pkg = srpkg.load_package()
    abi, sc, D = pkg.abi, pkg.scenes, pkg.dist
    scene = sc.scene_default(textured=True)
    bg = sc.skybox(2048, 1024)
    arr, _, _ = sc.default_texture_array()
    params = abi.default_params(max_steps=2000, percent_black=-1.0)
    W, H = 1920, 1080
    nf = 64
    cams = ([abi.camera_flyby((f + 0.5) / nf, 30.0, 10.0) for f in range(nf)] if args.camera == "flyby"
            else [abi.default_camera()] * nf)
    Fmax = max(args.inflight)
    rs = []
    for _ in range(Fmax):
        r = pkg.Renderer(0)
        r.set_scene(scene)
        r.set_background(bg)
        r.set_texture_array(arr)
        rs.append(r)
    ss = [torch.cuda.Stream() for _ in range(Fmax)]
    lines = []
    refs = {}
    lists_of = {}
    if args.balance == "cost":
        costs = D.block_costs(rs[0].wave_costs(cams[0], params, W, H))
        for _, world in (args.shard or [[0, 1]]):
            lists_of[world] = D.balanced_blocks(costs, world)
    for (rank, world), Bt, spec in [(sh, b, sp) for sh in (args.shard or [[0, 1]]) for b in args.batch
                                    for sp in args.split]:
        # zeroed: padding rows (a share shorter than the tile, -1 list entries) are never written
        outs = [torch.zeros((Bt, D.tile_rows(world, H, 8), W, 4), dtype=torch.uint8, device="cuda")
                for _ in range(Fmax)]
        lst = lists_of[world][rank] if world in lists_of else None

        def go(k, f, n=None):  # launch f: frames f*Bt .. f*Bt + n - 1 (n <= Bt) on context k
            n = Bt if n is None else n
            if lst is not None:
                cs = [cams[(f * Bt + j) % nf] for j in range(n)]
                rs[k].render_block_list(cs, params, W, H, 8, lst, out=outs[k][:n], stream=ss[k])
            elif n == 1:
                rs[k].render_blocks(cams[f * Bt % nf], params, W, H, 8, rank, world, out=outs[k][0], stream=ss[k])
            else:
                cs = [cams[(f * Bt + j) % nf] for j in range(n)]
                rs[k].render_blocks_batch(cs, params, W, H, 8, rank, world, out=outs[k][:n], stream=ss[k])

        fields = spec.split(":")
        K, lanes, mn = (int(x) for x in fields[:3])
        latency_mode = len(fields) > 3 and fields[3] == "L"  # K:LANES:MIN:L = with sr_set_latency_mode
        for r in rs:
            r.set_split(K, lanes, mn)
            r.set_latency_mode(latency_mode)
        for k in range(Fmax):  # learn each context's launch order (twice: split codes need costs)
            for f in range(3):
                go(k, f)
        torch.cuda.synchronize()
        frame = outs[0][0].cpu().numpy()
        refs.setdefault((rank, world), frame)
        same = bool(np.array_equal(refs[(rank, world)], frame)) if args.camera == "static" else None
        # latency: frames alone on context 0
        lat = []
        for f in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(ss[0])
            go(0, f)
            e1.record(ss[0])
            torch.cuda.synchronize()
            lat.append(e0.elapsed_time(e1))
        rec = {"lib": Path(args.lib).name if args.lib else "libsr.so", "batch": Bt, "split": spec,
               "balance": args.balance,
               "shard": f"{rank}/{world}", "camera": args.camera, "latency_ms": round(sorted(lat)[2], 4),
               "identical": same}
        for F in args.inflight:
            for r in rs[:F]:
                r.set_timing(args.frames)
            t0 = time.perf_counter()
            # exactly args.frames frames, as bench.py times K steps: the last launch takes the remainder
            launches = -(-args.frames // Bt)
            for f in range(launches):
                go(f % F, f, min(Bt, args.frames - f * Bt))
            torch.cuda.synchronize()
            rec[f"ms_per_frame_F{F}"] = round((time.perf_counter() - t0) * 1e3 / args.frames, 4)
            kt = np.concatenate([r.kernel_times(launches) for r in rs[:F]], axis=0)
            for r in rs[:F]:
                r.set_timing(0)
            # mean integrate / shade / resume+order durations of this run's frames (overlapping F-fold)
            rec[f"kernel_ms_F{F}"] = [round(float(x), 4) for x in kt.mean(axis=0)]
        print(json.dumps(rec), flush=True)
        lines.append(rec)
    for r in rs:
        r.close()
    if args.out:
        Path(args.out).write_text("".join(json.dumps(x) + "\n" for x in lines))


if __name__ == "__main__":
    main()
