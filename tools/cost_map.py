#!/usr/bin/env python3
"""Per-wave cost data of the headline frame for block-cost models
(dist.wave_costs, balanced_blocks): the executed-steps map (render_debug) of
the production library and, from an SR_STATS build, every integrate wave's
max steps, budget events, exact chords and duration.
  python tools/cost_map.py lib/variants/libsr_stats.so --out gpurun_out/cost"""
import argparse
import ctypes as C
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats_lib")
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    os.environ["SR_LIB"] = str(Path(args.stats_lib).resolve())
    import numpy as np
    import torch

    import srpkg

    pkg = srpkg.load_package()
    abi, sc = pkg.abi, pkg.scenes
    lib = abi.load()
    lib.sr_debug_stats.restype = C.c_int
    lib.sr_debug_stats.argtypes = [C.POINTER(C.c_ulonglong)]
    lib.sr_debug_wave_times.restype = C.c_int
    lib.sr_debug_wave_times.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    r = pkg.Renderer(0)
    r.set_scene(sc.scene_default(textured=True))
    r.set_background(sc.skybox(2048, 1024))
    arr, _, _ = sc.default_texture_array()
    r.set_texture_array(arr)
    W, H = 1920, 1080
    cam = abi.default_camera()
    params = abi.default_params(max_steps=2000, percent_black=-1.0)
    out = Path(args.out)
    out.mkdir(parents=True, exist_ok=True)
    _, _, steps = r.render_debug(cam, params, W, H)
    torch.cuda.synchronize()
    np.save(out / "steps.npy", steps.cpu().numpy().astype(np.int32))
    buf = (C.c_ulonglong * 32)()
    for _ in range(2):
        lib.sr_debug_stats(buf)
        r.render(cam, params, W, H)
        torch.cuda.synchronize()
    nw = ((W + 15) // 16) * ((H + 15) // 16) * 4
    tb = (C.c_ulonglong * (16 * nw))()
    assert lib.sr_debug_wave_times(tb, nw) == 0
    t = np.frombuffer(tb, dtype=np.uint64).reshape(nw, 16).astype(np.int64)
    np.save(out / "waves.npy", t)
    print("saved", out, steps.shape, t.shape, flush=True)
    r.close()


if __name__ == "__main__":
    main()
