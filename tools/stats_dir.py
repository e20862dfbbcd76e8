#!/usr/bin/env python3
"""Object-slot triggers by the lane's radial direction (SR_STATS + SR_STATS_DIR
measurement build): lanes whose budget for the accretion disk (slot 3) or the
rectangle (slot 5) did not cover the event's chord, split into outward (u' <
0, u < 0.6), incoming (u' > 0) and other; and lanes with any object trigger.
  python tools/stats_dir.py lib/variants/libsr_dirstats.so"""
import ctypes as C
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    os.environ["SR_LIB"] = str(Path(sys.argv[1]).resolve())
    import torch

    import srpkg

    pkg = srpkg.load_package()
    abi, sc = pkg.abi, pkg.scenes
    lib = abi.load()
    lib.sr_debug_stats.restype = C.c_int
    lib.sr_debug_stats.argtypes = [C.POINTER(C.c_ulonglong)]
    r = pkg.Renderer(0)
    r.set_scene(sc.scene_default(textured=True))
    r.set_background(sc.skybox(2048, 1024))
    arr, _, _ = sc.default_texture_array()
    r.set_texture_array(arr)
    params = abi.default_params(max_steps=2000, percent_black=-1.0)
    buf = (C.c_ulonglong * 32)()
    lib.sr_debug_stats(buf)
    r.render(abi.default_camera(), params, 1920, 1080)
    torch.cuda.synchronize()
    lib.sr_debug_stats(buf)  # clear after the first (centre-out order) frame
    r.render(abi.default_camera(), params, 1920, 1080)
    torch.cuda.synchronize()
    assert lib.sr_debug_stats(buf) == 0
    names = ["disk_outward", "disk_incoming", "disk_other", "rect_outward", "rect_incoming", "rect_other",
             "any_object_outward", "any_object_incoming", "any_object"]
    print(json.dumps({"events": int(buf[1]), **{n: int(buf[23 + k]) for k, n in enumerate(names)}}))


if __name__ == "__main__":
    main()
