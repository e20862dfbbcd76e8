#!/usr/bin/env python3
"""Black-hole budget triggers by lane orbit state (SR_STATS + SR_STATS_BH
build): lanes whose black-hole budget did not cover the event's chord,
split into inside the horizon (u > 1), at the shell (0.9 < u <= 1), near
the photon orbit (0.55 < u <= 0.9, |u'| < 0.1), falling (u' > 0) and
climbing (u' <= 0); lanes with an event of their own; events with a
black-hole trigger; active lanes at events.
  python tools/stats_bh.py lib/variants/libsr_bhstats.so"""
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
    for _ in range(2):
        lib.sr_debug_stats(buf)
        r.render(abi.default_camera(), params, 1920, 1080)
        torch.cuda.synchronize()
    assert lib.sr_debug_stats(buf) == 0
    names = ["inside", "shell", "ring", "falling", "climbing", "lanes_own_event", "bh_hard_lanes",
             "events_with_bh_trigger", "active_lanes_at_events"]
    out = {"events": int(buf[1]), **{n: int(buf[23 + k]) for k, n in enumerate(names)}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
