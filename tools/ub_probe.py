"""Post-mortem of single pixels of the press-R overlay frame (c2t: 640x360,
1000 steps, default scene + tests' 1000-point test ray) through the library in
SR_LIB (default libsr.so): renders the debug frame, copies the integrate ->
shade hand-off (sr_debug_pixel_state) and prints each chosen pixel's record
(status, logged hits, steps, direction), its hit records and its ray origin.
The kernel itself is not instrumented, so the library's register allocation
is the one under suspicion.

    SR_LIB=.../libsr_w7.so python tools/ub_probe.py OUT.json [x,y ...]
"""
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import srpkg  # noqa: E402

PS_HITS = 4
PS_PLANES = 4 + 8 * PS_HITS
PS_RO = 5


def pixel_id(px: int, k: int, width: int) -> int:
    """geodesic.hip pixel_of / sr_lds_pid for a whole-tile, single-frame launch."""
    gx = (width + 15) >> 4
    block = (k >> 4) * gx + (px >> 4)
    wave = ((k >> 3) & 1) * 2 + ((px >> 3) & 1)
    lane = (k & 7) * 8 + (px & 7)
    return block * 256 + wave * 64 + lane


def main():
    out = sys.argv[1]
    pts = [tuple(int(v) for v in a.split(",")) for a in sys.argv[2:]] or [(300, 0), (320, 180), (284, 10), (100, 100)]
    pkg = srpkg.load_package()
    import torch

    abi, sc, A = pkg.abi, pkg.scenes, pkg.assets
    W, H, N = 640, 360, 1000
    r = pkg.Renderer(0)
    r.set_scene(sc.scene_default(textured=True))
    r.set_background(A.skybox("2k"))
    arr, _, _ = A.texture_array()
    r.set_texture_array(arr)
    r.set_test_ray(sc.test_ray_overlay())
    params = abi.default_params(max_steps=N, percent_black=-1.0)
    f, b, s = r.render_debug(abi.default_camera(), params, W, H)
    torch.cuda.synchronize()
    b, s = b.cpu().numpy(), s.cpu().numpy()
    if not hasattr(r.lib, "sr_debug_pixel_state"):  # an older library (bisection): the frame only
        np.save(out.replace(".json", "_frame.npy"), np.concatenate([b.astype(np.int32), s[..., None]], -1))
        json.dump({"lib": os.environ.get("SR_LIB", "libsr.so")}, open(out, "w"))
        return
    ps = r.pixel_state()
    n = ps.size // abi.PS_FIELDS
    res = {"lib": os.environ.get("SR_LIB", "libsr.so"), "n_ids": int(n), "pixels": []}
    np.save(out.replace(".json", "_frame.npy"), np.concatenate([b.astype(np.int32), s[..., None]], -1))
    for (x, y) in pts:
        i = pixel_id(x, y, W)
        rec = ps[4 * i:4 * i + 4]
        w = int(rec[:1].view(np.int32)[0])
        st, nh, steps = w & 7, (w >> 3) & 31, (w >> 8) & 0xFFFFFF
        hits = []
        for j in range(min(nh, PS_HITS)):
            h = ps[4 * n + (j * n + i) * 8:4 * n + (j * n + i) * 8 + 8]
            kw = int(h[3:4].view(np.int32)[0])
            hits.append({"p": [float(v) for v in h[:3]], "key": (kw & 255) - 24, "steps": kw >> 8,
                         "dir": [float(v) for v in h[4:7]]})
        ro = [float(ps[(PS_PLANES + PS_RO + k) * n + i]) for k in range(3)]
        res["pixels"].append({"x": x, "y": y, "id": i, "rgba": b[y, x].tolist(), "steps_map": int(s[y, x]),
                              "status": st, "nhits": nh, "steps": steps,
                              "rd": [float(v) for v in rec[1:4]], "hits": hits, "ro": ro})
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res)[:3000])


if __name__ == "__main__":
    main()
