#!/usr/bin/env python3
"""Per-wave cycle breakdown of sr_integrate_kernel by step-loop section, from
an SR_PROF build (tools/build_variant.sh NAME -DSR_PROF):
  python tools/prof_waves.py lib/variants/libsr_NAME.so [--rows 704 720] [--scene tex|untex|bh|stress]
Sections: fast loop, reseeds, slow-path entry + approximate chord, budget
events, exact chord + intersect, hit classification + log."""
import argparse
import ctypes as C
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
NREC = 24  # SR_PROF_N
SECTIONS = ["fast", "reseed", "slow_entry", "budget_phase1", "exact_chord", "hit_class", "budget_phase2"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--rows", type=int, nargs=2, default=[0, 1080])
    ap.add_argument("--scene", default="tex")
    ap.add_argument("--top", type=int, default=10)
    ap.add_argument("--test-ray", action="store_true", help="the press-R overlay (scenes.test_ray_overlay)")
    args = ap.parse_args()
    os.environ["SR_LIB"] = str(Path(args.lib).resolve())
    import torch

    import srpkg

    pkg = srpkg.load_package()
    abi, sc = pkg.abi, pkg.scenes
    lib = abi.load()
    lib.sr_debug_prof.restype = C.c_int
    lib.sr_debug_prof.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    r = pkg.Renderer(0)
    r.set_scene(sc.scene_black_hole_only() if args.scene == "bh" else sc.scene_stress() if args.scene == "stress"
                else sc.scene_default(textured=args.scene == "tex"))
    if args.test_ray:
        r.set_test_ray(sc.test_ray_overlay())
    r.set_background(sc.skybox(2048, 1024))
    arr, _, _ = sc.default_texture_array()
    r.set_texture_array(arr)
    cam = abi.default_camera()
    params = abi.default_params(max_steps=2000, percent_black=-1.0)
    a, b = args.rows
    for _ in range(2):
        r.render(cam, params, 1920, 1080, a, b)
    torch.cuda.synchronize()
    nw = ((1920 + 15) // 16) * ((b - a + 15) // 16) * 4
    buf = (C.c_ulonglong * (NREC * nw))()
    assert lib.sr_debug_prof(buf, nw) == 0
    t = np.frombuffer(buf, dtype=np.uint64).reshape(nw, NREC).astype(np.int64)
    total = t[:, 7] & ((1 << 48) - 1)
    steps = t[:, 7] >> 48
    ok = total > 0
    out = {"rows": [a, b], "scene": args.scene, "waves": int(ok.sum())}
    sums = t[ok, :7].sum(0)
    out["cycles_by_section_all_waves"] = {k: int(v) for k, v in zip(SECTIONS, sums)}
    out["cycles_total_all_waves"] = int(total[ok].sum())
    out["reanchors_by_slot_all_waves"] = [int(v) for v in t[ok, 8:16].sum(0)]
    out["events_all_waves"] = int(t[ok, 16].sum())
    out["slow_entries_all_waves"] = int(t[ok, 19].sum())
    out["phase1_ballots_all_waves"] = int(t[ok, 20].sum())
    out["tail_top_all_waves"] = int(t[ok, 21].sum())
    out["budget_init_all_waves"] = int(t[ok, 22].sum())  # builds since round 4 (0 before)
    out["ray_setup_all_waves"] = int(t[ok, 23].sum())  # kernel start to integrate: launch code, pixel, ray
    out["unaccounted_cycles_all_waves"] = int(total[ok].sum() - sums.sum() - t[ok, 20].sum() - t[ok, 21].sum()
                                              - t[ok, 22].sum() - t[ok, 23].sum())
    gx = (1920 + 15) // 16
    top = np.argsort(-total)[: args.top]
    out["slowest"] = [
        {"wave": int(w), "block_xy": [int(w // 4 % gx), int(w // 4 // gx)], "steps": int(steps[w]),
         "total_cycles": int(total[w]), "cycles_per_step": round(float(total[w]) / max(1, int(steps[w])), 1),
         **{k: int(v) for k, v in zip(SECTIONS, t[w, :7])}, "reanchors_by_slot": [int(v) for v in t[w, 8:16]],
         "events": int(t[w, 16]), "events_slot0_only": int(t[w, 17]), "lane_slot0_spends": int(t[w, 18]),
         "slow_entries": int(t[w, 19]), "phase1_ballots": int(t[w, 20]), "tail_top": int(t[w, 21])}
        for w in top]
    print(json.dumps(out, indent=1))
    r.close()


if __name__ == "__main__":
    main()
