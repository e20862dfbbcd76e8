#!/usr/bin/env python3
"""Event counters of an SR_STATS build (tools/build_variant.sh NAME -DSR_STATS):
renders the headline frame once and prints the step loop's wave-level counts.
  python tools/stats_frame.py lib/variants/libsr_NAME.so [--scene tex|untex|bh|stress]"""
import argparse
import ctypes as C
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

NAMES = {0: "wave_steps", 1: "events", 11: "coast_wave_steps", 12: "object_tests", 13: "lane_steps"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--scene", default="tex")
    ap.add_argument("--test-ray", action="store_true",
                    help="the press-R overlay (scenes.test_ray_overlay); counters 22 / 10 of a test-ray "
                         "instantiation are the test ray's re-anchors / reaches")
    ap.add_argument("--max-steps", type=int, default=2000)
    ap.add_argument("--save", default="", help="write the raw per-wave records (.npy) here")
    ap.add_argument("--rows", type=int, nargs=2, default=[0, 1080], help="render only rows [a, b) (waves alone on the chip)")
    ap.add_argument("--trig", action="store_true", help="an SR_STATS_TRIG build (counters 44..63)")
    ap.add_argument("--stephist", action="store_true", help="an SR_STATS_STEPHIST build (counters 44..55)")
    ap.add_argument("--near", action="store_true", help="an SR_STATS_NEAR build (counters 44..61)")
    ap.add_argument("--xcyl", action="store_true", help="an SR_STATS_XCYL build (counters 44..54)")
    args = ap.parse_args()
    os.environ["SR_LIB"] = str(Path(args.lib).resolve())
    import torch  # noqa: F401  (HIP runtime up before the library)

    import srpkg

    pkg = srpkg.load_package()
    abi, sc = pkg.abi, pkg.scenes
    lib = abi.load()
    lib.sr_debug_stats.restype = C.c_int
    lib.sr_debug_stats.argtypes = [C.POINTER(C.c_ulonglong)]
    r = pkg.Renderer(0)
    if args.scene == "bh":
        r.set_scene(sc.scene_black_hole_only())
    elif args.scene == "stress":
        r.set_scene(sc.scene_stress())
    else:
        r.set_scene(sc.scene_default(textured=args.scene == "tex"))
    if args.test_ray:
        r.set_test_ray(sc.test_ray_overlay())
    r.set_background(sc.skybox(2048, 1024))
    arr, _, _ = sc.default_texture_array()
    r.set_texture_array(arr)
    cam = abi.default_camera()
    params = abi.default_params(max_steps=args.max_steps, percent_black=-1.0)
    buf = (C.c_ulonglong * 32)()
    lib.sr_debug_stats(buf)  # clear
    ra, rb = args.rows
    r.render(cam, params, 1920, 1080, ra, rb)  # first frame: centre-out launch order
    lib.sr_debug_stats(buf)  # clear
    if hasattr(lib, "sr_debug_stats_hi"):
        lib.sr_debug_stats_hi.restype = C.c_int
        lib.sr_debug_stats_hi.argtypes = [C.POINTER(C.c_ulonglong)]
        lib.sr_debug_stats_hi((C.c_ulonglong * 32)())  # clear
    r.render(cam, params, 1920, 1080, ra, rb)  # steady state: cost-ordered launch
    assert lib.sr_debug_stats(buf) == 0
    def name(k):
        if k in NAMES:
            return NAMES[k]
        return f"slot{k - 2}_reached" if 2 <= k <= 10 else f"slot{k - 14}_spent"

    out = {name(k): int(buf[k]) for k in range(23)}
    # the hand-off (plain SR_STATS builds): pixels, logged hit records, pixels by status
    out["handoff"] = {"pixels": int(buf[23]), "hit_records": int(buf[24]),
                      **{n: int(buf[25 + k]) for k, n in enumerate(["done", "hit", "more", "flat", "bg", "bh"])}}
    out["event_frac"] = out["events"] / max(1, out["wave_steps"])
    out["cm_wave_steps"] = int(buf[31])  # plain SR_STATS builds: wave-steps of the cylinder-plane fast loop
    if hasattr(lib, "sr_debug_stats_hi"):  # counters 32..63 of the same frame
        hi = (C.c_ulonglong * 32)()
        lib.sr_debug_stats_hi.restype = C.c_int
        lib.sr_debug_stats_hi.argtypes = [C.POINTER(C.c_ulonglong)]
        assert lib.sr_debug_stats_hi(hi) == 0
        out["event_interval_steps"] = dict(zip(["1", "2-3", "4-7", "8-15", "16-63", "64+"], [int(hi[k]) for k in range(6)]))
        out["event_trigger_lanes"] = dict(zip(["1", "2-3", "4-7", "8-15", "16-31", "32+"], [int(hi[6 + k]) for k in range(6)]))
        out["events_bh_window_only"] = int(hi[12])
        out["event_lanes"] = {k: int(hi[13 + n]) for n, k in enumerate(
            ["empty_ball", "bh_window", "triggered", "interval1_events_32plus", "interval1_empty_ball",
             "interval1_triggered", "interval1_reseeded", "interval1_budget_below_0.05", "interval1_cm_events",
             "cm_events"])}
        out["interval1_small_budget_lanes_by_slot"] = [int(hi[23 + j]) for j in range(9)]
        if args.stephist:  # an SR_STATS_STEPHIST build: events and their lanes by step bucket
            for k in ("event_lanes", "events_bh_window_only", "interval1_small_budget_lanes_by_slot"):
                out.pop(k, None)
            names = ["<25", "25-99", "100-299", "300-699", "700-1199", "1200+"]
            out["events_by_step"] = dict(zip(names, [int(hi[12 + k]) for k in range(6)]))
            out["event_lanes_by_step"] = dict(zip(names, [int(hi[18 + k]) for k in range(6)]))
            out["recover_up"] = {"end_replayed_wave_steps": int(hi[24]), "end_exits": int(hi[25]),
                                 "neg_u_replayed_wave_steps": int(hi[26]), "neg_u_exits": int(hi[27])}
        if args.near:  # an SR_STATS_NEAR build: back-to-back (interval-1) events
            for k in ("event_lanes", "events_bh_window_only", "interval1_small_budget_lanes_by_slot"):
                out.pop(k, None)
            out["spent_slots_interval1"] = dict(zip(["1", "2", "3+"], [int(hi[12 + k]) for k in range(3)]))
            out["spent_slots_longer"] = dict(zip(["1", "2", "3+"], [int(hi[15 + k]) for k in range(3)]))
            out["interval1_runs"] = dict(zip(["1", "2-3", "4-7", "8-15", "16+"], [int(hi[18 + k]) for k in range(5)]))
            out["interval1_one_slot_by_slot"] = [int(hi[23 + j]) for j in range(7)]
        if args.xcyl:  # an SR_STATS_XCYL build: the first budgeted cylinder's spends by orbital-plane distance
            for k in ("event_lanes", "events_bh_window_only", "interval1_small_budget_lanes_by_slot"):
                out.pop(k, None)
            ds = ["0.25", "1", "2", "4"]
            out["cyl_spent_lanes"] = int(hi[12])
            out["cyl_spent_lanes_plane_beyond_br_plus"] = dict(zip(ds, [int(hi[13 + k]) for k in range(4)]))
            out["cyl_events"] = int(hi[17])
            out["cyl_alone_events"] = int(hi[22])
            out["cyl_alone_events_all_lanes_beyond_br_plus"] = dict(zip(ds, [int(hi[18 + k]) for k in range(4)]))
        if args.trig:  # an SR_STATS_TRIG build: counters 44..63 hold the lanes that spent each slot
            for k in ("event_lanes", "events_bh_window_only", "interval1_small_budget_lanes_by_slot"):
                out.pop(k, None)
            out["own_spent_lanes_ring"] = [int(hi[12 + j]) for j in range(7)]
            out["own_spent_lanes_other"] = [int(hi[19 + j]) for j in range(7)]
            out["lookahead_only_events"] = [int(hi[26 + j]) for j in range(6)]
    # wave timeline of the integrate kernel (lane 0 of each wave that had pixels)
    import numpy as np

    nw = ((1920 + 15) // 16) * ((1080 + 15) // 16) * 4
    tb = (C.c_ulonglong * (16 * nw))()
    lib.sr_debug_wave_times.restype = C.c_int
    lib.sr_debug_wave_times.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    assert lib.sr_debug_wave_times(tb, nw) == 0
    t = np.frombuffer(tb, dtype=np.uint64).reshape(nw, 16).astype(np.int64)
    if args.save:
        np.save(args.save, t)
    wid = np.arange(nw)[t[:, 1] > 0]
    t = t[t[:, 1] > 0]
    t0 = t[:, 0].min()
    s_, e_ = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0  # microseconds
    span = e_.max()
    grid = np.linspace(0, span, 41)
    active = [int(((s_ <= x) & (e_ > x)).sum()) for x in grid]
    out["timeline_us"] = round(float(span), 1)
    out["active_waves_at_5pct"] = active
    out["wave_us_mean"] = round(float((e_ - s_).mean()), 1)
    out["wave_us_max"] = round(float((e_ - s_).max()), 1)
    out["last_start_us"] = round(float(s_.max()), 1)
    out["busy_frac"] = round(float((e_ - s_).sum() / (span * max(active))), 3)
    # in-kernel shader clock (rec[15]: s_memtime cycles of the wave over its
    # s_memrealtime span at 100 MHz; MI355X_MICROARCH.md DVFS item 6). Use an
    # SR_STATS_NOCOUNT build: the counters' atomics distort the timeline.
    ok = (t[:, 15] > 0) & (e_ - s_ > 50.0)
    if ok.any():
        ghz = t[ok, 15] / ((e_ - s_)[ok] * 1e3)
        out["clock_ghz"] = {"median": round(float(np.median(ghz)), 3), "p10": round(float(np.percentile(ghz, 10)), 3),
                            "p90": round(float(np.percentile(ghz, 90)), 3), "waves": int(ok.sum())}
    dur = e_ - s_
    top = np.argsort(-dur)[:8]
    gx = (1920 + 15) // 16
    out["slowest_waves"] = [
        {"us": round(float(dur[k]), 1), "start_us": round(float(s_[k]), 1), "block_xy": [int(wid[k] // 4 % gx), int(wid[k] // 4 // gx)],
         "wave": int(wid[k] % 4), "max_steps": int(t[k, 2]), "events": int(t[k, 3] >> 32), "exact_chords": int(t[k, 3] & 0xffffffff),
         "reach_by_slot": [int(x) for x in t[k, 4:13]]}
        for k in top]
    ms = t[:, 2].astype(float)
    out["us_per_step_by_steps"] = {f"{lo}-{hi}": round(float((dur[(ms >= lo) & (ms < hi)] / ms[(ms >= lo) & (ms < hi)]).mean()), 3)
                                   for lo, hi in [(100, 500), (500, 1000), (1000, 1500), (1500, 2001)] if ((ms >= lo) & (ms < hi)).any()}
    print(json.dumps(out))
    r.close()


if __name__ == "__main__":
    main()
