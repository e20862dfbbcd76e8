#!/usr/bin/env python3
"""Executed FP32 work of the integrate kernel from rocprofv3 --pmc passes,
calibrated against tools/microbench/flops_calib.hip, written as
profiles/pmc_latest.json for bench.py's roofline.

  python tools/pmc_flops.py --calib gpurun_out/S/calib --frame gpurun_out/S/p1 [gpurun_out/S/p2 ...]
      --width 1920 --height 1080 --max-steps 2000 --out profiles/pmc_latest.json --source "..."

Every directory holds one rocprofv3 run (`-d DIR -o run --output-format csv`).
Counters are summed over XCDs / shader engines per dispatch and averaged over
the integrate dispatches of the frame's grid (the most common grid size of
sr_integrate_kernel<true, false>: bench.py's frames; the step-count and band launches
have other grids or are few).
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

# flops_calib.hip: lanes x the known work per lane, per template instance
CALIB_LANES = 1024 * 256
CALIB_WORK = {  # (mode, half) -> (FP32 FLOP per launch, transcendental ops per launch)
    (0, False): (CALIB_LANES * 256 * 4 * 2, 0),
    (0, True): (CALIB_LANES // 2 * 256 * 4 * 2, 0),
    (1, False): (CALIB_LANES * 256 * 2 * 4, 0),
    (2, False): (CALIB_LANES * 256 * 4, 0),
    (3, False): (CALIB_LANES * 256 * 4, 0),
    (4, False): (0, CALIB_LANES * 256 * 4),
}


def dispatches(root):
    """{dispatch_id: (kernel, grid, {counter: value summed over dimensions})}"""
    out = {}
    for p in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(p)):
            d = r["Dispatch_Id"]
            if d not in out:
                out[d] = (r.get("Kernel_Name", ""), int(float(r.get("Grid_Size", 0) or 0)), collections.defaultdict(float))
            out[d][2][r["Counter_Name"]] += float(r["Counter_Value"])
    return out


def calib_factors(root):
    """FLOP per unit of SQ_INSTS_VALU_FLOPS_FP32 (and _TRANS) on each calibration kernel."""
    rows = []
    for _, (name, _, c) in sorted(dispatches(root).items(), key=lambda kv: int(kv[0])):
        if "calib<" not in name:
            continue
        args = name[name.index("calib<") + 6:name.index(">")].split(",")
        key = (int(args[0]), args[1].strip() == "true")
        flop, trans = CALIB_WORK[key]
        rows.append({"kernel": name.split("(")[0], "flop": flop, "trans": trans,
                     **{k: v for k, v in c.items()}})
    return rows


def frame_counters(roots, kernel="sr_integrate_kernel<true, false"):
    per = collections.defaultdict(list)
    grids = collections.Counter()
    recs = []
    for root in roots:
        for _, (name, grid, c) in dispatches(root).items():
            if kernel in name:
                recs.append((grid, c))
                grids[grid] += 1
    if not recs:
        raise SystemExit(f"no {kernel} dispatches under {roots}")
    frame_grid = grids.most_common(1)[0][0]
    for grid, c in recs:
        if grid == frame_grid:
            for k, v in c.items():
                per[k].append(v)
    return frame_grid, {k: sum(v) / len(v) for k, v in per.items()}, {k: len(v) for k, v in per.items()}


def frames_per_dispatch(grid_threads, width, height):
    """Frames one integrate dispatch of a whole-frame grid renders: the grid is
    B x (16x16 tiles) x 256 threads (sr_render_blocks_batch; split tiles off)."""
    tiles = ((width + 15) // 16) * ((height + 15) // 16)
    B, rem = divmod(int(grid_threads), tiles * 256)
    if rem or B < 1:
        raise SystemExit(f"grid of {grid_threads} threads is not a whole number of {width}x{height} frames")
    return B


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calib", required=True)
    ap.add_argument("--frame", nargs="+", required=True)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--max-steps", type=int, default=2000)
    ap.add_argument("--variant", default="default", choices=["default", "stress", "testray"],
                    help="the bench's scene variant (--scene stress / --test-ray on)")
    ap.add_argument("--out", default=str(ROOT / "profiles" / "pmc_latest.json"))
    ap.add_argument("--source", default="")
    args = ap.parse_args()
    import bench

    cal = calib_factors(args.calib)
    for r in cal:
        f = r.get("SQ_INSTS_VALU_FLOPS_FP32", 0.0)
        t = r.get("SQ_INSTS_VALU_FLOPS_FP32_TRANS", 0.0)
        print(f"{r['kernel']:28s} expect flop {r['flop']:.4g} trans {r['trans']:.4g} | FLOPS_FP32 {f:.4g} "
              f"TRANS {t:.4g} VALU {r.get('SQ_INSTS_VALU', 0):.4g} FMA {r.get('SQ_INSTS_VALU_FMA_F32', 0):.4g}")
    # The counter tallies each wave-instruction's FP32 FLOP (FMA 2, packed FMA
    # 4, add / mul / transcendental 1) once per wave, whatever the exec mask:
    # the half-active kernel reads the same as the full one. So it measures
    # the VALU's FP32 issue, 64 lanes per wave-instruction; the factor is
    # fitted on the full-wave kernels (the epilogue's few adds per wave
    # keep it a little under 64).
    full = [r for r in cal if r["flop"] and not r["kernel"].endswith("true>") and r.get("SQ_INSTS_VALU_FLOPS_FP32")]
    k_flop = sum(r["flop"] for r in full) / sum(r["SQ_INSTS_VALU_FLOPS_FP32"] for r in full)
    spread = max(abs(r["flop"] / r["SQ_INSTS_VALU_FLOPS_FP32"] / k_flop - 1.0) for r in full)
    half = [r for r in cal if r["kernel"].endswith("true>")]
    mask_blind = bool(half) and all(abs(h.get("SQ_INSTS_VALU_FLOPS_FP32", 0) / max(1.0, f.get("SQ_INSTS_VALU_FLOPS_FP32", 1))
                                        - 1.0) < 0.02 for h in half for f in full[:1])
    tr = [r for r in cal if r["trans"] and r.get("SQ_INSTS_VALU_FLOPS_FP32_TRANS")]
    k_trans = (sum(r["trans"] for r in tr) / sum(r["SQ_INSTS_VALU_FLOPS_FP32_TRANS"] for r in tr)) if tr else k_flop
    trans_in_fp32 = bool(tr) and all(r.get("SQ_INSTS_VALU_FLOPS_FP32", 0) >= r["SQ_INSTS_VALU_FLOPS_FP32_TRANS"] for r in tr)
    print(f"FLOP per FLOPS_FP32 unit {k_flop:.4g} (max deviation over full-wave kernels {spread:.3%}); "
          f"exec-mask blind: {mask_blind}; transcendentals inside FLOPS_FP32: {trans_in_fp32}; per TRANS unit {k_trans:.4g}")

    grid, c, n = frame_counters(args.frame)
    B = frames_per_dispatch(grid, args.width, args.height)
    flop = c.get("SQ_INSTS_VALU_FLOPS_FP32", 0.0) * k_flop  # transcendentals included (1 each)
    trans = c.get("SQ_INSTS_VALU_FLOPS_FP32_TRANS", 0.0) * k_trans
    rec = {
        "kernel": "sr_integrate_kernel<true, false, NB>",
        "kernel_sha": bench.kernel_sha(),
        "width": args.width,
        "height": args.height,
        "max_steps": args.max_steps,
        "variant": args.variant,
        "grid_threads": grid,
        "dispatches_averaged": max(n.values()) if n else 0,
        "frames_per_launch": B,
        "flop_per_launch": flop,
        "trans_ops_per_launch": trans,
        "valu_insts_per_launch": c.get("SQ_INSTS_VALU"),
        "flop_per_frame": flop / B,
        "valu_insts_per_frame": None if c.get("SQ_INSTS_VALU") is None else c["SQ_INSTS_VALU"] / B,
        "calibration": {"flop_per_unit": k_flop, "trans_per_unit": k_trans, "max_deviation": spread,
                        "exec_mask_blind": mask_blind, "trans_inside_fp32": trans_in_fp32},
        "counters": c,
        "note": ("flop_per_launch = SQ_INSTS_VALU_FLOPS_FP32 x flop_per_unit per integrate dispatch of the frame "
                 "grid: FP32 FLOP issued by the VALU, 64 lanes per wave-instruction (the counter ignores the exec "
                 "mask, so lanes of a wave whose rays have ended still count: issue, not useful work); "
                 "transcendentals count 1. Calibrated on flops_calib.hip (v_fma_f32, v_pk_fma_f32, v_add_f32, "
                 "v_mul_f32, v_rcp_f32; full and half-active waves)"),
        "source": args.source,
    }
    Path(args.out).write_text(json.dumps(rec, indent=1) + "\n")
    print(json.dumps({k: rec[k] for k in ("frames_per_launch", "flop_per_launch", "flop_per_frame",
                                          "valu_insts_per_launch", "dispatches_averaged")}))


if __name__ == "__main__":
    main()
