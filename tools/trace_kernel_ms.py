#!/usr/bin/env python3
"""Mean duration of bench.py's timed integrate launches in a rocprofv3
kernel trace, to set beside the bench line's own roofline.kernel_ms (HIP
events on every frame's stream over the same timed region).

bench.py's integrate<true> dispatches, in dispatch order: one step-count
render (render_debug), the warmup launches (max(warmup, F x B) frames in
launches of B), then the timed launches (K frames in launches of B, the
last with the rest), then the latency and reference-loop launches.
  python tools/trace_kernel_ms.py RUN_DIR --warmup 4 --steps 20 [--bench-json bench_stats.json]
(with --bench-json, B and F come from its config)"""
import argparse
import csv
import glob
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("run")
    ap.add_argument("--warmup", type=int, required=True, help="bench.py --warmup")
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--bench-json", default="")
    a = ap.parse_args()
    rows = []
    for p in glob.glob(f"{a.run}/**/*kernel_trace.csv", recursive=True):
        rows += [r for r in csv.DictReader(open(p)) if "sr_integrate_kernel<true, false" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    B, F = 1, 4
    if a.bench_json:
        cfg = json.load(open(a.bench_json))["config"]
        B, F = cfg.get("frames_per_launch", 1), cfg.get("launches_in_flight", cfg.get("frames_in_flight", 4))
    warm = -(-max(a.warmup, F * B) // B)
    timed = ms[1 + warm: 1 + warm + -(-a.steps // B)]
    out = {"integrate_dispatches": len(ms), "timed_dispatches": len(timed),
           "timed_mean_ms": round(sum(timed) / len(timed), 4), "timed_min_ms": round(min(timed), 4),
           "timed_max_ms": round(max(timed), 4), "all_mean_ms": round(sum(ms) / len(ms), 4)}
    if a.bench_json:
        b = json.load(open(a.bench_json))
        out["bench_kernel_ms"] = b["roofline"]["kernel_ms"]
        out["bench_ms_per_step"] = b["ms_per_step"]
        out["agreement"] = round(out["timed_mean_ms"] / b["roofline"]["kernel_ms"], 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
