#!/usr/bin/env python3
"""Mean duration of bench.py's timed integrate launches in a rocprofv3
kernel trace, to set beside the bench line's own roofline.kernel_ms (HIP
events on every frame's stream over the same timed region).

bench.py's integrate<true> dispatches, in dispatch order: one step-count
render (render_debug), max(warmup, F) warmup frames, then the K timed frames
(then the latency and reference-loop frames).
  python tools/trace_kernel_ms.py RUN_DIR --warmup 4 --steps 20 [--bench-json bench_stats.json]"""
import argparse
import csv
import glob
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("run")
    ap.add_argument("--warmup", type=int, required=True, help="max(--warmup, frames in flight)")
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--bench-json", default="")
    a = ap.parse_args()
    rows = []
    for p in glob.glob(f"{a.run}/**/*kernel_trace.csv", recursive=True):
        rows += [r for r in csv.DictReader(open(p)) if "sr_integrate_kernel<true>" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    timed = ms[1 + a.warmup: 1 + a.warmup + a.steps]
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
