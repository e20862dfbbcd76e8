#!/usr/bin/env python3
"""Per-stream timeline of a rocprofv3 kernel trace (run_kernel_trace.csv):
the last N dispatches in start order with their stream, duration and the gap
since the previous kernel on the same stream ended, plus each stream's busy
fraction over the window those dispatches span.
  python tools/stream_timeline.py RUN_DIR [--last 80]"""
import argparse
import csv
import json
from pathlib import Path


def short(name):
    for k in ("sr_integrate_kernel", "sr_shade_kernel", "sr_resume_kernel", "sr_order_kernel", "sr_assemble"):
        if k in name:
            return k.replace("sr_", "").replace("_kernel", "")
    return name.split("(")[0][-24:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("run_dir")
    ap.add_argument("--last", type=int, default=80)
    a = ap.parse_args()
    f = next(Path(a.run_dir).rglob("*kernel_trace.csv"))
    rows = [r for r in csv.DictReader(open(f)) if r["Kind"] == "KERNEL_DISPATCH"]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-a.last:]
    t0 = int(rows[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in rows)
    last_end = {}
    busy = {}
    out = []
    for r in rows:
        s, e, q = int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"]
        gap = (s - last_end[q]) / 1e6 if q in last_end else None
        last_end[q] = e
        busy[q] = busy.get(q, 0) + (e - s)
        out.append({"stream": q, "kernel": short(r["Kernel_Name"]), "start_ms": round((s - t0) / 1e6, 3),
                    "ms": round((e - s) / 1e6, 3), "gap_ms": None if gap is None else round(gap, 3)})
    for o in out:
        print(json.dumps(o))
    span = (t1 - t0) / 1e6
    print(json.dumps({"window_ms": round(span, 3),
                      "busy_frac_by_stream": {q: round(b / 1e6 / span, 3) for q, b in busy.items()}}))


if __name__ == "__main__":
    main()
