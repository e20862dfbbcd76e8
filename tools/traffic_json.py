#!/usr/bin/env python3
"""profiles/traffic_latest.json from a FETCH_SIZE / WRITE_SIZE PMC session
(tools/pmc_session.sh, separate passes) of the headline frame:
per-launch HBM-side bytes of sr_integrate_kernel<true, false>.

rocprofv3 reports both in KiB. MI355X_MICROARCH.md (HBM): FETCH_SIZE reads half
the bytes of wide (16 B/lane) coalesced streaming reads; this kernel's reads
are scalar loads of the scene and step table plus dword gathers of the opacity
map, an uncalibrated width, so the raw value is recorded next to the x2 bound.
WRITE_SIZE is exact for its dword stores (the pixel-state hand-off planes).
  python tools/traffic_json.py --frame <FETCH_SIZE run dir> <WRITE_SIZE run dir> [--out profiles/traffic_latest.json]
(per dispatch of the frame grid, tools/pmc_flops.py frame_counters)"""
import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from pmc_flops import frame_counters, frames_per_dispatch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frame", nargs="+", required=True)
    ap.add_argument("--out", default=str(Path(__file__).resolve().parents[1] / "profiles" / "traffic_latest.json"))
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--max-steps", type=int, default=2000)
    ap.add_argument("--variant", default="default", choices=["default", "stress", "testray"],
                    help="the bench's scene variant (--scene stress / --test-ray on)")
    a = ap.parse_args()
    import bench

    grid, c, _ = frame_counters(a.frame)
    B = frames_per_dispatch(grid, a.width, a.height)
    fetch = c["FETCH_SIZE"] * 1024.0
    write = c["WRITE_SIZE"] * 1024.0
    rec = {
        "kernel": "sr_integrate_kernel<true, false, NB>",
        "kernel_sha": bench.kernel_sha(),
        "width": a.width, "height": a.height, "max_steps": a.max_steps, "variant": a.variant,
        "fetch_bytes_raw": fetch, "fetch_bytes_x2_bound": 2 * fetch, "write_bytes": write,
        "hbm_bytes_per_launch": fetch + write,
        "frames_per_launch": B,
        "hbm_bytes_per_frame": (fetch + write) / B,
        "note": "reads: scene/step table (scalar, cache-resident) + opacity map; writes: pixel-state planes "
                "for the shade kernel (DESIGN.md §6); the algorithmic output is the shade kernel's 4 B/px store",
        "source": " ".join(a.frame),
    }
    Path(a.out).write_text(json.dumps(rec, indent=1) + "\n")
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
