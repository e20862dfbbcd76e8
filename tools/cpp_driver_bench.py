#!/usr/bin/env python3
"""The C++ node driver (examples/bin/sr_multi_gpu) against bench.py on one
GPU, interleaved: both at the headline config with the reference's textures
(the driver reads them as raw files written here), the same pipeline (B
frames per launch, F launches in flight, K timed frames). Prints one JSON
line per run and a summary line; the driver's last frame is checked against
the oracle's row hashes (tests/golden/frame_hashes.npz c3).

  python tools/cpp_driver_bench.py [--rounds 3] [--frames 20] [--batch 16] [--inflight 2]
"""
import argparse
import hashlib
import json
import statistics
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--inflight", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=32)
    args = ap.parse_args()
    import srpkg

    pkg = srpkg.load_package()
    A = pkg.assets
    sky = np.ascontiguousarray(A.skybox("2k"))
    arr, _, _ = A.texture_array()
    a = np.ascontiguousarray(arr)
    if a.shape[-1] == 3:
        a = np.concatenate([a, np.full(a.shape[:-1] + (1,), 255, np.uint8)], axis=-1)
    W, H, N = 1920, 1080, 2000
    tmp = Path(tempfile.mkdtemp())
    (tmp / "sky.rgb").write_bytes(sky.tobytes())
    (tmp / "arr.rgba").write_bytes(a.tobytes())
    exe = ROOT / "examples" / "bin" / "sr_multi_gpu"
    drv = [str(exe), "--gpus", "1", "--width", str(W), "--height", str(H), "--max-steps", str(N),
           "--frames", str(args.frames), "--batch", str(args.batch), "--inflight", str(args.inflight),
           "--warmup", str(args.warmup), "--skybox", f"{tmp / 'sky.rgb'}:{sky.shape[1]}:{sky.shape[0]}",
           "--array", f"{tmp / 'arr.rgba'}:{a.shape[2]}:{a.shape[1]}:{a.shape[0]}", "--out-raw", str(tmp / "f.rgba")]
    bench = [sys.executable, str(ROOT / "bench.py"), "--steps", str(args.frames), "--batch", str(args.batch),
             "--inflight", str(args.inflight), "--cpu-baseline", "off", "--critical-path", "off",
             "--reference-loop", "off", "--single-frame", "off"]
    with np.load(ROOT / "tests" / "golden" / "frame_hashes.npz") as z:
        rows, ref = z["c3/rows"], z["c3/rgba_sha"]
    res = {"cpp": [], "bench": []}
    for k in range(args.rounds):
        for name, cmd in (("cpp", drv), ("bench", bench)):
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                print(r.stdout[-2000:], r.stderr[-3000:], file=sys.stderr)
                sys.exit(r.returncode)
            line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
            if name == "cpp":
                fr = np.frombuffer((tmp / "f.rgba").read_bytes(), dtype=np.uint8).reshape(H, W, 4)
                sha = np.stack([np.frombuffer(hashlib.sha256(fr[y].tobytes()).digest(), dtype=np.uint8) for y in rows])
                line["parity"] = {"fixture": "tests/golden/frame_hashes.npz c3",
                                  "rows_differing": int((sha != ref).any(-1).sum())}
            else:
                line = {k_: line[k_] for k_ in ("value", "ms_per_step", "parity")}
            res[name].append(line)
            print(json.dumps({"round": k, "run": name, **line}), flush=True)
    mc = statistics.median(x["value"] for x in res["cpp"])
    mb = statistics.median(x["value"] for x in res["bench"])
    print(json.dumps({"summary": True, "cpp_median_mpix_s": mc, "bench_median_mpix_s": mb,
                      "cpp_over_bench": round(mc / mb, 4), "rounds": args.rounds,
                      "cpp_parity_rows_differing": [x["parity"]["rows_differing"] for x in res["cpp"]]}), flush=True)


if __name__ == "__main__":
    main()
