#!/usr/bin/env python3
"""Full-frame parity fixture: per-row SHA-256 of the CPU oracle's frames at the
BASELINE.json GPU configs, on the bench's own inputs.

TEST INFRASTRUCTURE (runs the oracle, oracle/sr_oracle.c, as the checker).
Inputs are exactly what bench.py renders: the app's default scene and camera
(src/main.cpp:222-268), the reference's own textures decoded to stb_image's
bytes (assets/textures: the 2k skybox, the 8k one for the 7680x4320 still as
BACKGROUND_TEXTURE_QUALITY selects it, src/main.cpp:57-63; uv_checker +
cubemap as the texture array, src/main.cpp:207-218), curved mode, noise mask
off, LERP filtering.

For every row y of a config the fixture holds sha256(RGBA8 row bytes) and
sha256(int32 executed-step row bytes), 32 bytes each, rows bottom-up (GL
order, as sr_render writes them). The frames themselves are not committed.
tests/test_gpu_frames.py renders the same frames on the GPU and compares every
row hash exactly; bench.py compares a timed frame's hash.

Work is chunked and resumable (scratch chunks under tests/golden/.fh_work/,
git-ignored), so the 7680x4320 / 8000-step still (about two hours of eight
cores here) can run in the background and be merged whenever rows are done:
    python tests/golden/make_frame_hashes.py                # configs 2, 3, 4, then 5
    python tests/golden/make_frame_hashes.py --config c5 --rows ring   # 512 rows through the hole + 64 spread
    python tests/golden/make_frame_hashes.py --merge        # write tests/golden/frame_hashes.npz
"""
from __future__ import annotations

import argparse
import hashlib
import os
import sys
import time
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path.insert(0, str(ROOT))
import srpkg  # noqa: E402

OUT = HERE / "frame_hashes.npz"
WORK = HERE / ".fh_work"
# BASELINE.json configs 2-5: name -> (width, height, max_steps, skybox)
CONFIGS = {
    "c2": (640, 360, 1000, "2k"),
    "c3": (1920, 1080, 2000, "2k"),
    "c4": (3840, 2160, 4000, "2k"),
    "c5": (7680, 4320, 8000, "8k"),
    # config 2's size with what the default scene hides (bench.py --scene
    # stress / --test-ray on): the max-capacity scene, and the default scene
    # with the press-R overlay's 1000-point polyline
    "c2s": (640, 360, 1000, "2k"),
    "c2t": (640, 360, 1000, "2k"),
    # the same at the headline size (round 6: bench.py --scene stress /
    # --test-ray on at 1920x1080 / 2000 steps)
    "c3s": (1920, 1080, 2000, "2k"),
    "c3t": (1920, 1080, 2000, "2k"),
}
VARIANTS = {"c2s": "stress", "c2t": "testray", "c3s": "stress", "c3t": "testray"}  # the others: "default"
CHUNK = 16


def row_hashes(rgba8: np.ndarray, steps: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """[rows, 32] uint8 SHA-256 of each RGBA8 row and each int32 (little-endian) step row."""
    rows = rgba8.shape[0]
    hr = np.zeros((rows, 32), dtype=np.uint8)
    hs = np.zeros((rows, 32), dtype=np.uint8)
    st = np.ascontiguousarray(steps.astype("<i4"))
    px = np.ascontiguousarray(rgba8)
    for k in range(rows):
        hr[k] = np.frombuffer(hashlib.sha256(px[k].tobytes()).digest(), dtype=np.uint8)
        hs[k] = np.frombuffer(hashlib.sha256(st[k].tobytes()).digest(), dtype=np.uint8)
    return hr, hs


def frame_digest(row_sha: np.ndarray) -> str:
    """One frame's hash: sha256 over its rows' RGBA8 hashes in row order."""
    return hashlib.sha256(np.ascontiguousarray(row_sha, dtype=np.uint8).tobytes()).hexdigest()


def inputs(pkg, skybox: str, variant: str = "default"):
    """scene, camera, skybox, texture array and test ray (None: hidden) of a config"""
    A, sc, abi = pkg.assets, pkg.scenes, pkg.abi
    bg = A.skybox(skybox)
    arr, _, _ = A.texture_array()
    scene = sc.scene_stress() if variant == "stress" else sc.scene_default(textured=True)
    test_ray = sc.test_ray_overlay() if variant == "testray" else None
    return scene, abi.default_camera(), bg, arr, test_ray


def ring_rows(H: int) -> list[int]:
    """512 rows centred on the black hole (the frame's longest rays) plus 64
    rows spread over the frame."""
    c = H // 2
    band = list(range(c - 256, c + 256))
    spread = [int(v) for v in np.linspace(0, H - 1, 64).round()]
    return sorted(set(band) | set(spread))


def chunk_path(cfg: str, y0: int) -> Path:
    return WORK / f"{cfg}_{y0:05d}.npz"


def run(cfg: str, rows: list[int], threads: int) -> None:
    pkg = srpkg.load_package()
    oracle = srpkg.load_oracle()
    W, H, N, sky = CONFIGS[cfg]
    scene, cam, bg, arr, test_ray = inputs(pkg, sky, VARIANTS.get(cfg, "default"))
    tex = oracle.TextureSet(bg, arr)
    params = pkg.abi.default_params(max_steps=N, percent_black=-1.0)
    WORK.mkdir(exist_ok=True)
    want = sorted(set(rows))
    # chunks: runs of consecutive rows, at most CHUNK long, aligned to CHUNK
    chunks = []
    for y in want:
        if chunks and y == chunks[-1][1] and y % CHUNK:
            chunks[-1][1] = y + 1
        else:
            chunks.append([y, y + 1])
    t0 = time.time()
    done_rows = 0
    for y0, y1 in chunks:
        p = chunk_path(cfg, y0)
        if p.exists():
            with np.load(p) as z:
                if int(z["y1"]) >= y1:
                    done_rows += y1 - y0
                    continue
        rgba8, _, steps = oracle.render(scene, cam, params, W, H, tex, test_ray, y0, y1, threads)
        hr, hs = row_hashes(rgba8, steps)
        tmp = p.with_suffix(".tmp.npz")
        np.savez(tmp, y0=y0, y1=y1, rgba_sha=hr, steps_sha=hs, steps_sum=steps.astype(np.int64).sum(axis=1))
        os.replace(tmp, p)
        done_rows += y1 - y0
        el = time.time() - t0
        print(f"{cfg} rows [{y0},{y1}) {done_rows}/{len(want)} {el:7.1f}s", flush=True)


def merge() -> None:
    store = {}
    if OUT.exists():
        with np.load(OUT) as z:
            store = {k: z[k] for k in z.files}
    for cfg, (W, H, N, sky) in CONFIGS.items():
        parts = sorted(WORK.glob(f"{cfg}_*.npz")) if WORK.exists() else []
        if not parts:
            continue
        hr = np.zeros((H, 32), dtype=np.uint8)
        hs = np.zeros((H, 32), dtype=np.uint8)
        ss = np.zeros(H, dtype=np.int64)
        have = np.zeros(H, dtype=bool)
        if f"{cfg}/rows" in store:  # keep rows merged earlier
            r = store[f"{cfg}/rows"]
            hr[r], hs[r], ss[r] = store[f"{cfg}/rgba_sha"], store[f"{cfg}/steps_sha"], store[f"{cfg}/steps_sum"]
            have[r] = True
        for p in parts:
            if p.name.endswith(".tmp.npz"):
                continue
            with np.load(p) as z:
                y0, y1 = int(z["y0"]), int(z["y1"])
                hr[y0:y1], hs[y0:y1], ss[y0:y1] = z["rgba_sha"], z["steps_sha"], z["steps_sum"]
                have[y0:y1] = True
        rows = np.flatnonzero(have).astype(np.int32)
        store[f"{cfg}/rows"] = rows
        store[f"{cfg}/rgba_sha"] = hr[rows]
        store[f"{cfg}/steps_sha"] = hs[rows]
        store[f"{cfg}/steps_sum"] = ss[rows]
        store[f"{cfg}/config"] = np.array([W, H, N], dtype=np.int32)
        store[f"{cfg}/skybox"] = np.frombuffer(sky.encode(), dtype=np.uint8)
        store[f"{cfg}/variant"] = np.frombuffer(VARIANTS.get(cfg, "default").encode(), dtype=np.uint8)
        if len(rows) == H:
            store[f"{cfg}/frame_sha"] = np.frombuffer(bytes.fromhex(frame_digest(hr)), dtype=np.uint8)
        print(f"{cfg}: {len(rows)}/{H} rows, mean steps {ss[rows].sum() / (len(rows) * W):.2f}"
              + (f", frame {frame_digest(hr)[:16]}" if len(rows) == H else ""))
    np.savez_compressed(OUT, **store)
    print("wrote", OUT, OUT.stat().st_size, "bytes")


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=sorted(CONFIGS), action="append")
    ap.add_argument("--rows", choices=["all", "ring"], default="all")
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--merge", action="store_true")
    args = ap.parse_args(argv)
    if args.merge:
        merge()
        return
    for cfg in args.config or ["c2", "c3", "c4", "c5"]:
        H = CONFIGS[cfg][1]
        rows = ring_rows(H) if args.rows == "ring" else list(range(H))
        run(cfg, rows, args.threads)
        merge()


if __name__ == "__main__":
    main()
