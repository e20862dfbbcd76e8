"""Full-frame, exact parity at every GPU config of BASELINE.json, on the
bench's own inputs (the reference's textures, the app's default scene and
camera, src/main.cpp:57-63, 207-268).

tests/golden/make_frame_hashes.py ran the CPU oracle over these frames in the
build container and committed, per row, sha256 of the RGBA8 bytes and of the
int32 executed-step counts (tests/golden/frame_hashes.npz). Here the GPU
renders the same frames - through the paths bench.py uses: batched launches
with a learned launch order, and config 4 as its eight cost-balanced rank
shares reassembled by the library's sr_assemble_blocks - and every row hash
must be equal.
No tolerance: the arithmetic contract makes the kernel's
pixels the oracle's bit for bit. Mismatching rows are re-run through the
oracle for the failure message.
"""
import hashlib
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FIXTURE = Path(__file__).resolve().parent / "golden" / "frame_hashes.npz"
BLOCK_ROWS = 8


@pytest.fixture(scope="module")
def fh():
    if not FIXTURE.exists():
        pytest.skip("tests/golden/frame_hashes.npz missing (python tests/golden/make_frame_hashes.py)")
    with np.load(FIXTURE) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="module")
def assets(pkg):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    A = pkg.assets
    if not A.available():
        pytest.skip("assets/textures missing")
    arr, _, _ = A.texture_array()
    return {"2k": A.skybox("2k"), "arr": arr}


def renderer(pkg, assets, skybox):
    r = pkg.Renderer(0)
    r.set_scene(pkg.scenes.scene_default(textured=True))
    r.set_background(assets[skybox] if skybox in assets else pkg.assets.skybox(skybox))
    r.set_texture_array(assets["arr"])
    return r


def sha_rows(a: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(a)
    return np.stack([np.frombuffer(hashlib.sha256(a[k].tobytes()).digest(), dtype=np.uint8)
                     for k in range(a.shape[0])])


def compare(pkg, fh, cfg, rgba8, steps=None, what=""):
    """Every fixture row of the frame: RGBA8 (and step) hashes equal."""
    W, H, N = (int(v) for v in fh[f"{cfg}/config"])
    rows = fh[f"{cfg}/rows"]
    assert rgba8.shape == (H, W, 4)
    bad = np.flatnonzero((sha_rows(rgba8[rows]) != fh[f"{cfg}/rgba_sha"]).any(-1))
    bad_s = np.array([], dtype=np.int64)
    if steps is not None:
        bad_s = np.flatnonzero((sha_rows(steps[rows].astype("<i4")) != fh[f"{cfg}/steps_sha"]).any(-1))
    if len(bad) or len(bad_s):
        msg = [f"{cfg} {what}: {len(bad)} RGBA8 rows and {len(bad_s)} step rows of {len(rows)} differ"]
        try:  # diagnostics: the oracle's pixels of the first mismatching rows
            import srpkg

            oracle = srpkg.load_oracle()
            sky = bytes(fh[f"{cfg}/skybox"]).decode()
            A = pkg.assets
            arr, _, _ = A.texture_array()
            tex = oracle.TextureSet(A.skybox(sky), arr)
            params = pkg.abi.default_params(max_steps=N, percent_black=-1.0)
            for k in list(bad[:3]) + list(bad_s[:2]):
                y = int(rows[k])
                rb, _, rs = oracle.render(pkg.scenes.scene_default(textured=True), pkg.abi.default_camera(), params,
                                          W, H, tex, None, y, y + 1)
                px = (rb[0] != rgba8[y]).any(-1)
                msg.append(f"row {y}: {int(px.sum())} px differ (first at x={np.flatnonzero(px)[:5].tolist()})"
                           + ("" if steps is None else f", {int((rs[0] != steps[y]).sum())} step counts"))
        except Exception as e:  # noqa: BLE001
            msg.append(f"(oracle diagnostics failed: {e})")
        raise AssertionError("\n".join(msg))
    return len(rows)


def frame_digest(rgba8):
    return hashlib.sha256(np.ascontiguousarray(sha_rows(rgba8)).tobytes()).hexdigest()


def test_fixture_covers_the_configs(fh):
    """configs 2-5 and the stress / test-ray variants of configs 2 and 3 in
    full (every row), each with its frame hash"""
    for cfg, H in (("c2", 360), ("c3", 1080), ("c4", 2160), ("c5", 4320), ("c2s", 360), ("c2t", 360),
                   ("c3s", 1080), ("c3t", 1080)):
        assert len(fh[f"{cfg}/rows"]) == H, cfg
        assert f"{cfg}/frame_sha" in fh, cfg


@pytest.mark.parametrize("cfg", ["c2", "c3"])
def test_full_frame_exact(pkg, fh, assets, cfg):
    """Configs 2 and 3 (the metric): the debug render (steps) and the bench's
    batched launches (eight static-camera frames, second launch on the
    learned cost order), every row of every frame."""
    import torch

    W, H, N = (int(v) for v in fh[f"{cfg}/config"])
    abi = pkg.abi
    r = renderer(pkg, assets, "2k")
    params = abi.default_params(max_steps=N, percent_black=-1.0)
    cam = abi.default_camera()
    _, b, s = r.render_debug(cam, params, W, H)
    torch.cuda.synchronize()
    compare(pkg, fh, cfg, b.cpu().numpy(), s.cpu().numpy(), "debug render")
    B = 8
    for _ in range(2):
        out, rows = r.render_blocks_batch([cam] * B, params, W, H, BLOCK_ROWS, 0, 1)
    torch.cuda.synchronize()
    assert rows == H
    frames = out.cpu().numpy()
    for f in range(B):
        compare(pkg, fh, cfg, frames[f, :H], None, f"batched frame {f}")
    if f"{cfg}/frame_sha" in fh:
        assert frame_digest(frames[B - 1, :H]) == bytes(fh[f"{cfg}/frame_sha"]).hex()
    r.close()


def test_config4_rank_shares_assembled(pkg, fh, assets):
    """Config 4 (3840x2160, 4000 steps, row-tiled over 8 GPUs): the eight
    cost-balanced rank shares of bench.py (sr_wave_costs -> dist.block_costs
    -> balanced_blocks -> sr_render_block_list, two frames per launch)
    reassembled by sr_assemble_blocks on the device, and the step map of the
    debug render."""
    import torch

    W, H, N = (int(v) for v in fh["c4/config"])
    abi, D = pkg.abi, pkg.dist
    r = renderer(pkg, assets, "2k")
    params = abi.default_params(max_steps=N, percent_black=-1.0)
    cam = abi.default_camera()
    _, b, s = r.render_debug(cam, params, W, H)
    torch.cuda.synchronize()
    compare(pkg, fh, "c4", b.cpu().numpy(), s.cpu().numpy(), "debug render")
    del b, s
    world = 8
    lists = D.balanced_blocks(D.block_costs(r.wave_costs(cam, params, W, H)), world)
    tiles = []
    for lst in lists:
        for _ in range(2):  # the second launch runs the list's learned order
            t = r.render_block_list([cam, cam], params, W, H, BLOCK_ROWS, lst)
        tiles.append(t.clone())
    # the root's reassembly: the library's kernel (sr_assemble_blocks, as bench.py's
    # FrameGather runs it) and dist.assemble_lists' statement of it
    stacked = torch.stack(tiles)
    frames = D.assemble_blocks_abi(stacked, lists, H, BLOCK_ROWS)
    torch.cuda.synchronize()
    frames = frames.cpu().numpy()
    assert np.array_equal(frames, D.assemble_lists(stacked.cpu().numpy(), lists, H, BLOCK_ROWS))
    for f in range(2):
        compare(pkg, fh, "c4", frames[f], None, f"8 rank shares, frame {f}")
    r.close()


def test_config5_still_8k(pkg, fh, assets):
    """Config 5 (7680x4320 offline still, 8000 steps, the 8k skybox): every
    row, RGBA8 and step counts, and a second frame through the learned order."""
    import torch

    W, H, N = (int(v) for v in fh["c5/config"])
    abi = pkg.abi
    r = renderer(pkg, assets, bytes(fh["c5/skybox"]).decode())
    params = abi.default_params(max_steps=N, percent_black=-1.0)
    cam = abi.default_camera()
    _, b, s = r.render_debug(cam, params, W, H)
    torch.cuda.synchronize()
    compare(pkg, fh, "c5", b.cpu().numpy(), s.cpu().numpy(), "debug render")
    del b, s
    for _ in range(2):
        out = r.render(cam, params, W, H)
    torch.cuda.synchronize()
    compare(pkg, fh, "c5", out.cpu().numpy(), None, "second frame")
    r.close()


def test_cpp_multi_gpu_driver_frame(pkg, fh, assets, tmp_path):
    """examples/sr_multi_gpu (C++ over the C-ABI, RCCL): the node-level path -
    sr_render_block_list on F slots per GPU with B frames per launch and the
    gathers on a collective stream, ordered by events (no host wait in the
    timed loop); N > 1 adds sr_wave_costs -> sr_block_costs ->
    sr_balanced_blocks and ncclGather + sr_assemble_blocks - renders the
    headline frame with the reference's textures (raw files) equal row for
    row to the oracle fixture, and reports its rate."""
    import json
    import subprocess

    exe = Path(__file__).resolve().parents[1] / "examples" / "bin" / "sr_multi_gpu"
    if not exe.exists():
        pytest.skip("examples/bin/sr_multi_gpu not built")
    W, H, N = (int(v) for v in fh["c3/config"])
    sky, arr = assets["2k"], assets["arr"]
    (tmp_path / "sky.rgb").write_bytes(np.ascontiguousarray(sky).tobytes())
    a = np.ascontiguousarray(arr)
    if a.shape[-1] == 3:
        a = np.concatenate([a, np.full(a.shape[:-1] + (1,), 255, np.uint8)], axis=-1)
    (tmp_path / "arr.rgba").write_bytes(a.tobytes())
    out = tmp_path / "frame.rgba"
    cmd = [str(exe), "--gpus", "1", "--width", str(W), "--height", str(H), "--max-steps", str(N), "--frames", "7",
           "--batch", "2", "--inflight", "3", "--warmup", "6",
           "--skybox", f"{tmp_path / 'sky.rgb'}:{sky.shape[1]}:{sky.shape[0]}",
           "--array", f"{tmp_path / 'arr.rgba'}:{a.shape[2]}:{a.shape[1]}:{a.shape[0]}", "--out-raw", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    # the pipeline: 2 frames per launch, 3 launches in flight (the last launch renders one frame)
    assert line["world_size"] == 1 and line["frames"] == 7 and line["ranks"][0]["render_ms_per_frame"] > 0
    assert line["frames_per_launch"] == 2 and line["launches_in_flight"] == 3
    assert line["unit"] == "Mpixels/s" and line["value"] > 0 and line["ms_per_frame"] > 0
    frame = np.frombuffer(out.read_bytes(), dtype=np.uint8).reshape(H, W, 4)
    compare(pkg, fh, "c3", frame, None, "C++ driver pipeline")
    # the N > 1 path on the one GPU: priced lists, ncclGather (one rank) and sr_assemble_blocks
    r = subprocess.run(cmd + ["--force-gather"], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["collective"].startswith("ncclGather") and line["value"] > 0
    frame = np.frombuffer(out.read_bytes(), dtype=np.uint8).reshape(H, W, 4)
    compare(pkg, fh, "c3", frame, None, "C++ RCCL driver (gather path)")


def test_frame_gather_device_reassembly(pkg, fh, assets):
    """bench.py's FrameGather on device tiles (the nccl path without the
    collective: world 1): a cost-balanced list rendered by
    sr_render_block_list, reassembled by sr_assemble_blocks into the
    gather's frame buffer, equals the oracle's headline frame; then three
    frames of a batch."""
    import torch

    W, H, N = (int(v) for v in fh["c3/config"])
    abi, D = pkg.abi, pkg.dist
    r = renderer(pkg, assets, "2k")
    params = abi.default_params(max_steps=N, percent_black=-1.0)
    cam = abi.default_camera()
    costs = D.block_costs(r.wave_costs(cam, params, W, H))
    lists = D.balanced_blocks(costs[::-1].copy(), 1)  # one rank: every block, in some order
    lists = [sorted(lists[0], key=lambda b: (b * 7) % 135)]  # a permuted list exercises the reassembly
    tile = torch.zeros((3, len(lists[0]) * BLOCK_ROWS, W, 4), dtype=torch.uint8, device="cuda")
    g = D.FrameGather(tile, 1, 0, H, BLOCK_ROWS)
    g.set_lists(lists)
    for _ in range(2):
        r.render_block_list([cam] * 3, params, W, H, BLOCK_ROWS, lists[0], out=tile)
        frames = g(3)
    torch.cuda.synchronize()
    assert tuple(frames.shape) == (3, H, W, 4)
    for f in range(3):
        compare(pkg, fh, "c3", frames[f].cpu().numpy(), None, f"FrameGather frame {f}")
    r.close()


@pytest.mark.parametrize("cfg,variant", [("c2s", "stress"), ("c2t", "testray"), ("c3s", "stress"),
                                         ("c3t", "testray")])
def test_variant_frames_exact(pkg, fh, assets, cfg, variant):
    """What the default scene hides, at config 2's size and at the headline's
    (bench.py --scene stress / --test-ray on): the max-capacity scene (21
    objects, every one a budget slot of the large instantiation; 10
    materials, 4 lights) and the default scene with the press-R overlay's
    1000-point polyline (1000 cylinders against every chord). The debug
    render (steps) and two batched launches, every row against the oracle's
    hashes."""
    import torch

    W, H, N = (int(v) for v in fh[f"{cfg}/config"])
    assert bytes(fh[f"{cfg}/variant"]).decode() == variant
    abi, sc = pkg.abi, pkg.scenes
    r = pkg.Renderer(0)
    r.set_scene(sc.scene_stress() if variant == "stress" else sc.scene_default(textured=True))
    r.set_background(assets["2k"])
    r.set_texture_array(assets["arr"])
    r.set_test_ray(sc.test_ray_overlay() if variant == "testray" else abi.default_test_ray())
    params = abi.default_params(max_steps=N, percent_black=-1.0)
    cam = abi.default_camera()
    _, b, s = r.render_debug(cam, params, W, H)
    torch.cuda.synchronize()
    b, s = b.cpu().numpy(), s.cpu().numpy()
    rows = fh[f"{cfg}/rows"]
    assert not (sha_rows(b[rows]) != fh[f"{cfg}/rgba_sha"]).any(), f"{cfg}: RGBA8 rows differ"
    assert not (sha_rows(s[rows].astype("<i4")) != fh[f"{cfg}/steps_sha"]).any(), f"{cfg}: step rows differ"
    B = 4
    for _ in range(2):
        out, n = r.render_blocks_batch([cam] * B, params, W, H, BLOCK_ROWS, 0, 1)
    torch.cuda.synchronize()
    frames = out.cpu().numpy()
    for f in range(B):
        assert frame_digest(frames[f, :H]) == bytes(fh[f"{cfg}/frame_sha"]).hex(), f"{cfg}: batched frame {f}"
    r.close()
