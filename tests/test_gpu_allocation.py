"""Register-allocation independence of the kernel.

Round 5 built the small integrate instantiation for 7 waves per SIMD (72
VGPRs, spilling) and that build of the same source rendered the press-R
overlay frame wrong (16,507 pixels of c2t) and faulted in the golden cases.
The post-mortem (tools/ub_probe.py over the
integrate -> shade hand-off) found lanes of the overlay waves whose hit-log
count, ray origin and direction were garbage (7 .. 31 logged hits, rd = -inf):
registers corrupted, not a wrong decision. The present source is held to the
same bits at two register allocations: libsr.so builds the small
instantiation for 7 waves per SIMD since round 6 (72 VGPRs), and `make` also
builds lib/libsr_alt.so, the identical kernel source at 6 waves per SIMD (80
VGPRs; the Makefile's ALT_WAVES). Every case here must equal the oracle's
fixtures or libsr.so's own output bit for bit (float FragColor, RGBA8, step
counts).
"""
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent
LIBALT = ROOT / "schwarzschild-raytracer_amd" / "lib" / "libsr_alt.so"
BLOCK_ROWS = 8


@pytest.fixture(scope="module")
def libalt(pkg):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    assert LIBALT.exists(), "lib/libsr_alt.so not built (make -C schwarzschild-raytracer_amd)"
    return pkg.abi.load(LIBALT)


@pytest.fixture(scope="module")
def fh():
    from test_gpu_frames import FIXTURE

    with np.load(FIXTURE) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="module")
def assets(pkg):
    A = pkg.assets
    if not A.available():
        pytest.skip("assets/textures missing")
    arr, _, _ = A.texture_array()
    return {"2k": A.skybox("2k"), "arr": arr}


def debug(r, scene, cam, params, w, h, test_ray):
    import torch

    r.set_scene(scene)
    r.set_test_ray(test_ray)
    f, b, s = r.render_debug(cam, params, w, h)
    torch.cuda.synchronize()
    return f.cpu().numpy().view(np.uint32), b.cpu().numpy(), s.cpu().numpy()


def test_alt_library_shares_the_abi(pkg, libalt):
    """The test library differs from libsr.so only in the kernel's
    allocation: same ABI (struct sizes)."""
    import ctypes as C

    n = 6
    a, b = (C.c_size_t * n)(), (C.c_size_t * n)()
    pkg.abi.load().sr_abi_struct_sizes(a, n)
    libalt.sr_abi_struct_sizes(b, n)
    assert list(a) == list(b)


@pytest.mark.parametrize("cfg,variant", [("c2t", "testray"), ("c2s", "stress"), ("c2", "default")])
def test_alt_frames_exact(pkg, libalt, fh, assets, cfg, variant):
    """The frames that failed in round 5's 7-wave build (c2t: the overlay's
    1000 cylinders, whose waves lost their registers), the max-capacity scene
    and config 2, through the other allocation: the debug render and two
    batched launches of four frames, every row against the oracle's hashes
    (tests/golden/frame_hashes.npz)."""
    import torch
    from test_gpu_frames import frame_digest, sha_rows

    W, H, N = (int(v) for v in fh[f"{cfg}/config"])
    abi, sc = pkg.abi, pkg.scenes
    r = pkg.Renderer(0, lib=libalt)
    r.set_background(assets["2k"])
    r.set_texture_array(assets["arr"])
    scene = sc.scene_stress() if variant == "stress" else sc.scene_default(textured=True)
    tr = sc.test_ray_overlay() if variant == "testray" else abi.default_test_ray()
    params = abi.default_params(max_steps=N, percent_black=-1.0)
    cam = abi.default_camera()
    _, b, s = debug(r, scene, cam, params, W, H, tr)
    rows = fh[f"{cfg}/rows"]
    bad = np.flatnonzero((sha_rows(b[rows]) != fh[f"{cfg}/rgba_sha"]).any(-1))
    assert not len(bad), f"{cfg} (the other allocation): {len(bad)} RGBA8 rows differ, first {rows[bad[:5]].tolist()}"
    assert not (sha_rows(s[rows].astype("<i4")) != fh[f"{cfg}/steps_sha"]).any(), f"{cfg}: step rows differ"
    B = 4
    for _ in range(2):
        out, _ = r.render_blocks_batch([cam] * B, params, W, H, BLOCK_ROWS, 0, 1)
    torch.cuda.synchronize()
    frames = out.cpu().numpy()
    for f in range(B):
        assert frame_digest(frames[f, :H]) == bytes(fh[f"{cfg}/frame_sha"]).hex(), f"{cfg}: batched frame {f}"
    r.close()


def test_alt_golden_cases_equal_the_shipping_build(pkg, libalt, golden, golden_cases, textures):
    """Every golden case (the case set that faulted in round 5's 7-wave
    build) rendered by both allocations: identical float FragColor, RGBA8 and
    step counts (libsr.so is held to the oracle by test_golden_cases_bit_exact)."""
    from conftest import case_texture_kind, load_case, texture_array_of

    bg, _ = textures
    by_kind = {}
    for name in golden_cases:
        by_kind.setdefault(case_texture_kind(golden, name), []).append(name)
    for kind, names in by_kind.items():
        arr = texture_array_of(pkg, kind)
        rs = [pkg.Renderer(0), pkg.Renderer(0, lib=libalt)]
        for r in rs:
            r.set_background(bg)
            r.set_texture_array(arr)
        for name in names:
            scene, cam, params, tr, w, h = load_case(pkg, golden, name)
            outs = [debug(r, scene, cam, params, w, h, tr) for r in rs]
            for k, what in enumerate(("FragColor", "RGBA8", "steps")):
                assert np.array_equal(outs[0][k], outs[1][k]), f"{name}: {what} differs between the allocations"
        for r in rs:
            r.close()


@pytest.mark.parametrize("seed", range(6))
def test_alt_random_scenes_and_overlays_equal(pkg, libalt, textures, seed):
    """Random stress scenes (18-21 objects: the general and large
    instantiations, logged translucent hits, resumed rays) and random
    cameras with and without a visible test ray: both allocations agree
    bit for bit."""
    sc, abi = pkg.scenes, pkg.abi
    bg, arr = textures
    rs = [pkg.Renderer(0), pkg.Renderer(0, lib=libalt)]
    for r in rs:
        r.set_background(bg)
        r.set_texture_array(arr)
    cases = [(sc.scene_random(500 + seed, planes=seed % 2 == 0), sc.random_camera(600 + seed), abi.default_test_ray()),
             (sc.scene_default(textured=True), sc.random_camera(700 + seed), sc.test_ray_overlay())]
    params = abi.default_params(max_steps=800, percent_black=-1.0)
    for i, (scene, cam, tr) in enumerate(cases):
        outs = [debug(r, scene, cam, params, 128, 72, tr) for r in rs]
        for k, what in enumerate(("FragColor", "RGBA8", "steps")):
            assert np.array_equal(outs[0][k], outs[1][k]), f"seed {seed} case {i}: {what} differs"
    for r in rs:
        r.close()
