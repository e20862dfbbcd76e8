"""C-ABI library checks that need no GPU: the library loads, exports every
symbol include/sr/sr.h declares, its struct layout matches the ctypes mirror,
argument validation, and the host-side pieces (defaults, ObjectLoader packing
of the app's scene, the press-R geodesic)."""
import ctypes as C
import math
import re
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]


def header_functions():
    text = (ROOT / "include" / "sr" / "sr.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sr_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_header_symbol(pkg):
    lib = pkg.abi.load()
    names = header_functions()
    assert len(names) >= 18
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) == set(pkg.abi.SIGNATURES), "abi.py SIGNATURES out of sync with sr.h"


def test_struct_layout(pkg):
    sizes = pkg.abi.check_layout()
    assert sizes["camera"] == 52 and sizes["params"] == 36


def test_version_and_status_strings(pkg):
    lib = pkg.abi.load()
    assert b"gfx950" in lib.sr_version()
    assert lib.sr_status_string(pkg.abi.SR_E_CAPACITY) == b"capacity exceeded"


def test_create_without_device(pkg):
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("a HIP device is present")
    ctx = C.c_void_p()
    assert pkg.abi.load().sr_create(C.byref(ctx), 0) == pkg.abi.SR_E_NO_DEVICE
    assert not ctx.value


def test_null_arguments_rejected(pkg):
    abi = pkg.abi
    lib = abi.load()
    cam, prm, scene = abi.default_camera(), abi.default_params(), abi.default_scene()
    assert lib.sr_create(None, 0) == abi.SR_E_INVALID
    assert lib.sr_set_scene(None, C.byref(scene)) == abi.SR_E_INVALID
    assert lib.sr_set_background(None, None, 1, 1, 3) == abi.SR_E_INVALID
    assert lib.sr_render(None, C.byref(cam), C.byref(prm), 4, 4, 0, 4, C.c_void_p(16), 16, None) == abi.SR_E_INVALID
    assert lib.sr_render_blocks(None, C.byref(cam), C.byref(prm), 4, 4, 0, 0, 1, C.c_void_p(16), 16, None) \
        == abi.SR_E_INVALID


def test_params_defaults_are_shader_initializers(pkg):
    p = pkg.abi.default_params()
    # black_hole.frag:19-39; max_revolutions keeps 2 (src/main.cpp:297 upload rejected)
    assert (p.max_steps, p.max_revolutions, p.crosshair, p.raytrace_type) == (100, 2, 0, 0)
    assert p.u_f == pytest.approx(0.01) and p.curved_percentage == 0.5 and p.percent_black == pytest.approx(0.75)
    t = pkg.abi.default_test_ray()
    assert t.visible == 0 and t.radius == pytest.approx(0.025) and t.extended_length == 1000.0
    assert list(t.curved_color) == [1, 0, 0, 1] and list(t.flat_color) == [0, 1, 0, 1]


def test_default_scene_packing_matches_object_loader(pkg):
    """objectLoader.cpp:27-109 on src/main.cpp:222-268."""
    s = pkg.abi.default_scene()
    objs = [(s.objects[i].type, s.objects[i].index, s.objects[i].material_index) for i in range(s.num_objects)]
    assert objs == [(0, 0, 1), (2, 0, 1), (3, 0, 1), (4, 0, 1), (5, 0, 1), (6, 0, 2)]
    # materials[0] is never written (matMap default-inserts 0 before size())
    assert bytes(memoryview(s.materials[0])) == bytes(C.sizeof(s.materials[0]))
    m1, m2 = s.materials[1], s.materials[2]
    assert (m1.texture_index, m2.texture_index) == (0, 1)
    assert list(m1.color) == [0.5, 0.0, 0.5, 1.0]
    assert (m1.ambient, m1.diffuse, m1.specular, m1.shininess) == pytest.approx((0.1, 0.9, 0.5, 32.0))
    assert m1.double_sided_normals == 1 and m1.flip_normals == 0
    assert s.num_lights == 1
    L = s.lights[0]
    assert list(L.transform.pos) == [10, 10, 10] and L.intensity == 8.0
    assert (L.attenuation_constant, L.attenuation_linear, L.attenuation_quadratic) == pytest.approx((1, 0.09, 0.032))
    assert list(s.spheres[0].transform.pos) == [-10, 0, 0] and s.spheres[0].radius == 1.0
    d = s.disks[0]
    assert list(d.plane.transform.pos) == [0, 0, -10] and d.radius == 2.0
    # toMat3(angleAxis(pi/4, normalize(1,1,1)))
    a = np.array(d.plane.transform.axes, dtype=np.float64).reshape(3, 3)  # rows = columns of the matrix
    k = np.ones(3) / math.sqrt(3)
    th = math.pi / 4
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    R = np.eye(3) + math.sin(th) * K + (1 - math.cos(th)) * K @ K
    assert np.allclose(a.T, R, atol=2e-7)
    hd = s.hollow_disks[0]
    assert (hd.inner_radius, hd.outer_radius) == (2.5, 5.0) and hd.plane.repeat_texture == 1
    cy = s.cylinders[0]
    assert list(cy.transform.pos) == [0, 10, 0] and (cy.height, cy.radius) == (5.0, 2.0)
    r = s.rectangles[0]
    assert list(r.plane.transform.pos) == [0, 0, 10] and (r.width, r.height) == (3.0, 2.0)
    b = s.boxes[0]
    assert list(b.transform.pos) == [10, 0, 0] and (b.width, b.depth, b.height) == (1.0, 1.0, 1.0)
    assert [list(s.texture_sizes[i]) for i in range(2)] == [[600, 600], [1601, 1201]]
    assert list(s.max_texture_size) == [1601, 1201]


def test_default_camera(pkg):
    """Camera(pos, -normalize(pos), (1,0,0)) — camera.cpp:7-11, src/main.cpp:222."""
    c = pkg.abi.default_camera()
    assert list(c.transform.pos) == [0, 2, 15] and c.fov == 90.0
    ax = np.array(c.transform.axes, dtype=np.float32).reshape(3, 3)
    f = -np.array([0, 2, 15], dtype=np.float32)
    f = f * np.float32(1.0 / np.sqrt(np.float32(229.0)))
    assert np.array_equal(ax[0], np.array([1, 0, 0], dtype=np.float32))
    assert np.allclose(ax[2], f, atol=1e-7)
    assert abs(float(np.dot(ax[1], ax[2]))) < 1e-6 and ax[1][1] > 0.99


def test_blocks_row_count(pkg):
    lib = pkg.abi.load()
    assert lib.sr_blocks_row_count(1080, 8, 0, 1) == 1080
    total = sum(lib.sr_blocks_row_count(1080, 8, r, 8) for r in range(8))
    assert total == 1080
    assert lib.sr_blocks_row_count(13, 8, 1, 2) == 5
    assert lib.sr_blocks_row_count(13, 8, 2, 2) == 0


@pytest.mark.parametrize("pos,fwd", [
    ((3.0, 2.0, 14.0), (-0.2, -0.1, -1.0)),
    ((0.0, 2.0, 15.0), (1.0, -2.0, -15.0)),
    ((0.0, 2.0, 15.0), (3.0, -2.0, -15.0)),
    ((20.0, -5.0, 7.0), (-1.0, 0.3, 0.1)),
])
def test_press_r_points_product_equals_oracle(pkg, oracle, pos, fwd):
    """The product's host press-R geodesic (C++) and the oracle's restatement
    (C) of src/main.cpp:94-124 agree bit for bit."""
    v = np.array(fwd, dtype=np.float32)
    v = v * np.float32(1.0 / np.sqrt(np.float32(np.dot(v, v))))
    for n in (100, 2000):
        a = np.array(pkg.abi.test_ray_points(pos, v.tolist(), n, 2), dtype=np.float32)
        b = np.array(oracle.test_ray_points(pos, v.tolist(), n, 2), dtype=np.float32)
        assert a.shape == b.shape and a.shape[0] >= 2
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_press_r_quirks(pkg, oracle):
    """src/main.cpp:104: an exactly radial ray returns {origin, origin + dir}.
    The radial test is `abs(int)` of the dot product, so it fires
    only at |dot| >= 1 exactly. The app's default camera normalizes the
    forward twice (src/main.cpp:222 and camera.cpp:9) and lands on dot == -1.0
    exactly -> radial. A forward normalized once gives dot = -0.99999994 ->
    not radial -> normalize(cross(n, d)) of a zero vector -> NaN points."""
    pts = pkg.abi.test_ray_points((0.0, 0.0, 15.0), (0.0, 0.0, -1.0), 2000, 2)
    assert pts == [(0.0, 0.0, 14.0), (0.0, 0.0, 13.0)]
    cam = pkg.abi.default_camera()
    pts = pkg.abi.test_ray_points(list(cam.transform.pos), list(cam.transform.axes[6:9]), 100, 2)
    assert len(pts) == 2
    once = [-0.0, np.float32(-0.13216372).item(), np.float32(-0.99122787).item()]
    pts = pkg.abi.test_ray_points((0.0, 2.0, 15.0), once, 100, 2)
    ref = oracle.test_ray_points((0.0, 2.0, 15.0), once, 100, 2)
    assert len(pts) == len(ref) == 101 and all(math.isnan(p[0]) for p in pts[1:])


# Reference outputs of the press-R loop itself (src/main.cpp:73-124 compiled
# in the survey container): points per ray at N = 2000
# from the default camera position for four directions, and the mean points
# per ray of the 1920x1080 / 2000-step per-pixel sweep (468.4).
@pytest.mark.parametrize("fwd,n_points", [
    ((0.5, -2.0, -15.0), 75),
    ((1.0, -2.0, -15.0), 155),
    ((3.0, -2.0, -15.0), 759),
    ((6.0, -2.0, -15.0), 515),
])
def test_press_r_pinned_to_reference_outputs(pkg, oracle, fwd, n_points):
    v = np.array(fwd, dtype=np.float32)
    v = v * np.float32(1.0 / np.sqrt(np.float32(np.dot(v, v))))
    assert len(pkg.abi.test_ray_points((0.0, 2.0, 15.0), v.tolist(), 2000, 2)) == n_points
    assert len(oracle.test_ray_points((0.0, 2.0, 15.0), v.tolist(), 2000, 2)) == n_points


def test_press_r_sweep_mean_points_pinned(pkg, oracle):
    """the reference's loop swept over the headline frame's
    camera rays returns 468.4 points per ray on average."""
    n = oracle.pressr_sweep(pkg.abi.default_camera(), 1920, 1080, 2000, 2, 0, 1080, 0)
    assert abs(n / (1920 * 1080) - 468.4) < 0.05, n / (1920 * 1080)


def test_reference_assets_ingest_layout(pkg):
    """assets/textures decoded as the app loads them (src/main.cpp:205-218,
    image_utils.cpp:7-117): vertical flip (row 0 = bottom), RGB skybox, the
    array padded to 1601x1201 RGBA with alpha 255 inside the RGB layer."""
    A = pkg.assets
    if not A.available():
        pytest.skip("assets/textures missing")
    from PIL import Image

    bg = A.skybox("2k")
    assert bg.shape == (1024, 2048, 3) and bg.dtype == np.uint8
    with Image.open(A.SKYBOX["2k"]) as im:
        top = np.asarray(im.convert("RGB"))[0]
    assert np.array_equal(bg[-1], top)  # flipped: the picture's top row is the last row
    arr, sizes, mx = A.texture_array()
    assert arr.shape == (2, 1201, 1601, 4) and sizes == [(600, 600), (1601, 1201)] and mx == (1601, 1201)
    assert (arr[0, :600, :600, 3] == 255).all() and (arr[0, 600:, :, :] == 0).all() and (arr[0, :, 600:] == 0).all()
    scene = pkg.abi.default_scene()
    assert [tuple(scene.texture_sizes[i]) for i in range(2)] == [(600.0, 600.0), (1601.0, 1201.0)]


def test_flyby_camera_follows_the_hyperbola(pkg):
    """sr_camera_hyperbolic_trajectory (camera.cpp:20-39): starts on the +z axis
    at the initial distance, passes the closest distance at t = 0.5, looks at
    the origin, keeps the fov."""
    abi = pkg.abi
    c0, c5, c1 = abi.camera_flyby(0.0), abi.camera_flyby(0.5), abi.camera_flyby(1.0)
    p0, p5, p1 = (np.array(c.transform.pos[:3], dtype=np.float64) for c in (c0, c5, c1))
    assert abs(np.linalg.norm(p0) - 30.0) < 1e-3 and p0[2] > 29.99
    assert abs(np.linalg.norm(p5) - 10.0) < 1e-3 and abs(p1[2] + 30.0) < 1e-3
    for c, p in ((c0, p0), (c5, p5), (c1, p1)):
        fwd = np.array(c.transform.axes[6:9], dtype=np.float64)
        assert np.allclose(fwd, -p / np.linalg.norm(p), atol=1e-5) and c.fov == 90.0


def test_write_png_round_trip(pkg, tmp_path):
    """sr_write_png (presentation): the PNG decodes (PIL) to the frame with
    its bottom-up rows flipped, every filter path exercised by random, flat and
    gradient rows; bad arguments and unwritable paths are rejected."""
    PIL = pytest.importorskip("PIL.Image")
    abi = pkg.abi
    rng = np.random.default_rng(3)
    h, w = 37, 53
    frame = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
    frame[5:9] = 7  # flat rows
    frame[10:20] = (np.arange(w)[None, :, None] * 3 + np.arange(10)[:, None, None]).astype(np.uint8)
    for flip in (True, False):
        path = tmp_path / f"f{int(flip)}.png"
        abi.write_png(path, frame, flip_rows=flip)
        got = np.asarray(PIL.open(path).convert("RGBA"))
        assert np.array_equal(got, frame[::-1] if flip else frame)
    lib = abi.load()
    buf = np.zeros((4, 4, 4), np.uint8)
    assert lib.sr_write_png(None, buf.ctypes.data, 4, 4, 16, 1) == abi.SR_E_INVALID
    assert lib.sr_write_png(b"x.png", buf.ctypes.data, 4, 4, 8, 1) == abi.SR_E_INVALID  # pitch < 4 w
    assert lib.sr_write_png(str(tmp_path / "no" / "dir.png").encode(), buf.ctypes.data, 4, 4, 16, 1) == abi.SR_E_IO
    assert lib.sr_status_string(abi.SR_E_IO) == b"file write failed"
