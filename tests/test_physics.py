"""Known-answer physics checks of the Binet/RK4 integrator: the
reference has no tests, so these pin the integrator to Schwarzschild optics
(r_s = 1). They run on the oracle's restatements and on the product's host
press-R geodesic; tests/test_gpu_physics.py repeats the capture check on the
kernel.

  - photon capture iff impact parameter b < 3*sqrt(3)/2 (photon sphere r = 1.5)
  - weak-field deflection  delta = 2/b + 15 pi/(16 b^2) + 16/(3 b^3) + O(b^-4)
  - the orbit invariant (u')^2 + u^2 - u^3 = 1/b^2 along the integration
"""
import math

import numpy as np
import pytest

B_CRIT = 1.5 * math.sqrt(3.0)


def one_pixel(pkg, b, r0=60.0):
    """Camera at distance ~r0 whose 1x1 frame's only ray (uv = 0) has impact
    parameter b w.r.t. the hole; black-hole-only scene, flat grey skybox."""
    sc, abi = pkg.scenes, pkg.abi
    pos = np.array([r0, 0.0, b], dtype=np.float32)
    cam = sc.camera_look(pos, (-1.0, 0.0, 0.0), right=(0.0, 0.0, -1.0), fov=60.0)
    return cam


@pytest.mark.parametrize("b,captured", [(2.0, True), (2.45, True), (2.55, True), (2.65, False), (3.0, False),
                                        (6.0, False)])
def test_capture_threshold(pkg, oracle, b, captured):
    sc, abi = pkg.scenes, pkg.abi
    cam = one_pixel(pkg, b)
    scene = sc.scene_black_hole_only()
    bg = np.full((8, 16, 3), 200, dtype=np.uint8)
    params = abi.default_params(max_steps=4000, percent_black=-1.0)
    rgba8, _, steps = oracle.render(scene, cam, params, 1, 1, oracle.TextureSet(bg, None))
    px = rgba8[0, 0]
    if captured:
        assert list(px) == [0, 0, 0, 255], (b, px)
    else:
        assert list(px) == [200, 200, 200, 255], (b, px)


def deflection(points, origin, direction, b):
    """Angle at which u = 1/r reaches 0 (linear extrapolation of the last two
    points), minus the straight-line value pi - asin(b / r0)."""
    o = np.array(origin, dtype=np.float64)
    d = np.array(direction, dtype=np.float64)
    n = o / np.linalg.norm(o)
    t = np.cross(np.cross(n, d), n)
    t /= np.linalg.norm(t)
    p = np.array(points, dtype=np.float64)
    phi = np.unwrap(np.arctan2(p @ t, p @ n))
    u = 1.0 / np.linalg.norm(p, axis=1)
    # last two points before u changes sign
    u1, u2, f1, f2 = u[-2], u[-1], phi[-2], phi[-1]
    phi_inf = f2 + (f2 - f1) * u2 / (u1 - u2)
    r0 = np.linalg.norm(o)
    return phi_inf - (math.pi - math.asin(b / r0)), phi, u


@pytest.mark.parametrize("impl", ["oracle", "product"])
@pytest.mark.parametrize("b", [15.0, 30.0, 60.0])
def test_weak_field_deflection(pkg, oracle, impl, b):
    X = 3000.0
    origin = (X, 0.0, b)
    direction = (-1.0, 0.0, 0.0)
    # press-R starts at pos + dir (TEST_RAY_OFFSET = 1)
    pos = (X + 1.0, 0.0, b)
    fn = oracle.test_ray_points if impl == "oracle" else pkg.abi.test_ray_points
    pts = fn(pos, direction, 8000, 2)
    assert len(pts) > 100
    delta, phi, u = deflection(pts, origin, direction, b)
    # delta = 4M/b + (15 pi/4)(M/b)^2 + (128/3)(M/b)^3 + O((M/b)^4), M = r_s/2 = 1/2
    m = 0.5 / b
    expect = 4 * m + 15 * math.pi / 4 * m ** 2 + 128.0 / 3.0 * m ** 3
    tol = 3465 * math.pi / 64 * m ** 4 + 1.5e-4
    assert abs(delta - expect) < tol, (b, delta, expect)


@pytest.mark.parametrize("b", [3.5, 8.0, 25.0])
def test_orbit_invariant(oracle, b):
    """E = (du/dphi)^2 + u^2 - u^3 is constant (= 1/b^2) along the RK4 orbit;
    du/dphi by central differences of the integrated points."""
    X = 400.0
    pts = oracle.test_ray_points((X + 1.0, 0.0, b), (-1.0, 0.0, 0.0), 8000, 2)
    p = np.array(pts, dtype=np.float64)
    o = np.array([X, 0.0, b])
    d = np.array([-1.0, 0.0, 0.0])
    n = o / np.linalg.norm(o)
    t = np.cross(np.cross(n, d), n)
    t /= np.linalg.norm(t)
    phi = np.unwrap(np.arctan2(p @ t, p @ n))
    u = 1.0 / np.linalg.norm(p, axis=1)
    du = (u[2:] - u[:-2]) / (phi[2:] - phi[:-2])
    E = du ** 2 + u[1:-1] ** 2 - u[1:-1] ** 3
    E0 = 1.0 / b ** 2
    # points near the ends (u ~ 0) are excluded from the relative check by weighting
    rel = np.abs(E - E0) / E0
    assert np.median(rel) < 2e-3, (b, np.median(rel))
    assert np.max(rel[len(rel) // 10: -len(rel) // 10]) < 2e-2
