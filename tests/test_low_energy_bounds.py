"""The premises of the low-energy exclusions (geodesic.hip SR_XCYL /
SR_XPERI, sr_api.cpp clear_radius / xlow_need / xperi_e), checked on the
kernel's own integrator arithmetic over every step angle the exclusions are
enabled for (sr_api.cpp clear_radius: max_dphi <= SR_XLOW_DPHI_MAX = 0.2,
device_scene.h): the host's 16-byte step table in binary32 (sr_api.cpp
ensure_table: step_i = (max_angle - phi) / (N - i), frag:914-915) and
geodesic.hip rk4_step's binary32 operation order (fma(0.5, q h, a) half
steps, fma(2, k3, fma(2, k2, k1)) sums; every fma here adds an exact product,
so the numpy float32 expressions below round exactly as the kernel does).

For an orbit starting at u < 0.6 with E = u'^2 + u^2 (1 - u) <= SR_XCYL_EMAX:
  - u never passes u_t((E + 1e-6) / (1 - 1e-3)), the root of u^2 (1 - u) = .
    under 2/3: exactly what SR_XPERI's threshold E <= f(w) (1 - 1e-3) - 1e-6
    needs for the orbit to stay at u <= w;
  - one step changes u by at most kappa = sqrt(EMAX) 1.02 d + d^2 / 12 1.02 +
    1e-6 with d = max_dphi 1.001 (the host's bound on a chord's far end), and
    every table step is at most d;
  - E drifts by less than 2e-3 relative (the bound allows 2 %).
The cases are the schedules the ABI runs with the exclusions on: the app's
MAX_STEPS 100 (src/main.cpp:68) at one to three revolutions (0.063 ... 0.19
rad), 95 steps at three revolutions (0.198, just under the cap), and 300 ...
8000 steps (config 5). Orbits start at step 0 and at three quarters of the
table (a reseed starts a new orbit mid-table). Pure numpy, no GPU."""
import numpy as np
import pytest

EMAX = np.float32(0.14)  # device_scene.h SR_XCYL_EMAX
DPHI_CAP = np.float32(0.2)  # device_scene.h SR_XLOW_DPHI_MAX
PI = np.float32(3.1415926535)  # sr_api.cpp kPi (the shader's PI, frag:860)
f32 = np.float32


def f(u):
    return u * u * (1.0 - u)


def u_turn(E):
    """The root of u^2 (1 - u) = E below 2/3 (f increases on [0, 2/3]); vectorised."""
    E = np.asarray(E, dtype=np.float64)
    lo, hi = np.zeros_like(E), np.full_like(E, 2.0 / 3.0)
    for _ in range(80):
        mid = 0.5 * (lo + hi)
        below = f(mid) < E
        lo, hi = np.where(below, mid, lo), np.where(below, hi, mid)
    return hi


def step_table(max_steps: int, max_revs: int) -> np.ndarray:
    """sr_api.cpp ensure_table's step sizes, binary32 (cos / sin not needed)."""
    max_angle = f32(2.0) * f32(max_revs) * PI
    phi = f32(0.0)
    h = np.empty(max_steps, dtype=f32)
    for i in range(max_steps):
        step = f32(f32(max_angle - phi) / f32(max_steps - i))
        phi = f32(phi + step)
        h[i] = step
    return h


def max_dphi(max_steps: int, max_revs: int) -> float:
    """sr_api.cpp build_frame's out_dip and max_dphi."""
    max_angle = float(f32(2.0) * f32(max_revs) * PI)
    dphi = max_angle / max_steps
    out_dip = f32(1.0 - dphi * dphi / 8.0 - 1e-6)
    return float(np.nextafter(f32(np.sqrt(8.0 * (1.0 - float(out_dip)))), f32(np.inf)))


def ddu(u):
    return -u * (f32(1.0) - f32(1.5) * u)


def rk4_step(u, du, h, h6):
    """geodesic.hip rk4_step, bit for bit in binary32."""
    half = f32(0.5)
    k1 = du
    l1 = ddu(u)
    k2 = du + half * (l1 * h)
    l2 = ddu(u + half * (k1 * h))
    k3 = du + half * (l2 * h)
    l3 = ddu(u + half * (k2 * h))
    k4 = du + l3 * h
    l4 = ddu(u + k3 * h)
    un = u + h6 * ((k1 + f32(2.0) * k2 + f32(2.0) * k3) + k4)
    dun = du + h6 * ((l1 + f32(2.0) * l2 + f32(2.0) * l3) + l4)
    return un, dun


def low_energy_starts(rng, n):
    E = rng.uniform(1e-4, float(EMAX), n)
    ut = u_turn(E)
    u0 = np.maximum(rng.uniform(0.0, 1.0, n) * np.minimum(ut, 0.6), 0.006)
    ok = f(u0) <= E
    E, u0 = E[ok], u0[ok]
    du0 = np.sqrt(E - f(u0)) * np.where(rng.uniform(size=u0.size) < 0.5, -1.0, 1.0)
    u0, du0 = u0.astype(f32), du0.astype(f32)
    # the kernel's own E of the binary32 start state (geodesic.hip orbit_e:
    # fma(du, du, u u (1 - u)); du^2 is exact in binary64)
    E32 = (du0.astype(np.float64) ** 2 + (u0 * u0 * (f32(1.0) - u0)).astype(np.float64)).astype(f32)
    keep = (u0 < f32(0.6)) & (E32 <= EMAX)
    return u0[keep], du0[keep], E32[keep].astype(np.float64)


CASES = [(100, 1), (100, 2), (100, 3), (95, 3), (300, 2), (300, 3), (600, 2), (1000, 1), (1000, 2),
         (2000, 2), (2000, 3), (4000, 2), (8000, 2)]


@pytest.mark.parametrize("max_steps,max_revs", CASES)
def test_low_energy_orbits_respect_the_step_and_periapsis_bounds(max_steps, max_revs):
    md = max_dphi(max_steps, max_revs)
    assert md <= DPHI_CAP, "a case beyond the cap tests nothing the library runs"
    h = step_table(max_steps, max_revs)
    d = md * 1.001
    assert np.all(np.abs(h.astype(np.float64)) <= d), "every table step within the host's d"
    kappa = np.sqrt(float(EMAX)) * 1.02 * d + d * d / 12.0 * 1.02 + 1e-6
    rng = np.random.default_rng(max_steps * 10 + max_revs)
    for start in (0, (3 * max_steps) // 4):
        u, du, E0 = low_energy_starts(rng, 3000)
        cap = u_turn((E0 + 1e-6) / (1.0 - 1e-3))  # SR_XPERI's premise: u stays <= u_t of this
        alive = np.ones(u.size, dtype=bool)
        steps_run = 0
        for i in range(start, max_steps):
            hi = h[i]
            un, dun = rk4_step(u, du, hi, f32(hi / f32(6.0)))
            run = alive & (u > f32(0.005))  # the orbit ends (u < u_f) once u falls below it
            if not run.any():
                break
            steps_run += int(run.sum())
            d_u = np.abs(un.astype(np.float64) - u.astype(np.float64))
            assert np.all(np.where(run, d_u, 0.0) <= kappa), f"step {i}: |du| {d_u[run].max()} > kappa {kappa}"
            assert np.all(np.where(run, un.astype(np.float64), 0.0) <= cap), f"step {i}: u past the periapsis bound"
            alive = run
            u, du = un, dun
        assert steps_run > 0.1 * (max_steps - start) * u.size  # the orbits ran for many steps
        live = alive & (u > f32(0.005))
        if np.any(live):
            E_end = du.astype(np.float64) ** 2 + f(u.astype(np.float64))
            assert np.max(np.abs(E_end[live] - E0[live]) / E0[live]) < 2e-3


def test_step_angle_cap_matches_the_library():
    """The cap the test proves is the one the library applies (device_scene.h)."""
    from pathlib import Path
    import re

    h = (Path(__file__).resolve().parent.parent / "schwarzschild-raytracer_amd" / "csrc" / "device_scene.h").read_text()
    m = re.search(r"#define SR_XLOW_DPHI_MAX ([0-9.]+)f", h)
    assert m and f32(float(m.group(1))) == DPHI_CAP
    api = (Path(__file__).resolve().parent.parent / "schwarzschild-raytracer_amd" / "csrc" / "sr_api.cpp").read_text()
    assert "max_dphi <= SR_XLOW_DPHI_MAX" in api
    # schedules just beyond the cap are excluded from the proof and from the library
    assert max_dphi(94, 3) > DPHI_CAP and max_dphi(95, 3) <= DPHI_CAP


def test_periapsis_threshold_implies_the_radius():
    """xperi_e's E <= f(w) (1 - 1e-3) - 1e-6 puts u_t((E + 1e-6) / (1 - 1e-3))
    at or below w, so the orbit stays beyond 1 / w (the object's clearing
    radius, x 1.001)."""
    for w in np.linspace(0.02, 0.66, 200):
        e = min(f(w) * (1 - 1e-3) - 1e-6, float(EMAX))
        if e <= 0:
            continue
        assert u_turn((e + 1e-6) / (1 - 1e-3)) <= w * (1 + 1e-12)
