"""The premises of the low-energy exclusions (geodesic.hip SR_XCYL /
SR_XPERI, sr_api.cpp clear_radius / xlow_need / xperi_e), checked on the
same integrator arithmetic as the kernel's: binary32 RK4 of u'' = -u + 1.5 u^2
with the step angle 2 * max_revolutions * pi / max_steps (the kernel's
operation order differs; the bounds carry margins far above binary32
rounding).

For an orbit starting at u < 0.6 with E = u'^2 + u^2 (1 - u) <= SR_XCYL_EMAX:
  - u stays at or below u_t(E), the root of u^2 (1 - u) = E under 2/3
    (the periapsis the SR_XPERI threshold E <= f(w) (1 - 1e-3) - 1e-6 relies on);
  - one step changes u by at most kappa = sqrt(EMAX) 1.02 dphi 1.001 +
    dphi^2 / 12 1.02 + 1e-6 (the host's bound on a chord's far end);
  - E drifts by far less than the 2 % the bound allows.
Pure numpy, no GPU."""
import numpy as np
import pytest

EMAX = 0.14  # device_scene.h SR_XCYL_EMAX


def f(u):
    return u * u * (1.0 - u)


def u_turn(E):
    """The root of u^2 (1 - u) = E below 2/3 (f increases on [0, 2/3])."""
    lo, hi = 0.0, 2.0 / 3.0
    for _ in range(80):
        mid = 0.5 * (lo + hi)
        lo, hi = (mid, hi) if f(mid) < E else (lo, mid)
    return hi


def rk4_orbits(u0, du0, dphi, steps):
    """binary32 RK4 of u'' = -u + 1.5 u^2 over a batch of orbits."""
    f32 = np.float32
    u = u0.astype(f32)
    du = du0.astype(f32)
    h = f32(dphi)
    half = f32(0.5)
    us = [u.copy()]
    for _ in range(steps):
        def acc(x):
            return -x + f32(1.5) * x * x
        k1 = acc(u)
        u2 = u + half * h * du
        k2 = acc(u2)
        u3 = u2 + f32(0.25) * h * h * k1
        k3 = acc(u3)
        u4 = u + h * du + half * h * h * k2
        k4 = acc(u4)
        un = u + h * du + h * h / f32(6.0) * (k1 + k2 + k3)
        dun = du + h / f32(6.0) * (k1 + f32(2.0) * k2 + f32(2.0) * k3 + k4)
        u, du = un.astype(f32), dun.astype(f32)
        us.append(u.copy())
        if not np.any(u > f32(0.005)):
            break
    return np.stack(us), u, du


@pytest.mark.parametrize("max_steps", [600, 1000, 2000, 4000])
def test_low_energy_orbits_respect_the_step_and_periapsis_bounds(max_steps):
    dphi = 2 * 2 * np.pi / max_steps  # two revolutions (the default)
    rng = np.random.default_rng(max_steps)
    n = 4000
    E = rng.uniform(1e-4, EMAX, n)
    ut = np.array([u_turn(e) for e in E])
    u0 = rng.uniform(0.0, 1.0, n) * np.minimum(ut, 0.6)
    u0 = np.maximum(u0, 0.006)
    ok = f(u0) <= E
    E, ut, u0 = E[ok], ut[ok], u0[ok]
    du0 = np.sqrt(E - f(u0)) * np.where(rng.uniform(size=u0.size) < 0.5, -1.0, 1.0)
    us, u_end, du_end = rk4_orbits(u0, du0, dphi, max_steps)
    us = us.astype(np.float64)
    alive = us > 0.005  # the orbit ends (u < u_f) once u falls below it
    # periapsis: u never passes u_t(E) by more than the rounding
    assert np.all(np.where(alive, us, 0.0) <= ut * (1 + 1e-4) + 1e-6)
    # step bound: |u_{i+1} - u_i| <= kappa while the orbit runs
    d = np.abs(np.diff(us, axis=0))
    run = alive[:-1]
    assert run.sum() > 100 * u0.size  # the orbits ran for many steps
    kappa = np.sqrt(EMAX) * 1.02 * dphi * 1.001 + dphi * dphi / 12.0 * 1.02 + 1e-6
    assert np.all(np.where(run, d, 0.0) <= kappa)
    # energy drift along the run (orbits still inside u_f's sphere)
    live = u_end.astype(np.float64) > 0.005
    E_end = du_end.astype(np.float64) ** 2 + f(u_end.astype(np.float64))
    if np.any(live):
        assert np.max(np.abs(E_end[live] - E[live]) / E[live]) < 2e-3


def test_periapsis_threshold_implies_the_radius():
    """xperi_e's E <= f(w) (1 - 1e-3) - 1e-6 puts u_t(E) below w, so the orbit
    stays beyond 1 / w (the object's clearing radius, x 1.001)."""
    for w in np.linspace(0.02, 0.66, 200):
        e = min(f(w) * (1 - 1e-3) - 1e-6, EMAX)
        if e <= 0:
            continue
        assert u_turn(e) <= w
