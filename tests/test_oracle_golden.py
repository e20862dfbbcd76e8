"""Pins the CPU oracle to the reference itself: golden RGBA8 frames rendered
by the reference fragment shader (assets/shaders/black_hole.frag) on
SwiftShader 4.1 (tests/golden/make_golden.py).

Tolerance budget. SwiftShader's texture filter, sin/atan/asin
and interpolation of `uv` are one valid GL implementation, not bit-defined:
  - untextured scenes:   >= 99.9 % of pixels within 2/255 per channel and
                          every pixel within 4/255, except the named pixel
                          counts of ALLOW_GT4 (measured, exact: a regression
                          elsewhere cannot hide in them). The far-camera
                          reseed goldens (SURVEY §7 hard part 1: rays that
                          orbit the photon ring for hundreds of steps leave in
                          a direction that differs in the last bits and may
                          cross a skybox checker edge; 1-4 pixels); the
                          headline-size band of rows 704-719 (one pixel of
                          30,720, 5/255 after 1,237 equal steps); features_low
                          (a ray through several translucent surfaces sums
                          several of SwiftShader's fixed-point filter results:
                          one pixel, 5/255, equal step counts). Executed step
                          counts equal on >= 99.9 % of pixels;
  - textured scenes:     SwiftShader samples RGBA8 in 16-bit fixed point, so an
                          opaque texel reads alpha 65527..65531/65535 < 1 and
                          the ray does not stop at textured objects
                          (frag:932 `alpha == 1.`); the oracle's LERP filter
                          reads exactly 1.0 like hardware TMUs. Pinned on the
                          pixels whose ray never stops at a textured object
                          (equal step counts): same budget as above;
  - noise mask:          rand() = fract(sin(x) * 43758.5453) amplifies sin's
                          last-bit differences (frag:839-841): the masked
                          fraction must agree within 2 %, unmasked pixels match
                          within the untextured budget.
"""
from pathlib import Path

import numpy as np
import pytest

from conftest import case_rows, case_texture_kind, load_case, texture_array_of

UNTEXTURED = ["bh_default", "scene_untex", "mode_half_width", "mode_half_height", "crosshair", "steps_100",
              "test_ray"] + [f"rand_{i}" for i in range(1, 9)]
TEXTURED = ["scene_tex", "scene_tex_weighted", "scene_tex_2000", "mode_flat"]
# golden_r2.npz: the u < u_f reseed branch (frag:891-912) from cameras beyond
# r = 1/u_f = 100 and with u_f = 0.1 / 0.05, BASELINE config 2 at full size,
# and the material-flag scene (planes, normal maps, uv flags, single-sided,
# flipped and translucent materials, 4 lights; scenes.scene_features) whose
# textures are translucent everywhere, so the untextured budget applies.
RESEED = ["reseed_r120", "reseed_r300", "reseed_side", "reseed_uf01", "reseed_uf005_far"]
FEATURES = ["features_default", "features_oblique", "features_low", "features_below", "features_flat"]
R2_BUDGET = RESEED + ["config2_640x360"] + FEATURES
# golden_r3.npz: 16-row bands of the headline frame (1920x1080 / 2000 steps:
# rows 704-719, the photon-ring waves of the critical path, and 536-551,
# through the black hole) and of config 4 (3840x2160 / 4000 steps), rendered
# at full frame size under a scissor rectangle
BANDS_UNTEX = ["band1080_704_untex", "band1080_536_untex", "band2160_1408_untex"]
BANDS_TEX = ["band1080_704_tex", "band1080_536_tex"]
# The only pixels allowed beyond 4/255, by case (every other case: none). The
# counts are what the oracle gives against SwiftShader today; each is
# explained in the module docstring.
ALLOW_GT4 = {"reseed_r120": 4, "reseed_r300": 2, "reseed_side": 1, "features_low": 1, "band1080_704_untex": 1,
             "band1080_704_tex": 1}
# with the oracle's SwiftShader filter mode, on every pixel of the textured
# cases: two photon-ring rays each (1,674 steps in scene_tex_2000, rows 117;
# 1,618 vs SwiftShader's 1,617 steps in band1080_704_tex, row 706), the
# untextured allowance's kind (band1080_704_untex)
ALLOW_GT4_SS = {"scene_tex_2000": 2, "band1080_704_tex": 2}
# float FragColor pixels allowed at >= 0.02 from SwiftShader's, by case
ALLOW_F32 = {"reseed_r120": 2}


@pytest.fixture(scope="module")
def tex(oracle, textures):
    bg, arr = textures
    return oracle.TextureSet(bg, arr)


def run(pkg, oracle, golden, tex, name):
    if name + "/scene" not in golden:
        pytest.skip(f"{name}: golden missing (python tests/golden/make_golden.py --set r3)")
    scene, cam, params, tr, w, h = load_case(pkg, golden, name)
    kind = case_texture_kind(golden, name)
    if kind != "default":
        tex = oracle.TextureSet(tex.bg, texture_array_of(pkg, kind))
    if name + "/rgba8" not in golden:
        pytest.skip(f"{name}: golden missing (python tests/golden/make_golden.py --set r3)")
    y0, y1 = case_rows(golden, name, h)
    rgba8, rgba32, steps = oracle.render(scene, cam, params, w, h, tex, tr, y0, y1)
    return rgba8, rgba32, steps, golden[name + "/rgba8"]


def test_goldens_come_from_swiftshader(golden, golden_cases):
    for part in golden.parts:
        assert b"SwiftShader" in bytes(part["meta_renderer"])
    assert set(UNTEXTURED + TEXTURED + R2_BUDGET + ["noise_mask"]) <= set(golden_cases)


def test_reseed_goldens_take_the_branch(pkg, golden):
    """The reseed goldens really start beyond r = 1/u_f (every curved ray
    reseeds at step 0, frag:891-912): camera radius > 1/u_f."""
    import numpy as np

    for name in RESEED:
        _, cam, params, _, _, _ = load_case(pkg, golden, name)
        r = float(np.linalg.norm(np.array(cam.transform.pos[:3], dtype=np.float64)))
        assert r > 1.0 / params.u_f, (name, r, params.u_f)


@pytest.mark.parametrize("name", UNTEXTURED + R2_BUDGET + BANDS_UNTEX)
def test_untextured_within_budget(pkg, oracle, golden, tex, name):
    rgba8, _, steps, ref = run(pkg, oracle, golden, tex, name)
    d = np.abs(rgba8.astype(int) - ref.astype(int)).max(-1)
    assert np.mean(d <= 2) >= 0.999, (name, np.mean(d <= 2))
    # ring rays, far cameras, stacked translucent lookups: the named pixels only (docstring)
    assert int((d > 4).sum()) <= ALLOW_GT4.get(name, 0), (name, int((d > 4).sum()), d.max())
    if name + "/steps" in golden:
        assert np.mean(golden[name + "/steps"].astype(int) == steps) >= 0.999


@pytest.mark.parametrize("name", ["bh_default", "scene_untex", "reseed_r120", "reseed_uf01", "features_default"])
def test_float_fragcolor(pkg, oracle, golden, tex, name):
    """Unclamped FragColor from a float render target: median |diff| tiny,
    within the 8-bit texture quantum of SwiftShader's filter except on the
    chaotic photon-ring pixels of the RGBA8 budget (<= 0.05 %)."""
    _, rgba32, _, _ = run(pkg, oracle, golden, tex, name)
    ref = golden[name + "/rgba32"]
    d = np.abs(rgba32 - ref)
    assert np.median(d) < 2e-4
    assert int((d.max(-1) >= 0.02).sum()) <= ALLOW_F32.get(name, 0), (name, int((d.max(-1) >= 0.02).sum()), d.max())


@pytest.mark.parametrize("name", TEXTURED + BANDS_TEX)
def test_textured_pinned_where_alpha_semantics_agree(pkg, oracle, golden, tex, name):
    rgba8, _, steps, ref = run(pkg, oracle, golden, tex, name)
    d = np.abs(rgba8.astype(int) - ref.astype(int)).max(-1)
    if name + "/steps" in golden:
        same = golden[name + "/steps"].astype(int) == steps
    else:  # the scene_tex step map is the same for every frame of that camera at this size
        same = d <= 4
    # the headline bands cross the textured box / sphere / disk more often than
    # the small frames: more rays SwiftShader lets through (alpha < 1)
    assert same.mean() >= (0.6 if name in BANDS_TEX else 0.75), same.mean()
    assert np.mean(d[same] <= 2) >= 0.999
    # photon-ring rays of the untextured allowance (named pixels only)
    assert int((d[same] > 4).sum()) <= ALLOW_GT4.get(name, 0), (name, int((d[same] > 4).sum()))


def test_noise_mask_statistics(pkg, oracle, golden, tex):
    rgba8, _, _, ref = run(pkg, oracle, golden, tex, "noise_mask")
    black_o = (rgba8[..., :3] == 0).all(-1) & (rgba8[..., 3] == 0)
    black_r = (ref[..., :3] == 0).all(-1) & (ref[..., 3] == 0)
    assert abs(black_o.mean() - black_r.mean()) < 0.02
    both = ~black_o & ~black_r
    d = np.abs(rgba8.astype(int) - ref.astype(int)).max(-1)
    assert np.mean(d[both] <= 2) >= 0.999


SS_FILTER = Path(__file__).resolve().parent / "golden" / "ss_filter.npz"


def test_swiftshader_filter_model_bit_exact(oracle):
    """The oracle's SRO_FILTER_SWIFTSHADER sampler (sr_oracle.c
    sample_swiftshader: 0.16 fixed-point coordinates, UNORM16 texels and
    MulHigh weights) returns what SwiftShader's texture() returned, bit for
    bit, on every sample of tests/golden/ss_filter.npz (random RGBA8 arrays
    and RGB8 2D textures, POT and NPOT, coordinates beyond [0, 1]:
    tests/golden/probe_swiftshader_filter.py)."""
    if not SS_FILTER.exists():
        pytest.skip("tests/golden/ss_filter.npz missing (python tests/golden/probe_swiftshader_filter.py)")
    z = np.load(SS_FILTER)
    cases = bytes(z["meta_cases"]).decode().split("\n")
    assert b"SwiftShader" in bytes(z["meta_renderer"]) and len(cases) == 5
    for name in cases:
        tex, u, v, lay, out = (z[f"{name}/{k}"] for k in ("tex", "u", "v", "layer", "out"))
        got = np.stack([oracle.sample_texture(tex[int(lay[i])] if tex.ndim == 4 else tex, u[i], v[i],
                                              oracle.FILTER_SWIFTSHADER) for i in range(len(u))])
        assert np.array_equal(got.view(np.uint32), out.view(np.uint32)), (name, int((got != out).any(-1).sum()))
        # the LERP filter (the library's) differs from it: opaque texels read 1.0 there
        if tex.shape[-1] == 4:
            lerp = oracle.sample_texture(tex[int(lay[0])], u[0], v[0], 0)
            assert lerp.dtype == np.float32


@pytest.mark.parametrize("name", TEXTURED + BANDS_TEX)
def test_textured_all_pixels_with_swiftshader_filter(pkg, oracle, golden, tex, name):
    """T1 (frag:932, image_utils.cpp:12-18): with SwiftShader's own filter
    (SRO_FILTER_SWIFTSHADER) the oracle matches the textured goldens on EVERY
    pixel within the untextured budget, rays stopping at textured objects
    included: alpha semantics (SwiftShader's opaque texels read < 1, so its
    rays never stop there) are the only difference between the LERP-filter
    oracle, which the library matches bit for bit, and the reference run on
    SwiftShader."""
    if name + "/scene" not in golden:
        pytest.skip(f"{name}: golden missing")
    scene, cam, params, tr, w, h = load_case(pkg, golden, name)
    kind = case_texture_kind(golden, name)
    t = oracle.TextureSet(tex.bg, texture_array_of(pkg, kind)) if kind != "default" else tex
    params.filter_mode = oracle.FILTER_SWIFTSHADER
    y0, y1 = case_rows(golden, name, h)
    rgba8, _, steps = oracle.render(scene, cam, params, w, h, t, tr, y0, y1)
    ref = golden[name + "/rgba8"]
    d = np.abs(rgba8.astype(int) - ref.astype(int)).max(-1)
    assert np.mean(d <= 2) >= 0.999, (name, np.mean(d <= 2))
    assert int((d > 4).sum()) <= ALLOW_GT4_SS.get(name, 0), (name, int((d > 4).sum()), d.max())
    if name + "/steps" in golden:
        assert np.mean(golden[name + "/steps"].astype(int) == steps) >= 0.999
