import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

import srpkg  # noqa: E402

GOLDEN = ROOT / "tests" / "golden" / "golden.npz"
GOLDEN_R2 = ROOT / "tests" / "golden" / "golden_r2.npz"  # reseed, config 2, material flags
GOLDEN_R3 = ROOT / "tests" / "golden" / "golden_r3.npz"  # bands of the headline-size frames


class Golden:
    """The golden fixture files as one mapping (case keys are unique across
    files; meta_cases is the concatenation of their case lists)."""

    def __init__(self, paths):
        self.parts = [np.load(p) for p in paths]

    def __contains__(self, key):
        return any(key in p for p in self.parts)

    def __getitem__(self, key):
        for p in self.parts:
            if key in p:
                return p[key]
        raise KeyError(key)

    def cases(self):
        out = []
        for p in self.parts:
            out += bytes(p["meta_cases"]).decode().split("\n")
        return out


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); runs the gfx950 kernel")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def pkg():
    return srpkg.load_package()


@pytest.fixture(scope="session")
def oracle():
    return srpkg.load_oracle()


@pytest.fixture(scope="session")
def golden():
    if not GOLDEN.exists() or not GOLDEN_R2.exists():
        pytest.skip("golden fixtures missing (python tests/golden/make_golden.py [--set r2])")
    return Golden([GOLDEN, GOLDEN_R2] + ([GOLDEN_R3] if GOLDEN_R3.exists() else []))


@pytest.fixture(scope="session")
def golden_cases(golden):
    return golden.cases()


@pytest.fixture(scope="session")
def textures(pkg, golden):
    sc = pkg.scenes
    h, w = (int(v) for v in golden["meta_skybox_shape"])
    bg = sc.skybox(w, h)
    arr, _, _ = sc.default_texture_array()
    return bg, arr


def case_texture_kind(golden, name) -> str:
    """'default' (scenes.default_texture_array) or 'features'
    (scenes.feature_texture_array)."""
    return bytes(golden[name + "/textures"]).decode() if name + "/textures" in golden else "default"


def texture_array_of(pkg, kind):
    sc = pkg.scenes
    return (sc.feature_texture_array() if kind == "features" else sc.default_texture_array())[0]


def load_case(pkg, golden, name):
    abi, sc = pkg.abi, pkg.scenes
    scene = sc.struct_from_bytes(abi.Scene, golden[name + "/scene"])
    cam = sc.struct_from_bytes(abi.Camera, golden[name + "/camera"])
    params = sc.struct_from_bytes(abi.Params, golden[name + "/params"])
    tr = sc.struct_from_bytes(abi.TestRay, golden[name + "/test_ray"])
    w, h = (int(v) for v in golden[name + "/size"])
    return scene, cam, params, tr, w, h


def case_rows(golden, name, height):
    """(row_begin, row_end) a golden case holds: a band of the frame (the
    round-3 headline-size goldens) or the whole frame."""
    if name + "/rows" in golden:
        y0, y1 = (int(v) for v in golden[name + "/rows"])
        return y0, y1
    return 0, height
