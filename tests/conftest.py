import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

import srpkg  # noqa: E402

GOLDEN = ROOT / "tests" / "golden" / "golden.npz"


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
    if not GOLDEN.exists():
        pytest.skip("golden.npz missing (python tests/golden/make_golden.py)")
    return np.load(GOLDEN)


@pytest.fixture(scope="session")
def golden_cases(golden):
    return bytes(golden["meta_cases"]).decode().split("\n")


@pytest.fixture(scope="session")
def textures(pkg, golden):
    sc = pkg.scenes
    h, w = (int(v) for v in golden["meta_skybox_shape"])
    bg = sc.skybox(w, h)
    arr, _, _ = sc.default_texture_array()
    return bg, arr


def load_case(pkg, golden, name):
    abi, sc = pkg.abi, pkg.scenes
    scene = sc.struct_from_bytes(abi.Scene, golden[name + "/scene"])
    cam = sc.struct_from_bytes(abi.Camera, golden[name + "/camera"])
    params = sc.struct_from_bytes(abi.Params, golden[name + "/params"])
    tr = sc.struct_from_bytes(abi.TestRay, golden[name + "/test_ray"])
    w, h = (int(v) for v in golden[name + "/size"])
    return scene, cam, params, tr, w, h
