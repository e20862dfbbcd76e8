"""Texture ingest at the input, byte for byte: the
package's decode of the reference's assets equals the reference's own
decoder, stb_image (image_utils.cpp:22-23), built from the reference's
vendored stb_image.h into oracle/_ref/ when /root/reference is present. The
stored corrections (tools/make_stb_corrections.py) are checked everywhere."""
import ctypes as C
import hashlib
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
STB = ROOT / "oracle" / "_ref" / "libref_stbi.so"


def test_assets_decode_to_the_stored_stb_bytes(pkg):
    assets = pkg.assets
    if not assets.available():
        pytest.skip("assets/textures missing")
    with np.load(assets.CORRECTIONS) as c:
        for p in [assets.SKYBOX["2k"], *assets.ARRAY]:
            a = assets.decode(p)  # asserts the stb hash itself
            assert hashlib.sha256(a.tobytes()).digest() == c[f"{p.name}/sha_stb"].tobytes(), p.name
            assert tuple(a.shape) == tuple(c[f"{p.name}/shape"])
        # PIL differs from stb_image in a few bytes of every JPEG, never in the PNG
        assert c["2k.jpg/idx"].size > 0 and c["cubemap.png/idx"].size == 0


@pytest.mark.skipif(not STB.exists(), reason="oracle/_ref not built (make -C oracle ref; needs /root/reference)")
def test_assets_equal_reference_stb_image(pkg):
    sys.path.insert(0, str(ROOT / "tools"))
    from make_stb_corrections import load_stb, stb_decode

    lib = load_stb()
    for p in [*pkg.assets.SKYBOX.values(), *pkg.assets.ARRAY]:
        assert np.array_equal(pkg.assets.decode(p), stb_decode(lib, p)), p.name
