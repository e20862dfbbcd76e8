"""The reference's own texture assets through the ingest path (SURVEY §8f
row 1): the skybox of `loadTexture` (image_utils.cpp:7-40) and the texture
array of `loadTextureArray` (image_utils.cpp:42-117) as the app loads them
(src/main.cpp:57-63, 205-218).

The files under `assets/textures/` are data copied unchanged from the
reference's `assets/textures/` (see its sources.txt), so the GPU box, which
has no /root/reference, renders the real inputs. Decoding: the reference uses
stb_image (image_utils.cpp:4-5, 22-23). PIL decodes here, and the bytes where
its JPEG IDCT differs from stb_image's (a few per ten thousand in the
skyboxes, 5 % of uv_checker's; none in cubemap.png) are replaced from
`assets/textures/stb_corrections.npz`, which tools/make_stb_corrections.py
made with the reference's own stb_image: the decoded texels are stb_image's,
byte for byte (tests/test_assets_stb.py). Both hashes are checked; if this
machine's PIL decodes differently, the PIL texels are used with a warning.
The decoded images are flipped vertically as
`stbi_set_flip_vertically_on_load(true)` (image_utils.cpp:22) leaves them:
row 0 = v 0, the bottom of the picture.
"""
from __future__ import annotations

from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
TEXTURES = ROOT / "assets" / "textures"
# src/main.cpp:57-63 BACKGROUND_TEXTURE_QUALITY: 0 -> 2k, 1 -> 8k
SKYBOX = {"2k": TEXTURES / "background" / "2k.jpg", "8k": TEXTURES / "background" / "8k.jpg"}
# src/main.cpp:210-213, in texture-array layer order
ARRAY = [TEXTURES / "uv_checker.jpg", TEXTURES / "cubemap.png"]


CORRECTIONS = TEXTURES / "stb_corrections.npz"


def available() -> bool:
    return all(p.exists() for p in [*SKYBOX.values(), *ARRAY])


def decode_pil(path: Path) -> np.ndarray:
    """PIL's decode with the vertical flip: uint8 [h, w, channels], channels
    as stored (3 for the JPEGs, 4 for cubemap.png)."""
    from PIL import Image

    with Image.open(path) as im:
        mode = {"RGB": "RGB", "RGBA": "RGBA", "L": "RGB", "P": "RGBA", "LA": "RGBA"}.get(im.mode, "RGB")
        a = np.asarray(im.convert(mode), dtype=np.uint8)
    return np.ascontiguousarray(a[::-1])


def decode(path: Path) -> np.ndarray:
    """stbi_load(path, ..., 0) with the vertical flip (image_utils.cpp:22-23):
    PIL's decode with stb_image's bytes restored where they differ."""
    import hashlib
    import sys

    a = decode_pil(path)
    if not CORRECTIONS.exists():
        return a
    with np.load(CORRECTIONS) as c:
        key = Path(path).name
        if f"{key}/idx" not in c.files:
            return a
        if tuple(c[f"{key}/shape"]) != a.shape or hashlib.sha256(a.tobytes()).digest() != c[f"{key}/sha_pil"].tobytes():
            print(f"assets: PIL decodes {key} differently here; using PIL's texels, not stb_image's", file=sys.stderr)
            return a
        flat = a.reshape(-1)
        flat[c[f"{key}/idx"]] = c[f"{key}/val"]
        assert hashlib.sha256(a.tobytes()).digest() == c[f"{key}/sha_stb"].tobytes(), key
    return a


def skybox(quality: str = "2k") -> np.ndarray:
    """The background texture (RGB8, rows bottom-up) of BACKGROUND_TEXTURE_QUALITY."""
    return decode(SKYBOX[quality])


def texture_array():
    """loadTextureArray of the app's two textures: (padded array, sizes,
    max size) exactly as scenes.pad_texture_array lays them out (RGB layers
    get alpha 255 inside the image, every layer is zero-padded to the
    largest one)."""
    from .scenes import pad_texture_array

    return pad_texture_array([decode(p) for p in ARRAY])
