"""The reference's own texture assets through the ingest path (SURVEY §8f
row 1): the skybox of `loadTexture` (image_utils.cpp:7-40) and the texture
array of `loadTextureArray` (image_utils.cpp:42-117) as the app loads them
(src/main.cpp:57-63, 205-218).

The files under `assets/textures/` are data copied unchanged from the
reference's `assets/textures/` (see its sources.txt), so the GPU box, which
has no /root/reference, renders the real inputs. Decoding: the reference uses
stb_image v2.30 (image_utils.cpp:4-5), which is not importable here; PIL
decodes instead. cubemap.png is lossless, so its texels equal stb_image's;
the JPEGs may differ from stb_image's IDCT in the last bit of some texels
(parity is GPU vs oracle on the same decoded texels, so that only moves the
inputs, not the comparison). The decoded images are flipped vertically as
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


def available() -> bool:
    return all(p.exists() for p in [*SKYBOX.values(), *ARRAY])


def decode(path: Path) -> np.ndarray:
    """stbi_load(path, ..., 0) with the vertical flip: uint8 [h, w, channels],
    channels as stored (3 for the JPEGs, 4 for cubemap.png)."""
    from PIL import Image

    with Image.open(path) as im:
        mode = {"RGB": "RGB", "RGBA": "RGBA", "L": "RGB", "P": "RGBA", "LA": "RGBA"}.get(im.mode, "RGB")
        a = np.asarray(im.convert(mode), dtype=np.uint8)
    return np.ascontiguousarray(a[::-1])


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
