#!/usr/bin/env python3
"""Byte-exact inputs: the reference decodes its textures with stb_image
(image_utils.cpp:22-23); the package decodes them with PIL, whose JPEG IDCT
differs from stb_image's in a few bytes (2k skybox 0.05 %, 8k 0.03 %,
uv_checker 5 %; cubemap.png none). This script decodes every asset with the
reference's own stb_image (oracle/_ref/libref_stbi.so, built by
`make -C oracle ref` from /root/reference) and stores, per file, the bytes
where PIL's decode differs: assets/textures/stb_corrections.npz. The package
applies them (assets.decode), so the GPU box, which has no reference, gets
stb_image's bytes. Checked by tests/test_assets_stb.py.

  make -C oracle ref && python tools/make_stb_corrections.py
"""
import ctypes as C
import hashlib
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def stb_decode(lib, path: Path) -> np.ndarray:
    w, h, ch = C.c_int(), C.c_int(), C.c_int()
    ptr = lib.ref_stbi_load(str(path).encode(), 1, C.byref(w), C.byref(h), C.byref(ch))
    if not ptr:
        raise RuntimeError(f"stb_image could not decode {path}")
    a = np.ctypeslib.as_array(ptr, shape=(h.value, w.value, ch.value)).copy()
    lib.ref_stbi_free(ptr)
    return a


def load_stb():
    lib = C.CDLL(str(ROOT / "oracle" / "_ref" / "libref_stbi.so"))
    lib.ref_stbi_load.restype = C.POINTER(C.c_ubyte)
    lib.ref_stbi_load.argtypes = [C.c_char_p, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]
    lib.ref_stbi_free.argtypes = [C.POINTER(C.c_ubyte)]
    return lib


def main():
    import srpkg

    assets = srpkg.load_package().assets
    lib = load_stb()
    out = {}
    for p in [*assets.SKYBOX.values(), *assets.ARRAY]:
        stb = stb_decode(lib, p)
        pil = assets.decode_pil(p)
        assert stb.shape == pil.shape, (p, stb.shape, pil.shape)
        idx = np.flatnonzero(stb.reshape(-1) != pil.reshape(-1)).astype(np.uint32)
        key = p.name
        out[f"{key}/idx"] = idx
        out[f"{key}/val"] = stb.reshape(-1)[idx]
        out[f"{key}/shape"] = np.array(stb.shape, np.int64)
        out[f"{key}/sha_pil"] = np.frombuffer(hashlib.sha256(pil.tobytes()).digest(), np.uint8)
        out[f"{key}/sha_stb"] = np.frombuffer(hashlib.sha256(stb.tobytes()).digest(), np.uint8)
        print(f"{key}: {stb.shape}, {idx.size} bytes differ from PIL")
    np.savez_compressed(assets.CORRECTIONS, **out)
    print(f"wrote {assets.CORRECTIONS}")


if __name__ == "__main__":
    main()
