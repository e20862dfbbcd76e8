#!/usr/bin/env python3
"""Measures SwiftShader's texture filter (the one the golden renders ran
with) and writes tests/golden/ss_filter.npz: small random RGBA8 / RGB8
textures, random texture coordinates and the float32 RGBA SwiftShader's
`texture()` returned for them (GL_LINEAR, GL_REPEAT, no mipmaps, as
image_utils.cpp:12-18 / 111-114 set them up). The probe shader is our own
(a texelFetch of the coordinates, then texture()); no reference source is
involved. tests/test_oracle_golden.py checks the oracle's
SRO_FILTER_SWIFTSHADER mode (oracle/sr_oracle.c sample_swiftshader) against
every sample bit for bit.

    python tests/golden/probe_swiftshader_filter.py   # build container (SwiftShader via kaleido)
"""
from __future__ import annotations

import ctypes as C
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent))
import make_golden as mg  # noqa: E402  (the SwiftShader EGL/GLES wrapper)

OUT = Path(__file__).resolve().parent / "ss_filter.npz"
VS = """#version 300 es
layout(location = 0) in vec3 aPos;
void main() { gl_Position = vec4(aPos, 1.0); }
"""
FS = """#version 300 es
precision highp float;
precision highp sampler2DArray;
uniform highp sampler2D coords;
uniform %s tex;
out vec4 FragColor;
void main() {
    vec4 c = texelFetch(coords, ivec2(gl_FragCoord.xy), 0);
    FragColor = texture(tex, %s);
}
"""
GL_NEAREST, GL_FLOAT = 0x2600, 0x1406


def probe(ss, tex, u, v, lay, array=True, W=64):
    """tex: [L, H, W, C] uint8 (array) or [H, W, C] (2D)."""
    gl = ss.gl
    fs = FS % (("sampler2DArray", "vec3(c.x, c.y, c.z)") if array else ("highp sampler2D", "vec2(c.x, c.y)"))
    prog = gl.glCreateProgram()
    gl.glAttachShader(prog, ss._compile(mg.GL_VERTEX_SHADER, VS))
    gl.glAttachShader(prog, ss._compile(mg.GL_FRAGMENT_SHADER, fs))
    gl.glLinkProgram(prog)
    n = len(u)
    H = -(-n // W)
    c = np.zeros((H * W, 4), np.float32)
    c[:n, 0], c[:n, 1], c[:n, 2] = u, v, lay
    c = c.reshape(H, W, 4)
    t0 = C.c_uint()
    gl.glGenTextures(1, C.byref(t0))
    gl.glActiveTexture(mg.GL_TEXTURE0)
    gl.glBindTexture(mg.GL_TEXTURE_2D, t0)
    gl.glTexImage2D(mg.GL_TEXTURE_2D, 0, mg.GL_RGBA32F, W, H, 0, mg.GL_RGBA, GL_FLOAT, c.ctypes.data_as(C.c_void_p))
    gl.glTexParameteri(mg.GL_TEXTURE_2D, mg.GL_TEXTURE_MIN_FILTER, GL_NEAREST)
    gl.glTexParameteri(mg.GL_TEXTURE_2D, mg.GL_TEXTURE_MAG_FILTER, GL_NEAREST)
    t1 = C.c_uint()
    gl.glGenTextures(1, C.byref(t1))
    gl.glActiveTexture(mg.GL_TEXTURE0 + 1)
    target = mg.GL_TEXTURE_2D_ARRAY if array else mg.GL_TEXTURE_2D
    gl.glBindTexture(target, t1)
    gl.glPixelStorei(mg.GL_UNPACK_ALIGNMENT, 1)
    t = np.ascontiguousarray(tex, dtype=np.uint8)
    fmt = mg.GL_RGBA if t.shape[-1] == 4 else mg.GL_RGB
    if array:
        L, th, tw, _ = t.shape
        gl.glTexImage3D(target, 0, fmt, tw, th, L, 0, fmt, mg.GL_UNSIGNED_BYTE, t.ctypes.data_as(C.c_void_p))
    else:
        th, tw, _ = t.shape
        gl.glTexImage2D(target, 0, fmt, tw, th, 0, fmt, mg.GL_UNSIGNED_BYTE, t.ctypes.data_as(C.c_void_p))
    for p, val in ((mg.GL_TEXTURE_WRAP_S, mg.GL_REPEAT), (mg.GL_TEXTURE_WRAP_T, mg.GL_REPEAT),
                   (mg.GL_TEXTURE_MIN_FILTER, mg.GL_LINEAR), (mg.GL_TEXTURE_MAG_FILTER, mg.GL_LINEAR)):
        gl.glTexParameteri(target, p, val)
    gl.glUseProgram(prog)
    ss.u1i(prog, "coords", 0)
    ss.u1i(prog, "tex", 1)
    out = ss.draw(prog, W, H, float_target=True).reshape(-1, 4)[:n]
    gl.glDeleteTextures(1, C.byref(t0))
    gl.glDeleteTextures(1, C.byref(t1))
    return out


def main():
    ss = mg.SwiftShader()
    rng = np.random.default_rng(20261017)
    cases = {}
    # (name, texture shape, array?, coordinate range)
    for name, shape, array, lo, hi in (("arr7x5", (2, 5, 7, 4), True, -0.5, 1.5),
                                        ("arr1601x3", (2, 3, 1601, 4), True, -0.2, 1.2),
                                        ("arr120x100", (1, 100, 120, 4), True, 0.0, 1.0),
                                        ("rgb61x37", (37, 61, 3), False, -0.3, 1.3),
                                        ("rgb512x256", (256, 512, 3), False, 0.0, 1.0)):
        tex = rng.integers(0, 256, size=shape, dtype=np.uint8)
        if shape[-1] == 4:  # mostly opaque texels: the alpha == 1 question
            tex[..., 3] = np.where(rng.uniform(size=shape[:-1]) < 0.7, 255, tex[..., 3])
        n = 4096
        u = rng.uniform(lo, hi, n).astype(np.float32)
        v = rng.uniform(lo, hi, n).astype(np.float32)
        lay = rng.integers(0, shape[0], n).astype(np.float32) if array else np.zeros(n, np.float32)
        out = probe(ss, tex, u, v, lay, array)
        cases[name] = (tex, u, v, lay, out)
        print(name, "alpha of opaque reads:", np.unique(np.round(out[:, 3] * 65535))[-6:], flush=True)
    z = {"meta_renderer": np.frombuffer(ss.renderer.encode(), dtype=np.uint8), "meta_cases": np.frombuffer(
        "\n".join(cases).encode(), dtype=np.uint8)}
    for name, (tex, u, v, lay, out) in cases.items():
        z.update({f"{name}/tex": tex, f"{name}/u": u, f"{name}/v": v, f"{name}/layer": lay, f"{name}/out": out,
                  f"{name}/array": np.array(int(tex.ndim == 4))})
    np.savez_compressed(OUT, **z)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
