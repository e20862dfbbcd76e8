#!/usr/bin/env python3
"""Golden-vector generator: renders the REFERENCE fragment shader itself on
SwiftShader (a CPU OpenGL ES 3.0 implementation that ships in this image with
the kaleido package) and stores the RGBA8 frames as fixtures.

The shader source is read from /root/reference/assets/shaders/ at generation
time and edited mechanically in memory so an ES 3.00 compiler accepts it
(SURVEY.md Appendix A); no arithmetic is changed and no reference source is
written to the repository:
  1. `#version 330 core` -> `#version 300 es` (both shaders)
  2. `precision highp sampler2DArray;` added (ES has no default for it)
  3. uniform initializers stripped; the same defaults are set from the host
  4. int literals in float contexts made float (ES has no implicit conversion)
  5. MAX_* array capacities shrunk to fit SwiftShader's 261 uniform vectors
     (loops are bounded by num_objects / num_lights / num points, not MAX_*)
A "steps" variant adds a counter incremented at the top of the step loop
(frag:890) and writes it instead of the colour, for step-count parity.

Inputs are the library's own scene/camera structs (sr_default_scene =
the C++ mirror of src/main.cpp:222-268) and integer-procedural textures, so the
goldens do not depend on a JPEG decoder. Run in the build container:
    python tests/golden/make_golden.py            # writes tests/golden/golden.npz
    python tests/golden/make_golden.py --set r2   # writes tests/golden/golden_r2.npz
    python tests/golden/make_golden.py --set r3   # writes tests/golden/golden_r3.npz (headline-size bands)
"""
from __future__ import annotations

import argparse
import ctypes as C
import re
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import srpkg  # noqa: E402

PKG = srpkg.load_package()
abi, sc = PKG.abi, PKG.scenes

REF_SHADERS = Path("/root/reference/assets/shaders")
SS_DIR = Path("/usr/local/lib/python3.10/dist-packages/kaleido/executable/bin/swiftshader")

# ---- GL / EGL enums ------------------------------------------------------------
EGL_SURFACE_TYPE, EGL_PBUFFER_BIT, EGL_RENDERABLE_TYPE, EGL_OPENGL_ES3_BIT = 0x3033, 0x1, 0x3040, 0x40
EGL_RED_SIZE, EGL_GREEN_SIZE, EGL_BLUE_SIZE, EGL_ALPHA_SIZE, EGL_NONE = 0x3024, 0x3023, 0x3022, 0x3021, 0x3038
EGL_WIDTH, EGL_HEIGHT, EGL_OPENGL_ES_API, EGL_CONTEXT_CLIENT_VERSION = 0x3057, 0x3056, 0x30A0, 0x3098
GL_FRAGMENT_SHADER, GL_VERTEX_SHADER, GL_COMPILE_STATUS, GL_LINK_STATUS = 0x8B30, 0x8B31, 0x8B81, 0x8B82
GL_ARRAY_BUFFER, GL_ELEMENT_ARRAY_BUFFER, GL_STATIC_DRAW = 0x8892, 0x8893, 0x88E4
GL_FLOAT, GL_UNSIGNED_INT, GL_UNSIGNED_BYTE, GL_TRIANGLES = 0x1406, 0x1405, 0x1401, 0x0004
GL_TEXTURE_2D, GL_TEXTURE_2D_ARRAY, GL_TEXTURE0 = 0x0DE1, 0x8C1A, 0x84C0
GL_RGB, GL_RGBA, GL_RGBA8, GL_RGBA32F = 0x1907, 0x1908, 0x8058, 0x8814
GL_TEXTURE_WRAP_S, GL_TEXTURE_WRAP_T, GL_REPEAT = 0x2802, 0x2803, 0x2901
GL_TEXTURE_MIN_FILTER, GL_TEXTURE_MAG_FILTER, GL_LINEAR = 0x2801, 0x2800, 0x2601
GL_COLOR_BUFFER_BIT, GL_UNPACK_ALIGNMENT, GL_PACK_ALIGNMENT = 0x4000, 0x0CF5, 0x0D05
GL_FRAMEBUFFER, GL_RENDERBUFFER, GL_COLOR_ATTACHMENT0, GL_FRAMEBUFFER_COMPLETE = 0x8D40, 0x8D41, 0x8CE0, 0x8CD5
GL_SCISSOR_TEST = 0x0C11

ES_CAPACITIES = {
    "MAX_LIGHTS": 1, "MAX_TEXTURES": 2, "MAX_MATERIALS": 3, "MAX_SPHERES": 1, "MAX_PLANES": 1,
    "MAX_DISKS": 1, "MAX_HOLLOW_DISKS": 1, "MAX_CYLINDERS": 1, "MAX_RECTANGLES": 1, "MAX_BOXES": 1,
    "MAX_POINTS": 8,
}
# Capacity profiles: the 261 uniform vectors are traded between features.
# "features" gives up the press-R polyline (MAX_POINTS 1) for the reference's
# full 4 lights, 8 materials and 2 planes (the material-flag scene, cases_r2;
# 10 materials do not fit).
ES_PROFILES = {
    "default": ES_CAPACITIES,
    "features": dict(ES_CAPACITIES, MAX_LIGHTS=4, MAX_MATERIALS=8, MAX_PLANES=2, MAX_POINTS=1),
}


def es_sources(steps_variant: bool = False, caps: dict | None = None) -> tuple[str, str]:
    vert = (REF_SHADERS / "full_screen_quad.vert").read_text()
    frag = (REF_SHADERS / "black_hole.frag").read_text()
    vert = vert.replace("#version 330 core", "#version 300 es")
    frag = frag.replace("#version 330 core", "#version 300 es")
    frag = frag.replace("precision highp sampler2D;", "precision highp sampler2D;\nprecision highp sampler2DArray;")
    # 3. strip uniform initializers (defaults are uploaded by the host)
    frag = re.sub(r"^(\s*uniform\s+\w+\s+\w+)\s*=\s*[^;]+;", r"\1;", frag, flags=re.M)
    # 4. int -> float literals where ES requires them
    subs = [
        ("if(n1 > 0 && n2 > 0)", "if(n1 > 0. && n2 > 0.)"),
        ("else if(n1 > 0)", "else if(n1 > 0.)"),
        ("else if(n2 > 0)", "else if(n2 > 0.)"),
        ("sphere.transform.pos), 2)", "sphere.transform.pos), 2.)"),
        ("if(D < 0) {", "if(D < 0.) {"),
        ("res.is_hit = lambda >= 0 &&", "res.is_hit = lambda >= 0. &&"),
        ("is_in_range(alpha, 0, rectangle.width)", "is_in_range(alpha, 0., rectangle.width)"),
        ("is_in_range(beta, 0, rectangle.height)", "is_in_range(beta, 0., rectangle.height)"),
    ]
    for a, b in subs:
        if a not in frag:
            raise RuntimeError(f"ES edit anchor not found: {a!r}")
        frag = frag.replace(a, b)
    # 5. capacities
    for k, v in (caps or ES_CAPACITIES).items():
        frag, n = re.subn(rf"#define {k} \d+", f"#define {k} {v}", frag)
        if n != 1:
            raise RuntimeError(f"capacity {k} not found")
    if steps_variant:
        anchor = "for(int i = 0; i < max_steps; i++) {"
        if frag.count(anchor) != 1:
            raise RuntimeError("step-loop anchor not found")
        frag = frag.replace(anchor, anchor + "\n        g_steps++;")
        frag = frag.replace("void main() {", "int g_steps = 0;\nvoid ref_main() {", 1)
        frag += (
            "\nvoid main() {\n    ref_main();\n"
            "    FragColor = vec4(float(g_steps % 256) / 255., float((g_steps / 256) % 256) / 255., 0., 1.);\n}\n"
        )
    return vert, frag


class SwiftShader:
    def __init__(self):
        self.egl = C.CDLL(str(SS_DIR / "libEGL.so"))
        self.gl = C.CDLL(str(SS_DIR / "libGLESv2.so"))
        egl = self.egl
        egl.eglGetDisplay.restype = C.c_void_p
        egl.eglCreatePbufferSurface.restype = C.c_void_p
        egl.eglCreateContext.restype = C.c_void_p
        self.dpy = egl.eglGetDisplay(C.c_void_p(0))
        assert egl.eglInitialize(C.c_void_p(self.dpy), None, None)
        attrs = (C.c_int * 13)(EGL_SURFACE_TYPE, EGL_PBUFFER_BIT, EGL_RENDERABLE_TYPE, EGL_OPENGL_ES3_BIT,
                               EGL_RED_SIZE, 8, EGL_GREEN_SIZE, 8, EGL_BLUE_SIZE, 8, EGL_ALPHA_SIZE, 8, EGL_NONE)
        cfg = C.c_void_p()
        n = C.c_int()
        assert egl.eglChooseConfig(C.c_void_p(self.dpy), attrs, C.byref(cfg), 1, C.byref(n)) and n.value > 0
        surf = egl.eglCreatePbufferSurface(C.c_void_p(self.dpy), cfg, (C.c_int * 5)(EGL_WIDTH, 16, EGL_HEIGHT, 16, EGL_NONE))
        egl.eglBindAPI(EGL_OPENGL_ES_API)
        ctx = egl.eglCreateContext(C.c_void_p(self.dpy), cfg, None, (C.c_int * 3)(EGL_CONTEXT_CLIENT_VERSION, 3, EGL_NONE))
        assert ctx, "eglCreateContext failed"
        assert egl.eglMakeCurrent(C.c_void_p(self.dpy), C.c_void_p(surf), C.c_void_p(surf), C.c_void_p(ctx))
        gl = self.gl
        gl.glGetString.restype = C.c_char_p
        gl.glGetUniformLocation.restype = C.c_int
        gl.glCreateShader.restype = C.c_uint
        gl.glCreateProgram.restype = C.c_uint
        gl.glUniform1f.argtypes = [C.c_int, C.c_float]
        gl.glUniform2f.argtypes = [C.c_int, C.c_float, C.c_float]
        gl.glUniform3f.argtypes = [C.c_int, C.c_float, C.c_float, C.c_float]
        gl.glUniform4f.argtypes = [C.c_int, C.c_float, C.c_float, C.c_float, C.c_float]
        gl.glUniform1i.argtypes = [C.c_int, C.c_int]
        gl.glUniformMatrix3fv.argtypes = [C.c_int, C.c_int, C.c_ubyte, C.POINTER(C.c_float)]
        self.renderer = gl.glGetString(0x1F01).decode() + " / " + gl.glGetString(0x1F02).decode()
        self.programs = {}
        self._quad()

    def _quad(self):
        gl = self.gl
        verts = (C.c_float * 20)(1, 1, 0, 1, 1, 1, -1, 0, 1, -1, -1, -1, 0, -1, -1, -1, 1, 0, -1, 1)
        idx = (C.c_uint * 6)(0, 1, 3, 1, 2, 3)
        vao, vbo, ebo = C.c_uint(), C.c_uint(), C.c_uint()
        gl.glGenVertexArrays(1, C.byref(vao))
        gl.glGenBuffers(1, C.byref(vbo))
        gl.glGenBuffers(1, C.byref(ebo))
        gl.glBindVertexArray(vao)
        gl.glBindBuffer(GL_ARRAY_BUFFER, vbo)
        gl.glBufferData(GL_ARRAY_BUFFER, C.sizeof(verts), verts, GL_STATIC_DRAW)
        gl.glBindBuffer(GL_ELEMENT_ARRAY_BUFFER, ebo)
        gl.glBufferData(GL_ELEMENT_ARRAY_BUFFER, C.sizeof(idx), idx, GL_STATIC_DRAW)
        gl.glVertexAttribPointer(0, 3, GL_FLOAT, 0, 20, C.c_void_p(0))
        gl.glEnableVertexAttribArray(0)
        gl.glVertexAttribPointer(1, 2, GL_FLOAT, 0, 20, C.c_void_p(12))
        gl.glEnableVertexAttribArray(1)

    def _compile(self, kind, src):
        gl = self.gl
        sh = gl.glCreateShader(kind)
        b = src.encode()
        gl.glShaderSource(sh, 1, C.byref(C.c_char_p(b)), None)
        gl.glCompileShader(sh)
        ok = C.c_int()
        gl.glGetShaderiv(sh, GL_COMPILE_STATUS, C.byref(ok))
        if not ok.value:
            log = C.create_string_buffer(8192)
            gl.glGetShaderInfoLog(sh, 8192, None, log)
            raise RuntimeError("shader compile failed:\n" + log.value.decode())
        return sh

    def program(self, steps_variant=False, profile="default"):
        key = (steps_variant, profile)
        if key in self.programs:
            return self.programs[key]
        gl = self.gl
        vs, fs = es_sources(steps_variant, ES_PROFILES[profile])
        prog = gl.glCreateProgram()
        gl.glAttachShader(prog, self._compile(GL_VERTEX_SHADER, vs))
        gl.glAttachShader(prog, self._compile(GL_FRAGMENT_SHADER, fs))
        gl.glLinkProgram(prog)
        ok = C.c_int()
        gl.glGetProgramiv(prog, GL_LINK_STATUS, C.byref(ok))
        if not ok.value:
            log = C.create_string_buffer(8192)
            gl.glGetProgramInfoLog(prog, 8192, None, log)
            raise RuntimeError("link failed:\n" + log.value.decode())
        self.programs[key] = prog
        return prog

    # ---- uniforms ----------------------------------------------------------------
    def _loc(self, prog, name):
        return self.gl.glGetUniformLocation(prog, name.encode())

    def u1i(self, prog, name, v):
        self.gl.glUniform1i(self._loc(prog, name), int(v))

    def u1f(self, prog, name, v):
        self.gl.glUniform1f(self._loc(prog, name), float(v))

    def u2f(self, prog, name, v):
        self.gl.glUniform2f(self._loc(prog, name), float(v[0]), float(v[1]))

    def u3f(self, prog, name, v):
        self.gl.glUniform3f(self._loc(prog, name), float(v[0]), float(v[1]), float(v[2]))

    def u4f(self, prog, name, v):
        self.gl.glUniform4f(self._loc(prog, name), *[float(x) for x in v[:4]])

    def utransform(self, prog, prefix, t):
        self.u3f(prog, prefix + ".pos", t.pos)
        m = (C.c_float * 9)(*t.axes)
        self.gl.glUniformMatrix3fv(self._loc(prog, prefix + ".axes"), 1, 0, m)

    def uplane(self, prog, prefix, p):
        self.utransform(prog, prefix + ".transform", p.transform)
        self.u2f(prog, prefix + ".texture_offset", p.texture_offset)
        self.u1i(prog, prefix + ".repeat_texture", p.repeat_texture)
        self.u2f(prog, prefix + ".texture_size", p.texture_size)

    def set_uniforms(self, prog, scene, cam, params, test_ray, width, height, caps=None):
        """What Camera::loadShader, ObjectLoader::load, loadTextureArray and the
        main loop upload (src/main.cpp:272-297, 377-429)."""
        gl = self.gl
        caps = caps or ES_CAPACITIES
        assert scene.num_lights <= caps["MAX_LIGHTS"], "scene exceeds the ES light capacity"
        gl.glUseProgram(prog)
        self.u1i(prog, "background_texture", 0)
        self.u1i(prog, "textures", 1)
        self.u2f(prog, "resolution", (width, height))
        self.u1f(prog, "time", params.time)
        self.u1i(prog, "max_steps", params.max_steps)
        self.u1i(prog, "max_revolutions", params.max_revolutions)
        self.u1f(prog, "u_f", params.u_f)
        self.u1i(prog, "crosshair", params.crosshair)
        self.u1i(prog, "raytrace_type", params.raytrace_type)
        self.u1f(prog, "curved_percentage", params.curved_percentage)
        self.u1f(prog, "percent_black", params.percent_black)
        self.utransform(prog, "cam.transform", cam.transform)
        self.u1f(prog, "cam.fov", cam.fov)
        self.u1i(prog, "num_lights", scene.num_lights)
        for i in range(scene.num_lights):
            L, pre = scene.lights[i], f"lights[{i}]"
            self.utransform(prog, pre + ".transform", L.transform)
            self.u3f(prog, pre + ".color", L.color)
            self.u1f(prog, pre + ".intensity", L.intensity)
            self.u1f(prog, pre + ".attenuation_constant", L.attenuation_constant)
            self.u1f(prog, pre + ".attenuation_linear", L.attenuation_linear)
            self.u1f(prog, pre + ".attenuation_quadratic", L.attenuation_quadratic)
        for i in range(caps["MAX_TEXTURES"]):
            self.u2f(prog, f"texture_sizes[{i}]", scene.texture_sizes[i])
        self.u2f(prog, "max_texture_size", scene.max_texture_size)
        for m in range(caps["MAX_MATERIALS"]):
            M, pre = scene.materials[m], f"materials[{m}]"
            self.u4f(prog, pre + ".color", M.color)
            for f in ("ambient", "diffuse", "specular", "shininess"):
                self.u1f(prog, f"{pre}.{f}", getattr(M, f))
            for f in ("texture_index", "normal_map_index", "invert_uv_x", "invert_uv_y", "swap_uvs",
                      "double_sided_normals", "flip_normals"):
                self.u1i(prog, f"{pre}.{f}", getattr(M, f))
        self.u1i(prog, "num_objects", scene.num_objects)
        for i in range(scene.num_objects):
            o = scene.objects[i]
            self.u1i(prog, f"objects[{i}].type", o.type)
            self.u1i(prog, f"objects[{i}].index", o.index)
            self.u1i(prog, f"objects[{i}].material_index", o.material_index)
        for k in range(caps["MAX_SPHERES"]):
            self.utransform(prog, f"spheres[{k}].transform", scene.spheres[k].transform)
            self.u1f(prog, f"spheres[{k}].radius", scene.spheres[k].radius)
        for k in range(caps["MAX_PLANES"]):
            self.uplane(prog, f"planes[{k}]", scene.planes[k])
        for k in range(caps["MAX_DISKS"]):
            self.uplane(prog, f"disks[{k}].plane", scene.disks[k].plane)
            self.u1f(prog, f"disks[{k}].radius", scene.disks[k].radius)
        for k in range(caps["MAX_HOLLOW_DISKS"]):
            self.uplane(prog, f"hollow_disks[{k}].plane", scene.hollow_disks[k].plane)
            self.u1f(prog, f"hollow_disks[{k}].inner_radius", scene.hollow_disks[k].inner_radius)
            self.u1f(prog, f"hollow_disks[{k}].outer_radius", scene.hollow_disks[k].outer_radius)
        for k in range(caps["MAX_CYLINDERS"]):
            self.utransform(prog, f"cylinders[{k}].transform", scene.cylinders[k].transform)
            self.u1f(prog, f"cylinders[{k}].height", scene.cylinders[k].height)
            self.u1f(prog, f"cylinders[{k}].radius", scene.cylinders[k].radius)
        for k in range(caps["MAX_RECTANGLES"]):
            self.uplane(prog, f"rectangles[{k}].plane", scene.rectangles[k].plane)
            self.u1f(prog, f"rectangles[{k}].width", scene.rectangles[k].width)
            self.u1f(prog, f"rectangles[{k}].height", scene.rectangles[k].height)
        for k in range(caps["MAX_BOXES"]):
            b = scene.boxes[k]
            self.utransform(prog, f"boxes[{k}].transform", b.transform)
            self.u1f(prog, f"boxes[{k}].width", b.width)
            self.u1f(prog, f"boxes[{k}].depth", b.depth)
            self.u1f(prog, f"boxes[{k}].height", b.height)
        tr = test_ray
        self.u1i(prog, "test_ray_visible", tr.visible)
        self.u1f(prog, "test_ray_radius", tr.radius)
        self.u1f(prog, "test_ray_extended_length", tr.extended_length)
        self.u4f(prog, "test_ray_curved_color", tr.curved_color)
        self.u4f(prog, "test_ray_flat_color", tr.flat_color)
        self.u3f(prog, "test_ray_flat_origin", tr.flat_origin)
        self.u3f(prog, "test_ray_flat_dir", tr.flat_dir)
        self.u1i(prog, "num_test_ray_curved_points", tr.num_curved_points)
        for i in range(min(tr.num_curved_points, caps["MAX_POINTS"])):
            self.u3f(prog, f"test_ray_curved_points[{i}]", tr.curved_points[i])

    # ---- textures ----------------------------------------------------------------
    def set_textures(self, bg: np.ndarray | None, arr: np.ndarray | None):
        gl = self.gl
        gl.glPixelStorei(GL_UNPACK_ALIGNMENT, 1)
        for unit, target, data in ((0, GL_TEXTURE_2D, bg), (1, GL_TEXTURE_2D_ARRAY, arr)):
            tex = C.c_uint()
            gl.glGenTextures(1, C.byref(tex))
            gl.glActiveTexture(GL_TEXTURE0 + unit)
            gl.glBindTexture(target, tex)
            if data is not None:
                data = np.ascontiguousarray(data, dtype=np.uint8)
                fmt = GL_RGBA if data.shape[-1] == 4 else GL_RGB
                if target == GL_TEXTURE_2D:
                    h, w, _ = data.shape
                    gl.glTexImage2D(target, 0, fmt, w, h, 0, fmt, GL_UNSIGNED_BYTE, data.ctypes.data_as(C.c_void_p))
                else:
                    layers, h, w, _ = data.shape
                    gl.glTexImage3D(target, 0, fmt, w, h, layers, 0, fmt, GL_UNSIGNED_BYTE,
                                    data.ctypes.data_as(C.c_void_p))
            gl.glTexParameteri(target, GL_TEXTURE_WRAP_S, GL_REPEAT)
            gl.glTexParameteri(target, GL_TEXTURE_WRAP_T, GL_REPEAT)
            gl.glTexParameteri(target, GL_TEXTURE_MIN_FILTER, GL_LINEAR)
            gl.glTexParameteri(target, GL_TEXTURE_MAG_FILTER, GL_LINEAR)

    def draw(self, prog, width, height, float_target=False, rows=None):
        """The full-screen draw; rows=(y0, y1): only that band of the frame is
        rasterised (scissor test) and read back."""
        gl = self.gl
        fbo, rb = C.c_uint(), C.c_uint()
        gl.glGenFramebuffers(1, C.byref(fbo))
        gl.glBindFramebuffer(GL_FRAMEBUFFER, fbo)
        gl.glGenRenderbuffers(1, C.byref(rb))
        gl.glBindRenderbuffer(GL_RENDERBUFFER, rb)
        gl.glRenderbufferStorage(GL_RENDERBUFFER, GL_RGBA32F if float_target else GL_RGBA8, width, height)
        gl.glFramebufferRenderbuffer(GL_FRAMEBUFFER, GL_COLOR_ATTACHMENT0, GL_RENDERBUFFER, rb)
        if gl.glCheckFramebufferStatus(GL_FRAMEBUFFER) != GL_FRAMEBUFFER_COMPLETE:
            raise RuntimeError("framebuffer incomplete (float target unsupported?)")
        gl.glViewport(0, 0, width, height)
        gl.glClearColor(C.c_float(0), C.c_float(0), C.c_float(0), C.c_float(0))
        gl.glClear(GL_COLOR_BUFFER_BIT)
        y0, y1 = rows if rows else (0, height)
        if rows:
            gl.glEnable(GL_SCISSOR_TEST)
            gl.glScissor(0, y0, width, y1 - y0)
        gl.glUseProgram(prog)
        gl.glDrawElements(GL_TRIANGLES, 6, GL_UNSIGNED_INT, None)
        gl.glFinish()
        if rows:
            gl.glDisable(GL_SCISSOR_TEST)
        err = gl.glGetError()
        if err:
            raise RuntimeError(f"GL error 0x{err:x}")
        gl.glPixelStorei(GL_PACK_ALIGNMENT, 1)
        if float_target:
            out = np.zeros((y1 - y0, width, 4), dtype=np.float32)
            gl.glReadPixels(0, y0, width, y1 - y0, GL_RGBA, GL_FLOAT, out.ctypes.data_as(C.c_void_p))
        else:
            out = np.zeros((y1 - y0, width, 4), dtype=np.uint8)
            gl.glReadPixels(0, y0, width, y1 - y0, GL_RGBA, GL_UNSIGNED_BYTE, out.ctypes.data_as(C.c_void_p))
        gl.glDeleteFramebuffers(1, C.byref(fbo))
        gl.glDeleteRenderbuffers(1, C.byref(rb))
        return out  # rows bottom-up (GL order), like the kernel's output

    def render(self, scene, cam, params, width, height, test_ray=None, steps_variant=False, float_target=False,
               profile="default", rows=None):
        prog = self.program(steps_variant, profile)
        tr = test_ray if test_ray is not None else abi.default_test_ray()
        self.set_uniforms(prog, scene, cam, params, tr, width, height, ES_PROFILES[profile])
        return self.draw(prog, width, height, float_target, rows)


# ---- the golden case list ----------------------------------------------------------
SKYBOX_W, SKYBOX_H = 512, 256


def textures():
    bg = sc.skybox(SKYBOX_W, SKYBOX_H)
    arr, sizes, mx = sc.default_texture_array()
    return bg, arr, sizes, mx


def cases():
    """(name, scene_kind, camera, params, width, height, test_ray, extras)"""
    P = abi.default_params
    dcam = abi.default_camera()
    out = [
        ("bh_default", "bh", dcam, P(max_steps=1000, percent_black=-1.0), 160, 90, None, {"steps": True, "float": True}),
        ("scene_untex", "untex", dcam, P(max_steps=1000, percent_black=-1.0), 160, 90, None, {"steps": True, "float": True}),
        ("scene_tex", "tex", dcam, P(max_steps=1000, percent_black=-1.0), 160, 90, None, {"steps": True}),
        ("scene_tex_weighted", "tex", dcam, P(max_steps=1000, percent_black=-1.0, filter_mode=abi.FILTER_WEIGHTED),
         160, 90, None, {}),
        ("scene_tex_2000", "tex", dcam, P(max_steps=2000, percent_black=-1.0), 320, 180, None, {}),
        ("mode_flat", "tex", dcam, P(max_steps=300, percent_black=-1.0, raytrace_type=1), 96, 54, None, {}),
        ("mode_half_width", "untex", dcam, P(max_steps=300, percent_black=-1.0, raytrace_type=2,
                                             curved_percentage=0.5), 96, 54, None, {}),
        ("mode_half_height", "untex", dcam, P(max_steps=300, percent_black=-1.0, raytrace_type=3,
                                              curved_percentage=0.3), 96, 54, None, {}),
        ("noise_mask", "untex", dcam, P(max_steps=300, percent_black=0.75), 96, 54, None, {}),
        ("crosshair", "untex", dcam, P(max_steps=300, percent_black=-1.0, crosshair=1), 96, 54, None, {}),
        ("steps_100", "untex", dcam, P(max_steps=100, percent_black=-1.0), 96, 54, None, {"steps": True}),
    ]
    for seed in range(1, 9):
        cam = sc.random_camera(seed)
        kind = "bh" if seed % 2 else "untex"
        out.append((f"rand_{seed}", kind, cam, P(max_steps=500, percent_black=-1.0), 64, 36, None, {"steps": True}))
    # press-R overlay with <= 8 points (the ES build holds MAX_POINTS = 8)
    cam = sc.camera_look((3.0, 2.0, 14.0), (-0.2, -0.1, -1.0))
    fwd = list(cam.transform.axes[6:9])
    pts = abi.test_ray_points(list(cam.transform.pos), fwd, 7, 2)
    tr = abi.default_test_ray()
    tr.visible = 1
    tr.num_curved_points = len(pts)
    for i, p in enumerate(pts):
        tr.curved_points[i][0], tr.curved_points[i][1], tr.curved_points[i][2] = p
    tr.flat_origin[0], tr.flat_origin[1], tr.flat_origin[2] = (cam.transform.pos[k] + fwd[k] for k in range(3))
    tr.flat_dir[0], tr.flat_dir[1], tr.flat_dir[2] = fwd
    view = sc.camera_look((8.0, 6.0, 20.0), (-8.0, -6.0, -20.0))
    out.append(("test_ray", "untex", view, P(max_steps=300, percent_black=-1.0), 96, 54, tr, {}))
    return out


def cases_r2():
    """Round-2 goldens (golden_r2.npz): the u < u_f reseed branch (frag:891-912,
    phi not reset) from cameras beyond r = 1/u_f and with u_f = 0.1, the
    640x360 / 1000-step frame of BASELINE config 2, and the material-flag
    scene (scenes.scene_features: planes, normal maps, uv flags, single-sided,
    flipped and translucent materials, 4 lights) under the "features" ES
    capacity profile."""
    P = abi.default_params
    dcam = abi.default_camera()
    far120 = sc.camera_look((0.0, 12.0, 119.4), (0.0, -12.0, -119.4), fov=12.0)
    far300 = sc.camera_look((60.0, 40.0, 291.2), (-60.0, -40.0, -291.2), fov=5.0)
    side = sc.camera_look((-150.0, 3.0, 40.0), (150.0, -3.0, -41.0), fov=8.0)
    feat = {"profile": "features", "textures": "features"}
    out = [
        ("reseed_r120", "untex", far120, P(max_steps=1000, percent_black=-1.0), 160, 90, None,
         {"steps": True, "float": True}),
        ("reseed_r300", "untex", far300, P(max_steps=1000, percent_black=-1.0), 160, 90, None, {"steps": True}),
        ("reseed_side", "bh", side, P(max_steps=1000, percent_black=-1.0), 128, 72, None, {"steps": True}),
        ("reseed_uf01", "untex", dcam, P(max_steps=1000, percent_black=-1.0, u_f=0.1), 160, 90, None,
         {"steps": True, "float": True}),
        ("reseed_uf005_far", "untex", far120, P(max_steps=600, percent_black=-1.0, u_f=0.05), 96, 54, None,
         {"steps": True}),
        ("config2_640x360", "untex", dcam, P(max_steps=1000, percent_black=-1.0), 640, 360, None, {"steps": True}),
    ]
    fcams = [
        ("features_default", dcam, 0),
        ("features_oblique", sc.camera_look((12.0, 8.0, 14.0), (-12.0, -8.0, -14.0), fov=70.0), 0),
        ("features_low", sc.camera_look((-3.0, -2.5, 12.0), (3.0, 1.5, -12.0), fov=80.0), 0),
        ("features_below", sc.camera_look((2.0, -7.0, 10.0), (-2.0, 6.0, -10.0), fov=75.0), 0),
        ("features_flat", sc.camera_look((12.0, 8.0, 14.0), (-12.0, -8.0, -14.0), fov=70.0), 1),
    ]
    for name, cam, mode in fcams:
        ex = dict(feat, steps=mode == 0, float=name == "features_default")
        out.append((name, "features", cam, P(max_steps=600, percent_black=-1.0, raytrace_type=mode), 96, 54, None, ex))
    return out


def cases_r3():
    """Round-3 goldens (golden_r3.npz): bands of the headline frame itself
    (BASELINE config 3, 1920x1080 / 2000 steps, the app's camera) where its
    cost is - rows 704-719 hold the photon-ring waves that set the frame's
    critical path (bench roofline.critical_path), rows 536-551 run through the
    black hole - for the untextured and the textured default scene, and a
    3840-wide band of config 4 (4000 steps) through the ring. Each band is the
    full-size frame rasterised under a scissor rectangle: uv, resolution and
    every ray are the full frame's."""
    P = abi.default_params
    dcam = abi.default_camera()
    out = []
    for y0 in (704, 536):
        for kind in ("untex", "tex"):
            out.append((f"band1080_{y0}_{kind}", kind, dcam, P(max_steps=2000, percent_black=-1.0), 1920, 1080, None,
                        {"steps": True, "rows": (y0, y0 + 16)}))
    out.append(("band2160_1408_untex", "untex", dcam, P(max_steps=4000, percent_black=-1.0), 3840, 2160, None,
                {"steps": True, "rows": (1408, 1424)}))
    return out


def scene_for(kind, sizes, mx):
    if kind == "features":
        return sc.scene_features()
    if kind == "bh":
        s = sc.scene_black_hole_only()
    else:
        s = sc.scene_default(textured=(kind == "tex"))
    sc.set_scene_texture_sizes(s, sizes, mx)
    return s


def texture_set(kind):
    """(skybox, texture array, sizes, max size) of a golden case's texture kind."""
    bg = sc.skybox(SKYBOX_W, SKYBOX_H)
    if kind == "features":
        arr, sizes, mx = sc.feature_texture_array()
    else:
        arr, sizes, mx = sc.default_texture_array()
    return bg, arr, sizes, mx


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--set", choices=["r1", "r2", "r3"], default="r1",
                    help="r1: golden.npz (round-1 cases); r2: golden_r2.npz (reseed, config 2, material flags); "
                         "r3: golden_r3.npz (bands of the headline-size frames)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--only", default=None)
    args = ap.parse_args(argv)
    out_path = args.out or str(Path(__file__).resolve().parent / {"r1": "golden.npz", "r2": "golden_r2.npz",
                                                                    "r3": "golden_r3.npz"}[args.set])
    ss = SwiftShader()
    print("renderer:", ss.renderer)
    store = {"meta_renderer": np.frombuffer(ss.renderer.encode(), dtype=np.uint8),
             "meta_skybox_shape": np.array([SKYBOX_H, SKYBOX_W], dtype=np.int32)}
    names = []
    bound = None
    for name, kind, cam, params, W, H, tr, extras in {"r1": cases, "r2": cases_r2, "r3": cases_r3}[args.set]():
        if args.only and name != args.only:
            continue
        tex_kind = extras.get("textures", "default")
        bg, arr, sizes, mx = texture_set(tex_kind)
        if bound != tex_kind:
            ss.set_textures(bg, arr)
            bound = tex_kind
        profile = extras.get("profile", "default")
        scene = scene_for(kind, sizes, mx)
        rows = extras.get("rows")
        t0 = time.time()
        img = ss.render(scene, cam, params, W, H, tr, profile=profile, rows=rows)
        dt = time.time() - t0
        if rows:
            store[f"{name}/rows"] = np.array(rows, dtype=np.int32)
        store[f"{name}/rgba8"] = img
        store[f"{name}/scene"] = sc.struct_bytes(scene)
        store[f"{name}/camera"] = sc.struct_bytes(cam)
        store[f"{name}/params"] = sc.struct_bytes(params)
        store[f"{name}/size"] = np.array([W, H], dtype=np.int32)
        store[f"{name}/test_ray"] = sc.struct_bytes(tr if tr is not None else abi.default_test_ray())
        if tex_kind != "default":
            store[f"{name}/textures"] = np.frombuffer(tex_kind.encode(), dtype=np.uint8)
        msg = f"{name:22s} {W}x{H}{' rows %d-%d' % rows if rows else ''} steps={params.max_steps} {dt:6.2f}s"
        if extras.get("steps"):
            st = ss.render(scene, cam, params, W, H, tr, steps_variant=True, profile=profile, rows=rows)
            steps = st[:, :, 0].astype(np.int32) + 256 * st[:, :, 1].astype(np.int32)
            store[f"{name}/steps"] = steps.astype(np.uint16)
            msg += f" mean_steps={steps.mean():.1f}"
        if extras.get("float"):
            store[f"{name}/rgba32"] = ss.render(scene, cam, params, W, H, tr, float_target=True, profile=profile,
                                                rows=rows)
        names.append(name)
        print(msg, flush=True)
    store["meta_cases"] = np.frombuffer("\n".join(names).encode(), dtype=np.uint8)
    np.savez_compressed(out_path, **store)
    print("wrote", out_path, Path(out_path).stat().st_size, "bytes")


if __name__ == "__main__":
    main()
