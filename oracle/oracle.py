"""ctypes binding of the CPU ORACLE (oracle/sr_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() (as the
checker) and bench.py's cpu_baseline leg. The product never imports it.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

import srpkg

abi = srpkg.load_package().abi

LIB_PATH = Path(__file__).resolve().parent / "build" / "libsr_oracle.so"
LIB_O0_PATH = Path(__file__).resolve().parent / "build" / "libsr_oracle_O0.so"  # bench cpu_baseline -O0 leg


class Textures(C.Structure):
    _fields_ = [
        ("bg", C.c_void_p),
        ("bg_w", C.c_int),
        ("bg_h", C.c_int),
        ("bg_channels", C.c_int),
        ("arr", C.c_void_p),
        ("arr_w", C.c_int),
        ("arr_h", C.c_int),
        ("arr_layers", C.c_int),
        ("arr_channels", C.c_int),
    ]


_lib = None


def load() -> C.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise FileNotFoundError(f"{LIB_PATH} not built; run make -C oracle")
        lib = C.CDLL(str(LIB_PATH))
        lib.sro_render.restype = C.c_int
        lib.sro_render.argtypes = [C.POINTER(abi.Scene), C.POINTER(abi.TestRay), C.POINTER(Textures),
                                   C.POINTER(abi.Camera), C.POINTER(abi.Params), C.c_int, C.c_int, C.c_int,
                                   C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        lib.sro_shade_pixel.restype = C.c_int
        lib.sro_shade_pixel.argtypes = [C.POINTER(abi.Scene), C.POINTER(abi.TestRay), C.POINTER(Textures),
                                        C.POINTER(abi.Camera), C.POINTER(abi.Params), C.c_int, C.c_int, C.c_int,
                                        C.c_int, C.POINTER(C.c_float)]
        lib.sro_test_ray_points.restype = C.c_int
        lib.sro_test_ray_points.argtypes = [C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_int, C.c_int,
                                            C.POINTER(C.c_float), C.c_int]
        lib.sro_pressr_sweep.restype = C.c_int64
        lib.sro_pressr_sweep.argtypes = [C.POINTER(abi.Camera), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                         C.c_int, C.c_int]
        lib.sro_sample_texture.restype = C.c_int
        lib.sro_sample_texture.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_float, C.c_float, C.c_int,
                                           C.POINTER(C.c_float)]
        lib.sro_pressr_ray_repeat.restype = C.c_int
        lib.sro_pressr_ray_repeat.argtypes = [C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_int, C.c_int, C.c_int]
        _lib = lib
    return _lib


# filter_mode of the oracle only: SwiftShader 4.1's fixed-point sampler (test infrastructure)
FILTER_SWIFTSHADER = 2


def sample_texture(img: np.ndarray, u: float, v: float, mode: int) -> np.ndarray:
    """One texture() lookup of the oracle's sampler on an [H, W, C] uint8 image."""
    a = np.ascontiguousarray(img, dtype=np.uint8)
    out = (C.c_float * 4)()
    rc = load().sro_sample_texture(a.ctypes.data, a.shape[1], a.shape[0], a.shape[2], float(u), float(v), int(mode),
                                   out)
    assert rc == 0
    return np.frombuffer(out, dtype=np.float32).copy()


class TextureSet:
    """Keeps numpy buffers alive for the Textures struct."""

    def __init__(self, bg: np.ndarray | None = None, arr: np.ndarray | None = None):
        self.bg = None if bg is None else np.ascontiguousarray(bg, dtype=np.uint8)
        self.arr = None if arr is None else np.ascontiguousarray(arr, dtype=np.uint8)
        t = Textures()
        if self.bg is not None:
            t.bg = self.bg.ctypes.data
            t.bg_h, t.bg_w, t.bg_channels = self.bg.shape
        if self.arr is not None:
            t.arr = self.arr.ctypes.data
            t.arr_layers, t.arr_h, t.arr_w, t.arr_channels = self.arr.shape
        self.struct = t


def render(scene, cam, params, width, height, textures: TextureSet | None = None, test_ray=None,
           row_begin=0, row_end=None, nthreads=0):
    """-> (rgba8 [rows, W, 4] uint8, rgba32 [rows, W, 4] float32, steps [rows, W] int32)."""
    lib = load()
    row_end = height if row_end is None else row_end
    rows = row_end - row_begin
    rgba8 = np.zeros((rows, width, 4), dtype=np.uint8)
    rgba32 = np.zeros((rows, width, 4), dtype=np.float32)
    steps = np.zeros((rows, width), dtype=np.int32)
    tex = textures or TextureSet()
    tr = test_ray if test_ray is not None else abi.default_test_ray()
    rc = lib.sro_render(C.byref(scene), C.byref(tr), C.byref(tex.struct), C.byref(cam), C.byref(params), width,
                        height, row_begin, row_end, rgba8.ctypes.data, rgba32.ctypes.data, steps.ctypes.data,
                        nthreads)
    if rc != 0:
        raise RuntimeError(f"sro_render failed: {rc}")
    return rgba8, rgba32, steps


def shade_pixel(scene, cam, params, width, height, px, py, textures: TextureSet | None = None, test_ray=None):
    lib = load()
    out = (C.c_float * 4)()
    tex = textures or TextureSet()
    tr = test_ray if test_ray is not None else abi.default_test_ray()
    n = lib.sro_shade_pixel(C.byref(scene), C.byref(tr), C.byref(tex.struct), C.byref(cam), C.byref(params),
                            width, height, px, py, out)
    return list(out), n


def test_ray_points(pos, forward, max_steps, max_revolutions=2):
    lib = load()
    cap = max_steps + 2
    buf = (C.c_float * (3 * cap))()
    n = lib.sro_test_ray_points((C.c_float * 3)(*pos), (C.c_float * 3)(*forward), max_steps, max_revolutions,
                                buf, cap)
    return [(buf[3 * i], buf[3 * i + 1], buf[3 * i + 2]) for i in range(min(n, cap))]


def pressr_ray_repeat(pos, forward, max_steps, max_revolutions=2, reps=1) -> int:
    """One press-R ray (a std::vector of points per trace, src/main.cpp:94-124)
    traced `reps` times on the calling thread; returns its point count."""
    lib = load()
    return int(lib.sro_pressr_ray_repeat((C.c_float * 3)(*pos), (C.c_float * 3)(*forward), max_steps,
                                         max_revolutions, reps))


_lib_O0 = None


def pressr_sweep_O0(cam, width, height, max_steps, max_revolutions=2, row_begin=0, row_end=None, nthreads=0) -> int:
    """pressr_sweep built at -O0 (the reference's CMake default)."""
    global _lib_O0
    if _lib_O0 is None:
        if not LIB_O0_PATH.exists():
            raise FileNotFoundError(f"{LIB_O0_PATH} not built; run make -C oracle")
        lib = C.CDLL(str(LIB_O0_PATH))
        lib.sro_pressr_sweep.restype = C.c_int64
        lib.sro_pressr_sweep.argtypes = [C.POINTER(abi.Camera), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                         C.c_int, C.c_int]
        _lib_O0 = lib
    row_end = height if row_end is None else row_end
    return int(_lib_O0.sro_pressr_sweep(C.byref(cam), width, height, row_begin, row_end, max_steps, max_revolutions,
                                        nthreads))


def pressr_sweep(cam, width, height, max_steps, max_revolutions=2, row_begin=0, row_end=None, nthreads=0) -> int:
    lib = load()
    row_end = height if row_end is None else row_end
    return int(lib.sro_pressr_sweep(C.byref(cam), width, height, row_begin, row_end, max_steps, max_revolutions,
                                    nthreads))
