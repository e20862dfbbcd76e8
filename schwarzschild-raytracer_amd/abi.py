"""ctypes mirror of include/sr/sr.h and the loader for libsr.so.

The structs are field-for-field copies of the C-ABI (which itself mirrors the
GLSL uniform block of the reference's assets/shaders/black_hole.frag:15-192);
`check_layout()` compares every size against the compiled library.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
LIB_PATH = PKG_DIR / "lib" / "libsr.so"

MAX_LIGHTS = 4
MAX_TEXTURES = 10
MAX_MATERIALS = 10
MAX_SPHERES = 3
MAX_PLANES = 3
MAX_DISKS = 3
MAX_HOLLOW_DISKS = 3
MAX_CYLINDERS = 3
MAX_RECTANGLES = 3
MAX_BOXES = 3
MAX_OBJECTS = 21
MAX_POINTS = 1000
# floats per pixel of the integrate -> shade hand-off (csrc/device_scene.h SR_PS_FIELDS)
PS_FIELDS = 4 + 8 * 4 + 16

OBJECT_SPHERE, OBJECT_PLANE, OBJECT_DISK, OBJECT_HOLLOW_DISK = 0, 1, 2, 3
OBJECT_CYLINDER, OBJECT_RECTANGLE, OBJECT_BOX = 4, 5, 6
RAYTRACE_CURVED, RAYTRACE_FLAT, RAYTRACE_HALF_WIDTH, RAYTRACE_HALF_HEIGHT = 0, 1, 2, 3
FILTER_LERP, FILTER_WEIGHTED = 0, 1

SR_OK = 0
SR_E_INVALID = -1
SR_E_CAPACITY = -2
SR_E_HIP = -3
SR_E_NOMEM = -4
SR_E_NOT_READY = -5
SR_E_NO_DEVICE = -6
SR_E_IO = -7

F3 = C.c_float * 3
F9 = C.c_float * 9


class Transform(C.Structure):
    _fields_ = [("pos", F3), ("axes", F9)]


class Camera(C.Structure):
    _fields_ = [("transform", Transform), ("fov", C.c_float)]


class Light(C.Structure):
    _fields_ = [
        ("transform", Transform),
        ("color", F3),
        ("intensity", C.c_float),
        ("attenuation_constant", C.c_float),
        ("attenuation_linear", C.c_float),
        ("attenuation_quadratic", C.c_float),
    ]


class Material(C.Structure):
    _fields_ = [
        ("color", C.c_float * 4),
        ("ambient", C.c_float),
        ("diffuse", C.c_float),
        ("specular", C.c_float),
        ("shininess", C.c_float),
        ("texture_index", C.c_int32),
        ("normal_map_index", C.c_int32),
        ("invert_uv_x", C.c_int32),
        ("invert_uv_y", C.c_int32),
        ("swap_uvs", C.c_int32),
        ("double_sided_normals", C.c_int32),
        ("flip_normals", C.c_int32),
    ]


class Sphere(C.Structure):
    _fields_ = [("transform", Transform), ("radius", C.c_float)]


class Plane(C.Structure):
    _fields_ = [
        ("transform", Transform),
        ("texture_offset", C.c_float * 2),
        ("repeat_texture", C.c_int32),
        ("texture_size", C.c_float * 2),
    ]


class Disk(C.Structure):
    _fields_ = [("plane", Plane), ("radius", C.c_float)]


class HollowDisk(C.Structure):
    _fields_ = [("plane", Plane), ("inner_radius", C.c_float), ("outer_radius", C.c_float)]


class Cylinder(C.Structure):
    _fields_ = [("transform", Transform), ("height", C.c_float), ("radius", C.c_float)]


class Rectangle(C.Structure):
    _fields_ = [("plane", Plane), ("width", C.c_float), ("height", C.c_float)]


class Box(C.Structure):
    _fields_ = [("transform", Transform), ("width", C.c_float), ("depth", C.c_float), ("height", C.c_float)]


class Object(C.Structure):
    _fields_ = [("type", C.c_int32), ("index", C.c_int32), ("material_index", C.c_int32)]


class Scene(C.Structure):
    _fields_ = [
        ("num_objects", C.c_int32),
        ("objects", Object * MAX_OBJECTS),
        ("spheres", Sphere * MAX_SPHERES),
        ("planes", Plane * MAX_PLANES),
        ("disks", Disk * MAX_DISKS),
        ("hollow_disks", HollowDisk * MAX_HOLLOW_DISKS),
        ("cylinders", Cylinder * MAX_CYLINDERS),
        ("rectangles", Rectangle * MAX_RECTANGLES),
        ("boxes", Box * MAX_BOXES),
        ("materials", Material * MAX_MATERIALS),
        ("num_lights", C.c_int32),
        ("lights", Light * MAX_LIGHTS),
        ("texture_sizes", (C.c_float * 2) * MAX_TEXTURES),
        ("max_texture_size", C.c_float * 2),
    ]


class Params(C.Structure):
    _fields_ = [
        ("max_steps", C.c_int32),
        ("max_revolutions", C.c_int32),
        ("u_f", C.c_float),
        ("crosshair", C.c_int32),
        ("raytrace_type", C.c_int32),
        ("curved_percentage", C.c_float),
        ("percent_black", C.c_float),
        ("time", C.c_float),
        ("filter_mode", C.c_int32),
    ]


class TestRay(C.Structure):
    _fields_ = [
        ("visible", C.c_int32),
        ("radius", C.c_float),
        ("extended_length", C.c_float),
        ("curved_color", C.c_float * 4),
        ("flat_color", C.c_float * 4),
        ("flat_origin", F3),
        ("flat_dir", F3),
        ("num_curved_points", C.c_int32),
        ("curved_points", F3 * MAX_POINTS),
    ]


# Functions declared in include/sr/sr.h: name -> (restype, argtypes)
_p = C.c_void_p
_i = C.c_int
SIGNATURES = {
    "sr_version": (C.c_char_p, []),
    "sr_status_string": (C.c_char_p, [_i]),
    "sr_params_default": (None, [C.POINTER(Params)]),
    "sr_test_ray_default": (None, [C.POINTER(TestRay)]),
    "sr_scene_clear": (None, [C.POINTER(Scene)]),
    "sr_default_scene": (None, [C.POINTER(Scene)]),
    "sr_default_camera": (None, [C.POINTER(Camera)]),
    "sr_camera_hyperbolic_trajectory": (C.c_int, [C.POINTER(Camera), C.c_float, C.c_float, C.c_float]),
    "sr_create": (_i, [C.POINTER(_p), _i]),
    "sr_destroy": (None, [_p]),
    "sr_set_background": (_i, [_p, _p, _i, _i, _i]),
    "sr_set_texture_array": (_i, [_p, _p, _i, _i, _i, _i]),
    "sr_set_scene": (_i, [_p, C.POINTER(Scene)]),
    "sr_set_test_ray": (_i, [_p, C.POINTER(TestRay)]),
    "sr_render": (_i, [_p, C.POINTER(Camera), C.POINTER(Params), _i, _i, _i, _i, _p, C.c_size_t, _p]),
    "sr_render_blocks": (_i, [_p, C.POINTER(Camera), C.POINTER(Params), _i, _i, _i, _i, _i, _p, C.c_size_t, _p]),
    "sr_render_debug": (_i, [_p, C.POINTER(Camera), C.POINTER(Params), _i, _i, _i, _i, _p, _p, _p, _p]),
    "sr_blocks_row_count": (_i, [_i, _i, _i, _i]),
    "sr_set_split": (_i, [_p, _i, _i, _i]),
    "sr_set_latency_mode": (_i, [_p, _i]),
    "sr_write_png": (_i, [C.c_char_p, _p, _i, _i, C.c_size_t, _i]),
    "sr_render_blocks_batch": (_i, [_p, C.POINTER(Camera), _i, C.POINTER(Params), _i, _i, _i, _i, _i, _p,
                                    C.c_size_t, C.c_size_t, _p]),
    "sr_wave_costs": (_i, [_p, C.POINTER(Camera), C.POINTER(Params), _i, _i, _p, _p]),
    "sr_render_block_list": (_i, [_p, C.POINTER(Camera), _i, C.POINTER(Params), _i, _i, _i, C.POINTER(_i), _i, _p,
                                  C.c_size_t, C.c_size_t, _p]),
    "sr_abi_struct_sizes": (_i, [C.POINTER(C.c_size_t), _i]),
    "sr_diag_counters": (_i, [_p, C.POINTER(C.c_int64), _i]),
    "sr_test_ray_points": (_i, [C.POINTER(C.c_float), C.POINTER(C.c_float), _i, _i, C.POINTER(C.c_float), _i, C.POINTER(_i)]),
    "sr_block_costs": (_i, [_p, _i, _i, C.c_double, _p]),
    "sr_balanced_blocks": (_i, [_p, _i, _i, _p, _i, C.POINTER(_i)]),
    "sr_assemble_blocks": (_i, [_p, C.c_size_t, C.c_size_t, _p, _i, _i, _i, _i, C.c_size_t, _p, C.c_size_t, _i, _i,
                                _p]),
}
# exported beside the header set (parity tooling)
EXTRA_SIGNATURES = {
    "sr_debug_set_culling": (_i, [_p, _i]),
    "sr_debug_set_timing": (_i, [_p, _i]),
    "sr_debug_kernel_times": (_i, [_p, C.POINTER(C.c_float), _i, C.POINTER(_i)]),
    "sr_debug_last_order": (_i, [_p, C.POINTER(_i), _i, C.POINTER(_i)]),
    "sr_debug_pixel_state": (_i, [_p, C.POINTER(C.c_float), C.c_size_t, C.POINTER(C.c_size_t)]),
}

_lib = None


class SRError(RuntimeError):
    def __init__(self, status: int, what: str):
        super().__init__(f"{what}: {status_string(status)} ({status})")
        self.status = status


def load(path: str | os.PathLike | None = None) -> C.CDLL:
    """Load libsr.so (built in-tree by `make -C schwarzschild-raytracer_amd`).

    Raises FileNotFoundError when the library has not been built: there is no
    fallback implementation.
    """
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path else Path(os.environ.get("SR_LIB", LIB_PATH))
    if not p.exists():
        raise FileNotFoundError(f"{p} not built; run __graft_entry__.build() or make -C schwarzschild-raytracer_amd")
    lib = C.CDLL(str(p), mode=C.RTLD_GLOBAL)
    for name, (res, args) in {**SIGNATURES, **EXTRA_SIGNATURES}.items():
        if name in EXTRA_SIGNATURES and not hasattr(lib, name):
            continue  # debug tooling an older library (a bisection build) may lack
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def status_string(status: int) -> str:
    try:
        return load().sr_status_string(status).decode()
    except Exception:  # noqa: BLE001 - best effort in error paths
        return "status"


def check(status: int, what: str) -> None:
    if status != SR_OK:
        raise SRError(status, what)


def write_png(path, frame, flip_rows: bool = True) -> None:
    """sr_write_png: an [H, W, 4] uint8 frame (host array; rows bottom-up as
    sr_render leaves them when flip_rows) as an RGBA8 PNG."""
    import numpy as np

    a = np.ascontiguousarray(frame, dtype=np.uint8)
    if a.ndim != 3 or a.shape[2] != 4:
        raise ValueError(f"expected an [H, W, 4] frame, got {a.shape}")
    h, w, _ = a.shape
    check(load().sr_write_png(str(path).encode(), a.ctypes.data, w, h, w * 4, 1 if flip_rows else 0), "sr_write_png")


def check_layout() -> dict:
    lib = load()
    out = (C.c_size_t * 6)()
    check(lib.sr_abi_struct_sizes(out, 6), "sr_abi_struct_sizes")
    got = dict(zip(["camera", "params", "scene", "test_ray", "material", "light"], list(out)))
    want = {
        "camera": C.sizeof(Camera),
        "params": C.sizeof(Params),
        "scene": C.sizeof(Scene),
        "test_ray": C.sizeof(TestRay),
        "material": C.sizeof(Material),
        "light": C.sizeof(Light),
    }
    if got != want:
        raise AssertionError(f"ctypes layout mismatch: C {got} vs ctypes {want}")
    return got


def default_params(**overrides) -> Params:
    p = Params()
    load().sr_params_default(C.byref(p))
    for k, v in overrides.items():
        setattr(p, k, v)
    return p


def default_test_ray() -> TestRay:
    t = TestRay()
    load().sr_test_ray_default(C.byref(t))
    return t


def default_scene() -> Scene:
    s = Scene()
    load().sr_default_scene(C.byref(s))
    return s


def default_camera() -> Camera:
    c = Camera()
    load().sr_default_camera(C.byref(c))
    return c


def camera_flyby(t: float, initial_distance: float = 30.0, closest_distance: float = 10.0,
                 cam: Camera | None = None) -> Camera:
    """The app's H-key flyby camera at eased time t in [0, 1] (src/main.cpp:404-410:
    Camera::hyperbolicTrajectory(30, 10, t), camera.cpp:20-39)."""
    src = cam if cam is not None else default_camera()
    c = Camera()
    C.memmove(C.addressof(c), C.addressof(src), C.sizeof(Camera))
    check(load().sr_camera_hyperbolic_trajectory(C.byref(c), initial_distance, closest_distance, t),
          "sr_camera_hyperbolic_trajectory")
    return c


def test_ray_points(pos, forward, max_steps: int, max_revolutions: int = 2):
    """Host press-R geodesic (src/main.cpp:94-124) -> list of (x, y, z)."""
    lib = load()
    cap = max_steps + 2
    buf = (C.c_float * (3 * cap))()
    n = C.c_int()
    check(
        lib.sr_test_ray_points((C.c_float * 3)(*pos), (C.c_float * 3)(*forward), max_steps, max_revolutions, buf, cap, C.byref(n)),
        "sr_test_ray_points",
    )
    return [(buf[3 * i], buf[3 * i + 1], buf[3 * i + 2]) for i in range(min(n.value, cap))]
