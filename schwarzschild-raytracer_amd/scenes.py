"""Scene, camera and texture builders shared by tests, golden generation,
smoke and bench.

Textures are integer-procedural (bit-reproducible anywhere) stand-ins with the
reference's shapes: the 2k skybox is 2048x1024 RGB (assets/textures/
background/2k.jpg), the texture array holds uv_checker (600x600 RGB) and
cubemap (1601x1201 RGBA), padded as loadTextureArray does
(image_utils.cpp:42-117). The reference's JPEGs are not read at run time: the
GPU box has no /root/reference.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi


# ---- textures ----------------------------------------------------------------
def skybox(width: int = 2048, height: int = 1024) -> np.ndarray:
    """RGB8 equirectangular stand-in, rows bottom-up (already 'flipped')."""
    x = np.arange(width, dtype=np.int64)[None, :]
    y = np.arange(height, dtype=np.int64)[:, None]
    r = (x * 255) // max(width - 1, 1) + 0 * y
    g = (y * 255) // max(height - 1, 1) + 0 * x
    cell = max(width // 64, 1)
    b = np.where(((x // cell) + (y // cell)) % 2 == 0, 224, 48) + 0 * x + 0 * y
    img = np.stack([r, g, b], axis=-1).astype(np.uint8)
    return np.ascontiguousarray(img)


def uv_checker(size: int = 600) -> np.ndarray:
    """RGB8 stand-in for assets/textures/uv_checker.jpg (600x600)."""
    x = np.arange(size, dtype=np.int64)[None, :]
    y = np.arange(size, dtype=np.int64)[:, None]
    cell = max(size // 10, 1)
    r = np.where(((x // cell) + (y // cell)) % 2 == 0, 230, 30) + 0 * x + 0 * y
    g = (x * 255) // max(size - 1, 1) + 0 * y
    b = (y * 255) // max(size - 1, 1) + 0 * x
    return np.ascontiguousarray(np.stack([r, g, b], axis=-1).astype(np.uint8))


def cubemap(width: int = 1601, height: int = 1201) -> np.ndarray:
    """RGBA8 stand-in for assets/textures/cubemap.png: a 4x3 cube-cross atlas,
    opaque inside the six face cells and transparent outside (the box's uv
    layout, frag:667-692)."""
    x = np.arange(width, dtype=np.int64)[None, :]
    y = np.arange(height, dtype=np.int64)[:, None]
    cx = np.minimum((x * 4) // width, 3) + 0 * y
    cy = np.minimum((y * 3) // height, 2) + 0 * x
    faces = {(1, 0), (1, 1), (1, 2), (0, 1), (2, 1), (3, 1)}
    inside = np.zeros((height, width), dtype=bool)
    for fx, fy in faces:
        inside |= (cx == fx) & (cy == fy)
    r = (40 + 50 * cx) % 256
    g = (40 + 70 * cy) % 256
    b = (((x // 25) + (y // 25)) % 2) * 180 + 40
    a = np.where(inside, 255, 0)
    return np.ascontiguousarray(np.stack([r, g, b, a], axis=-1).astype(np.uint8))


def pad_texture_array(images: list[np.ndarray]) -> tuple[np.ndarray, list[tuple[int, int]], tuple[int, int]]:
    """image_utils.cpp:42-117: pad every layer to the max size/channels;
    RGB sources get alpha 255 inside the image and 0 in the padding."""
    max_w = max(im.shape[1] for im in images)
    max_h = max(im.shape[0] for im in images)
    max_c = max(im.shape[2] for im in images)
    out_c = 4 if max_c == 4 else 3
    arr = np.zeros((len(images), max_h, max_w, out_c), dtype=np.uint8)
    sizes = []
    for i, im in enumerate(images):
        h, w, c = im.shape
        arr[i, :h, :w, :c] = im[:, :, :out_c]
        if out_c == 4 and c < 4:
            arr[i, :h, :w, 3] = 255
        sizes.append((w, h))
    return np.ascontiguousarray(arr), sizes, (max_w, max_h)


def default_texture_array():
    """The app's texture array (src/main.cpp:210-218) with stand-in pixels."""
    return pad_texture_array([uv_checker(600), cubemap(1601, 1201)])


def feature_texture_array():
    """Texture array of the material-flag scene (scene_features): layer 0 a
    smaller translucent RGBA gradient (alpha 96..208, never 255; zero-padded;
    gradients of at most ~1.3 levels per texel, so a ray that lands a small
    fraction of a texel away on another GL implementation reads nearly the
    same colour, while swapped or inverted uv still change it),
    layer 1 a full-size RGB normal map (alpha 255). Every textured hit is
    translucent, so rays go on past it under every GL filter implementation:
    SwiftShader's 16-bit filter, whose alpha is never exactly 1 (DESIGN.md
    §3), then pins the textured paths too. The normal map has no padding and
    no zero texel: planes sample it at uv beyond [0, 1] (GL_REPEAT over the
    whole layer), and normalize(0) is undefined in GLSL (frag:409)."""
    w, h = 200, 150
    x = np.arange(w, dtype=np.int64)[None, :]
    y = np.arange(h, dtype=np.int64)[:, None]
    r = 40 + (x * y * 180) // ((w - 1) * (h - 1))
    g = (x * 255) // (w - 1) + 0 * y
    b = (y * 255) // (h - 1) + 0 * x
    a = 96 + (x * 112) // (w - 1) + 0 * y
    layer0 = np.stack([r, g, b, a], axis=-1).astype(np.uint8)
    nw, nh = 256, 192
    x = np.arange(nw, dtype=np.int64)[None, :]
    y = np.arange(nh, dtype=np.int64)[:, None]
    nr = 64 + (x * 128) // (nw - 1) + 0 * y
    ng = 64 + (y * 128) // (nh - 1) + 0 * x
    nb = 200 + 0 * x + 0 * y
    layer1 = np.stack([nr, ng, nb], axis=-1).astype(np.uint8)
    return pad_texture_array([layer0, layer1])


# ---- scenes --------------------------------------------------------------------
def scene_default(textured: bool = True) -> abi.Scene:
    """src/main.cpp:222-268 packed by the library's ObjectLoader mirror."""
    s = abi.default_scene()
    if not textured:
        for m in range(abi.MAX_MATERIALS):
            s.materials[m].texture_index = -1
    return s


def scene_black_hole_only() -> abi.Scene:
    s = abi.Scene()
    abi.load().sr_scene_clear(C.byref(s))
    return s


def _rand_axes(rng, skew: bool) -> list[float]:
    """Column-major axes of a random rotation (optionally one column scaled:
    a non-orthonormal frame the culling must treat as unbounded)."""
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    m = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                  [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                  [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])
    if skew:
        m[:, rng.integers(0, 3)] *= 1.3
    return [float(np.float32(v)) for v in m.T.reshape(-1)]


def scene_random(seed: int, n_objects: int = 21, translucent: bool = True, planes: bool = True) -> abi.Scene:
    """A stress scene: up to 3 of every primitive type (21 objects: more than
    the kernel's budget slots), random poses at r in [2.5, 25], some skewed
    frames, random materials (textures, normal maps, single-sided faces,
    flipped normals, alpha < 1) and 1-4 lights."""
    rng = np.random.default_rng(seed)
    s = abi.Scene()
    abi.load().sr_scene_clear(C.byref(s))
    set_scene_texture_sizes(s, [(600, 600), (1601, 1201)], (1601, 1201))
    for m in range(abi.MAX_MATERIALS):
        mat = s.materials[m]
        for k in range(3):
            mat.color[k] = float(np.float32(rng.uniform(0.1, 1.0)))
        mat.color[3] = 1.0 if (not translucent or rng.uniform() < 0.6) else float(np.float32(rng.choice([0.0, 0.5])))
        mat.ambient = float(np.float32(rng.uniform(0.0, 0.3)))
        mat.diffuse = float(np.float32(rng.uniform(0.3, 1.0)))
        mat.specular = float(np.float32(rng.uniform(0.0, 1.0)))
        mat.shininess = float(np.float32(rng.choice([4.0, 32.0, 100.0])))
        mat.texture_index = int(rng.choice([-1, 0, 1]))
        mat.normal_map_index = int(rng.choice([-1, -1, -1, 0]))
        mat.invert_uv_x = int(rng.uniform() < 0.2)
        mat.invert_uv_y = int(rng.uniform() < 0.2)
        mat.swap_uvs = int(rng.uniform() < 0.2)
        mat.double_sided_normals = int(rng.uniform() < 0.5)
        mat.flip_normals = int(rng.uniform() < 0.2)
    s.num_lights = int(rng.integers(1, abi.MAX_LIGHTS + 1))
    for i in range(s.num_lights):
        L = s.lights[i]
        for k in range(3):
            L.transform.pos[k] = float(np.float32(rng.uniform(-15, 15)))
            L.color[k] = float(np.float32(rng.uniform(0.5, 1.0)))
        L.intensity = float(np.float32(rng.uniform(2, 10)))
        L.attenuation_constant, L.attenuation_linear, L.attenuation_quadratic = 1.0, 0.09, 0.032
    types = [t for t in range(7) for _ in range(3) if planes or t != abi.OBJECT_PLANE]
    rng.shuffle(types)
    counts = [0] * 7
    n = 0
    for t in types[:n_objects]:
        k = counts[t]
        counts[t] += 1
        v = rng.normal(size=3)
        v = v / np.linalg.norm(v) * rng.uniform(2.5, 25.0)
        skew = t in (abi.OBJECT_CYLINDER, abi.OBJECT_RECTANGLE, abi.OBJECT_BOX) and rng.uniform() < 0.2
        tr = abi.Transform()
        for i in range(3):
            tr.pos[i] = float(np.float32(v[i]))
        ax = _rand_axes(rng, skew)
        for i in range(9):
            tr.axes[i] = ax[i]

        def plane(p):
            p.transform = tr
            p.texture_offset[0] = float(np.float32(rng.uniform(-1, 1)))
            p.texture_offset[1] = float(np.float32(rng.uniform(-1, 1)))
            p.repeat_texture = int(rng.uniform() < 0.5)
            p.texture_size[0] = float(np.float32(rng.uniform(1, 4)))
            p.texture_size[1] = float(np.float32(rng.uniform(1, 4)))

        if t == abi.OBJECT_SPHERE:
            s.spheres[k].transform = tr
            s.spheres[k].radius = float(np.float32(rng.uniform(0.3, 2.5)))
        elif t == abi.OBJECT_PLANE:
            plane(s.planes[k])
        elif t == abi.OBJECT_DISK:
            plane(s.disks[k].plane)
            s.disks[k].radius = float(np.float32(rng.uniform(0.5, 3.0)))
        elif t == abi.OBJECT_HOLLOW_DISK:
            plane(s.hollow_disks[k].plane)
            r0 = rng.uniform(0.5, 3.0)
            s.hollow_disks[k].inner_radius = float(np.float32(r0))
            s.hollow_disks[k].outer_radius = float(np.float32(r0 + rng.uniform(0.5, 3.0)))
        elif t == abi.OBJECT_CYLINDER:
            s.cylinders[k].transform = tr
            s.cylinders[k].height = float(np.float32(rng.uniform(0.5, 5.0)))
            s.cylinders[k].radius = float(np.float32(rng.uniform(0.2, 2.0)))
        elif t == abi.OBJECT_RECTANGLE:
            plane(s.rectangles[k].plane)
            s.rectangles[k].width = float(np.float32(rng.uniform(0.5, 4.0)))
            s.rectangles[k].height = float(np.float32(rng.uniform(0.5, 4.0)))
        else:
            s.boxes[k].transform = tr
            s.boxes[k].width = float(np.float32(rng.uniform(0.3, 2.0)))
            s.boxes[k].depth = float(np.float32(rng.uniform(0.3, 2.0)))
            s.boxes[k].height = float(np.float32(rng.uniform(0.3, 2.0)))
        o = s.objects[n]
        o.type, o.index, o.material_index = t, k, int(rng.integers(0, abi.MAX_MATERIALS))
        n += 1
    s.num_objects = n
    return s


# The bench's max-capacity scene (bench.py --scene stress; BASELINE.md / the
# verdict's "what the default scene hides"): every capacity of the uniform
# block filled (frag:63-182): 3 of each primitive (21 objects, all of them
# budget slots of the large integrate instantiation, SR_MAX_BUDGET = 21; its
# skewed rectangle by the bounding sphere of its parallelogram since round 6,
# sr_api.cpp set_bound_corners), 10 materials, 4 lights. Fixed seed:
# tests/golden/frame_hashes.npz holds its oracle frames (configs "c2s" at
# 640x360 / 1000 steps, "c3s" at the headline 1920x1080 / 2000).
STRESS_SEED = 2024


def scene_stress() -> abi.Scene:
    s = scene_random(STRESS_SEED, n_objects=21, translucent=True, planes=True)
    s.num_lights = abi.MAX_LIGHTS
    rng = np.random.default_rng(STRESS_SEED + 1)
    for i in range(abi.MAX_LIGHTS):
        L = s.lights[i]
        for k in range(3):
            L.transform.pos[k] = float(np.float32(rng.uniform(-15, 15)))
            L.color[k] = float(np.float32(rng.uniform(0.5, 1.0)))
        L.intensity = float(np.float32(rng.uniform(2, 10)))
        L.attenuation_constant, L.attenuation_linear, L.attenuation_quadratic = 1.0, 0.09, 0.032
    return s


# The press-R overlay of the bench (bench.py --test-ray on, src/main.cpp:375-391,
# frag:760-803): the test ray traced from the app's camera position along
# (3, -2, -15) (an escaping orbit; SURVEY App. B's second ray), its first
# SR_MAX_POINTS = 1000 points as the curved polyline (1000 cylinders tested
# against every chord) and the flat ray along the same direction.
TEST_RAY_FROM = ((0.0, 2.0, 15.0), (3.0, -2.0, -15.0))
TEST_RAY_STEPS = 2700  # 1000+ points of the press-R polyline


def test_ray_overlay() -> abi.TestRay:
    cam0 = camera_look(*TEST_RAY_FROM)
    fwd = list(cam0.transform.axes[6:9])
    pts = abi.test_ray_points(list(cam0.transform.pos), fwd, TEST_RAY_STEPS, 2)[:abi.MAX_POINTS]
    tr = abi.default_test_ray()
    tr.visible = 1
    tr.num_curved_points = len(pts)
    for i, p in enumerate(pts):
        tr.curved_points[i][0], tr.curved_points[i][1], tr.curved_points[i][2] = p
    for k in range(3):
        tr.flat_origin[k] = cam0.transform.pos[k] + fwd[k]
        tr.flat_dir[k] = fwd[k]
    return tr


def _axes_from(up, ref=(1.0, 0.0, 0.0)) -> list[float]:
    """Column-major orthonormal axes with axes[1] = normalize(up) (the plane
    normal / cylinder axis) and axes[0] in the plane of ref, float32."""
    u = np.asarray(up, dtype=np.float64)
    u = u / np.linalg.norm(u)
    a = np.asarray(ref, dtype=np.float64)
    a = a - u * np.dot(a, u)
    a = a / np.linalg.norm(a)
    c = np.cross(a, u)
    return [float(np.float32(v)) for v in (*a, *u, *c)]


def scene_features() -> abi.Scene:
    """The material-flag scene pinned by SwiftShader goldens (golden_r2):
    two planes (texture offset, size, repeat on/off), every primitive type
    once, 8 materials covering the calculate_lighting paths (frag:365-438):
    translucent textures, normal maps, swap / invert uv (plane-size aware
    inversion), single-sided and flipped normals, alpha < 1 - and 4 lights
    (the reference's MAX_LIGHTS). Textures: feature_texture_array()."""
    s = abi.Scene()
    abi.load().sr_scene_clear(C.byref(s))
    set_scene_texture_sizes(s, [(200, 150), (256, 192)], (256, 192))

    def mat(m, color, tex=-1, nmap=-1, inv_x=0, inv_y=0, swap=0, double=1, flip=0, amb=0.1, dif=0.9, spec=0.5,
            shin=32.0):
        M = s.materials[m]
        for k in range(4):
            M.color[k] = float(np.float32(color[k]))
        M.ambient, M.diffuse, M.specular, M.shininess = amb, dif, spec, shin
        M.texture_index, M.normal_map_index = tex, nmap
        M.invert_uv_x, M.invert_uv_y, M.swap_uvs = inv_x, inv_y, swap
        M.double_sided_normals, M.flip_normals = double, flip

    mat(0, (0.5, 0.0, 0.5, 1.0), tex=0, inv_x=1)                      # plane 0: textured, plane-size invert x
    mat(1, (0.5, 0.0, 0.5, 1.0), tex=0, nmap=1, swap=1)               # sphere: normal map + swap
    mat(2, (0.2, 0.8, 0.3, 1.0), double=0)                            # disk: single-sided, opaque
    mat(3, (0.9, 0.6, 0.1, 0.5), double=0, flip=1)                    # hollow disk: flipped, single-sided, alpha .5
    mat(4, (0.5, 0.0, 0.5, 1.0), tex=0, nmap=1, inv_y=1, spec=0.9, shin=8.0)  # cylinder
    mat(5, (0.3, 0.4, 0.9, 0.5), spec=1.0, shin=4.0)                  # rectangle: alpha .5
    mat(6, (0.5, 0.0, 0.5, 1.0), tex=0, swap=1, inv_x=1, inv_y=1, flip=1)  # box: every uv flag, flipped
    mat(7, (0.5, 0.0, 0.5, 1.0), tex=0, nmap=1, swap=1, inv_y=1, double=0)  # plane 1: single-sided

    def tr(t, pos, axes):
        for i in range(3):
            t.pos[i] = float(np.float32(pos[i]))
        for i in range(9):
            t.axes[i] = axes[i]

    ident = [1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0]
    objs = []
    p0 = s.planes[0]
    tr(p0.transform, (0.0, -4.0, 0.0), ident)
    p0.texture_offset[0], p0.texture_offset[1] = -2.0, -1.5
    p0.repeat_texture = 0  # far, grazing hits of an infinite plane are ill-conditioned: texture a patch
    p0.texture_size[0], p0.texture_size[1] = 5.0, 4.0
    objs.append((abi.OBJECT_PLANE, 0, 0))
    p1 = s.planes[1]
    tr(p1.transform, (0.0, 0.0, -30.0), _axes_from((0.0, 0.0, 1.0)))
    p1.texture_offset[0], p1.texture_offset[1] = -0.5, 0.1
    p1.repeat_texture = 1
    p1.texture_size[0], p1.texture_size[1] = 4.0, 3.0
    objs.append((abi.OBJECT_PLANE, 1, 7))
    tr(s.spheres[0].transform, (-6.0, 1.0, 0.0), _axes_from((0.3, 1.0, 0.2)))
    s.spheres[0].radius = 1.5
    objs.append((abi.OBJECT_SPHERE, 0, 1))
    tr(s.disks[0].plane.transform, (0.0, 0.0, -8.0), _axes_from((0.4, 0.3, 1.0)))
    s.disks[0].radius = 2.0
    objs.append((abi.OBJECT_DISK, 0, 2))
    tr(s.hollow_disks[0].plane.transform, (0.0, 0.0, 0.0), _axes_from((0.05, 1.0, 0.1)))
    s.hollow_disks[0].inner_radius, s.hollow_disks[0].outer_radius = 2.5, 5.0
    objs.append((abi.OBJECT_HOLLOW_DISK, 0, 3))
    tr(s.cylinders[0].transform, (0.0, 6.0, 0.0), _axes_from((0.2, 1.0, -0.1)))
    s.cylinders[0].height, s.cylinders[0].radius = 4.0, 1.5
    objs.append((abi.OBJECT_CYLINDER, 0, 4))
    tr(s.rectangles[0].plane.transform, (3.0, -1.0, 8.0), _axes_from((0.0, 0.3, 1.0)))
    s.rectangles[0].width, s.rectangles[0].height = 3.0, 2.0
    objs.append((abi.OBJECT_RECTANGLE, 0, 5))
    tr(s.boxes[0].transform, (7.0, 0.0, -2.0), _axes_from((0.2, 1.0, 0.3), (1.0, 0.0, 1.0)))
    s.boxes[0].width, s.boxes[0].depth, s.boxes[0].height = 1.5, 1.0, 2.0
    objs.append((abi.OBJECT_BOX, 0, 6))
    for n, (t, k, m) in enumerate(objs):
        o = s.objects[n]
        o.type, o.index, o.material_index = t, k, m
    s.num_objects = len(objs)
    lights = [((10.0, 10.0, 10.0), (1.0, 1.0, 1.0), 8.0, (1.0, 0.09, 0.032)),
              ((-12.0, 4.0, 6.0), (1.0, 0.6, 0.3), 6.0, (1.0, 0.05, 0.01)),
              ((0.0, -10.0, 12.0), (0.3, 0.5, 1.0), 10.0, (0.5, 0.1, 0.02)),
              ((4.0, 15.0, -10.0), (0.8, 1.0, 0.8), 5.0, (1.0, 0.0, 0.05))]
    s.num_lights = len(lights)
    for i, (pos, col, inten, att) in enumerate(lights):
        L = s.lights[i]
        for k in range(3):
            L.transform.pos[k] = pos[k]
            L.color[k] = col[k]
        for k in range(9):
            L.transform.axes[k] = ident[k]
        L.intensity = inten
        L.attenuation_constant, L.attenuation_linear, L.attenuation_quadratic = att
    return s


def set_scene_texture_sizes(s: abi.Scene, sizes, max_size) -> None:
    for i, (w, h) in enumerate(sizes):
        s.texture_sizes[i][0] = float(w)
        s.texture_sizes[i][1] = float(h)
    s.max_texture_size[0] = float(max_size[0])
    s.max_texture_size[1] = float(max_size[1])


# ---- cameras -------------------------------------------------------------------
def _f32(x) -> np.float32:
    return np.float32(x)


def _normalize(v: np.ndarray) -> np.ndarray:
    v = v.astype(np.float32)
    d = np.float32(np.float32(v[0] * v[0]) + np.float32(v[1] * v[1])) + np.float32(v[2] * v[2])
    k = np.float32(np.float32(1.0) / np.float32(np.sqrt(d)))
    return (v * k).astype(np.float32)


def _cross(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    return np.array(
        [
            np.float32(a[1] * b[2]) - np.float32(b[1] * a[2]),
            np.float32(a[2] * b[0]) - np.float32(b[2] * a[0]),
            np.float32(a[0] * b[1]) - np.float32(b[0] * a[1]),
        ],
        dtype=np.float32,
    )


def camera_look(pos, forward, right=None, fov: float = 90.0) -> abi.Camera:
    """Camera(pos, forward, right) (camera.cpp:7-11); right defaults to
    normalize(cross(forward, up)) as Camera::lookAt (camera.cpp:35-39)."""
    pos = np.asarray(pos, dtype=np.float32)
    f = _normalize(np.asarray(forward, dtype=np.float32))
    if right is None:
        right = _cross(f, np.array([0, 1, 0], dtype=np.float32))
        if float(np.dot(right, right)) < 1e-12:
            right = np.array([1, 0, 0], dtype=np.float32)
    r_raw = np.asarray(right, dtype=np.float32)
    r = _normalize(r_raw)
    u = _normalize(_cross(r_raw, f))
    cam = abi.Camera()
    for i in range(3):
        cam.transform.pos[i] = float(pos[i])
        cam.transform.axes[i] = float(r[i])
        cam.transform.axes[3 + i] = float(u[i])
        cam.transform.axes[6 + i] = float(f[i])
    cam.fov = float(fov)
    return cam


def random_camera(seed: int) -> abi.Camera:
    """SURVEY §8d parity sweep: r ~ U[3, 50], direction uniform on S^2,
    fov in {60, 90}; the camera looks at the hole with a random offset."""
    rng = np.random.default_rng(seed)
    r = rng.uniform(3.0, 50.0)
    v = rng.normal(size=3)
    v /= np.linalg.norm(v)
    pos = (v * r).astype(np.float32)
    target = rng.normal(size=3) * 0.35 * r
    fwd = (target - pos).astype(np.float32)
    fov = 60.0 if rng.integers(0, 2) == 0 else 90.0
    return camera_look(pos, fwd, fov=fov)


def camera_to_dict(cam: abi.Camera) -> dict:
    return {"pos": list(cam.transform.pos), "axes": list(cam.transform.axes), "fov": cam.fov}


def camera_from_arrays(pos, axes, fov) -> abi.Camera:
    cam = abi.Camera()
    for i in range(3):
        cam.transform.pos[i] = float(pos[i])
    for i in range(9):
        cam.transform.axes[i] = float(axes[i])
    cam.fov = float(fov)
    return cam


def struct_bytes(s) -> np.ndarray:
    return np.frombuffer(bytes(memoryview(s)), dtype=np.uint8).copy()


def struct_from_bytes(cls, data: np.ndarray):
    obj = cls()
    b = bytes(np.asarray(data, dtype=np.uint8))
    if len(b) != C.sizeof(cls):
        raise ValueError(f"{cls.__name__}: {len(b)} bytes, expected {C.sizeof(cls)}")
    C.memmove(C.addressof(obj), b, len(b))
    return obj
