"""HIP kernel (libsr.so, via the C-ABI) vs the CPU oracle.

Contract: both sides evaluate the reference shader's float32
expressions in the same order with the same rounding, so outputs are
bit-identical: float FragColor, RGBA8 pixel and executed step count, asserted
exactly (no pixel may differ). The binary64 transcendentals (glibc on the
host, ocml on the device) round to the same binary32 on every input these
tests and the full-frame fixtures (tests/test_gpu_frames.py) reach.
"""
import numpy as np
import pytest

from conftest import case_rows, case_texture_kind, load_case, texture_array_of

pytestmark = pytest.mark.gpu



@pytest.fixture(scope="module")
def gpu(pkg, textures):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    bg, arr = textures
    r = pkg.Renderer(0)
    r.set_background(bg)
    r.set_texture_array(arr)
    yield r
    r.close()


def gpu_debug(gpu, scene, cam, params, w, h, test_ray=None, row_begin=0, row_end=None):
    import torch

    gpu.set_scene(scene)
    gpu.set_test_ray(test_ray if test_ray is not None else gpu_default_test_ray())
    f, b, s = gpu.render_debug(cam, params, w, h, row_begin, row_end)
    torch.cuda.synchronize()
    return b.cpu().numpy(), f.cpu().numpy(), s.cpu().numpy()


def gpu_default_test_ray():
    import srpkg

    return srpkg.load_package().abi.default_test_ray()


def compare(gpu_out, ora_out, label):
    b, f, s = gpu_out
    rb, rf, rs = ora_out
    px_diff = (b != rb).any(-1)
    n = px_diff.size
    frac = px_diff.mean()
    steps_frac = (s != rs).mean()
    fbits = (f.view(np.uint32) != rf.view(np.uint32)).any(-1) & ~(np.isnan(f).any(-1) & np.isnan(rf).any(-1))
    msg = (f"{label}: rgba8 differ {px_diff.sum()}/{n}, float-bits differ {fbits.sum()}, "
           f"steps differ {(s != rs).sum()}, max byte diff {np.abs(b.astype(int) - rb.astype(int)).max()}")
    assert frac == 0, msg
    assert steps_frac == 0, msg
    assert fbits.sum() == 0, msg
    return msg


@pytest.fixture(scope="module")
def oracle_tex(oracle, textures):
    bg, arr = textures
    return oracle.TextureSet(bg, arr)


def test_golden_cases_bit_exact(pkg, oracle, golden, golden_cases, textures):
    """Every golden case (golden.npz, golden_r2.npz: the reseed branch,
    config 2 at full size, the material-flag scene; golden_r3.npz: bands of
    the headline-size frames), GPU == oracle."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    bg, _ = textures
    by_kind = {}
    for name in golden_cases:
        by_kind.setdefault(case_texture_kind(golden, name), []).append(name)
    for kind, names in by_kind.items():
        arr = texture_array_of(pkg, kind)
        r = pkg.Renderer(0)
        r.set_background(bg)
        r.set_texture_array(arr)
        otex = oracle.TextureSet(bg, arr)
        for name in names:
            scene, cam, params, tr, w, h = load_case(pkg, golden, name)
            y0, y1 = case_rows(golden, name, h)
            g = gpu_debug(r, scene, cam, params, w, h, tr, y0, y1)
            o = oracle.render(scene, cam, params, w, h, otex, tr, y0, y1)
            print(compare(g, o, name))
            if name.startswith(("reseed", "config2", "band")):
                assert (g[2] != o[2]).sum() == 0, f"{name}: step counts differ"
        r.close()


@pytest.mark.parametrize("seed", range(1, 17))
def test_random_cameras(pkg, gpu, oracle, oracle_tex, seed):
    sc, abi = pkg.scenes, pkg.abi
    scene = sc.scene_default(textured=bool(seed % 2))
    cam = sc.random_camera(100 + seed)
    params = abi.default_params(max_steps=400, percent_black=-1.0)
    g = gpu_debug(gpu, scene, cam, params, 80, 60)
    o = oracle.render(scene, cam, params, 80, 60, oracle_tex)
    compare(g, o, f"seed {seed}")


@pytest.mark.parametrize("mode,cp", [(0, 0.5), (1, 0.5), (2, 0.37), (3, 0.61)])
@pytest.mark.parametrize("filter_mode", [0, 1])
def test_modes_and_filters(pkg, gpu, oracle, oracle_tex, mode, cp, filter_mode):
    sc, abi = pkg.scenes, pkg.abi
    scene = sc.scene_default(textured=True)
    cam = abi.default_camera()
    params = abi.default_params(max_steps=600, percent_black=-1.0, raytrace_type=mode, curved_percentage=cp,
                                filter_mode=filter_mode, crosshair=1)
    g = gpu_debug(gpu, scene, cam, params, 96, 54)
    o = oracle.render(scene, cam, params, 96, 54, oracle_tex)
    compare(g, o, f"mode {mode} filter {filter_mode}")


def test_noise_mask(pkg, gpu, oracle, oracle_tex):
    sc, abi = pkg.scenes, pkg.abi
    scene = sc.scene_default(textured=True)
    cam = abi.default_camera()
    params = abi.default_params(max_steps=500, percent_black=0.75)
    g = gpu_debug(gpu, scene, cam, params, 128, 72)
    o = oracle.render(scene, cam, params, 128, 72, oracle_tex)
    compare(g, o, "noise mask")
    black = (g[0][..., :3] == 0).all(-1).mean()
    assert 0.6 < black < 0.95


def test_test_ray_overlay(pkg, gpu, oracle, oracle_tex):
    """Press-R overlay (src/main.cpp:375-391, frag:760-803) with a long polyline."""
    sc, abi = pkg.scenes, pkg.abi
    cam0 = sc.camera_look((3.0, 2.0, 14.0), (-0.2, -0.1, -1.0))
    fwd = list(cam0.transform.axes[6:9])
    pts = abi.test_ray_points(list(cam0.transform.pos), fwd, 200, 2)
    tr = abi.default_test_ray()
    tr.visible = 1
    tr.num_curved_points = len(pts)
    for i, p in enumerate(pts):
        tr.curved_points[i][0], tr.curved_points[i][1], tr.curved_points[i][2] = p
    for k in range(3):
        tr.flat_origin[k] = cam0.transform.pos[k] + fwd[k]
        tr.flat_dir[k] = fwd[k]
    view = sc.camera_look((8.0, 6.0, 20.0), (-8.0, -6.0, -20.0))
    scene = sc.scene_default(textured=False)
    params = abi.default_params(max_steps=200, percent_black=-1.0)
    g = gpu_debug(gpu, scene, view, params, 64, 36, tr)
    o = oracle.render(scene, view, params, 64, 36, oracle_tex, tr)
    compare(g, o, "test ray")
    gpu.set_test_ray(abi.default_test_ray())


@pytest.mark.parametrize("seed", range(6))
def test_culling_is_exact(pkg, gpu, seed):
    """Segment culling must not change a single bit (1080p-like aspect)."""
    import torch

    sc, abi = pkg.scenes, pkg.abi
    scene = sc.scene_default(textured=True)
    cam = abi.default_camera() if seed == 0 else sc.random_camera(200 + seed)
    params = abi.default_params(max_steps=1000, percent_black=-1.0)
    gpu.set_scene(scene)
    outs = []
    for cull in (True, False):
        gpu.set_culling(cull)
        f, b, s = gpu.render_debug(cam, params, 480, 270)
        torch.cuda.synchronize()
        outs.append((f.cpu().numpy().view(np.uint32), b.cpu().numpy(), s.cpu().numpy()))
    gpu.set_culling(True)
    assert np.array_equal(outs[0][0], outs[1][0])
    assert np.array_equal(outs[0][1], outs[1][1])
    assert np.array_equal(outs[0][2], outs[1][2])


@pytest.mark.parametrize("lanes", [16, 4, 1])
def test_split_tiles_bit_identical(pkg, gpu, lanes):
    """Split tiles (sr_set_split) change which rays share a wave, never a
    pixel: the costliest tiles of the previous frame, re-run as waves of 16,
    4 or 1 rays, give the same float FragColor, RGBA8 and step counts as whole
    tiles - full frames, a row band and a block-cyclic share."""
    import torch

    sc, abi = pkg.scenes, pkg.abi
    gpu.set_scene(sc.scene_default(textured=True))
    gpu.set_test_ray(abi.default_test_ray())
    params = abi.default_params(max_steps=2000, percent_black=-1.0)

    def frame(cam, W, H, rows):
        f, b, s = gpu.render_debug(cam, params, W, H, *rows)
        torch.cuda.synchronize()
        return f.cpu().numpy().view(np.uint32), b.cpu().numpy(), s.cpu().numpy()

    cases = [(abi.default_camera(), 480, 270, (0, None)), (sc.random_camera(7), 320, 200, (0, None)),
             (abi.default_camera(), 640, 360, (96, 224))]
    for cam, W, H, rows in cases:
        gpu.set_split(0)
        ref = frame(cam, W, H, rows)
        gpu.set_split(24, lanes, 1)
        frame(cam, W, H, rows)  # learns the tile costs (centre-out order, nothing split yet)
        codes = gpu.last_order()
        n_split = int(((codes >= 0) & ((codes & 0x80) != 0)).sum())
        assert n_split == 24 * (64 // lanes), (n_split, codes[:8])
        got = frame(cam, W, H, rows)  # runs the split launch
        gpu.set_split(0)
        for a, b_, what in zip(ref, got, ("float", "rgba8", "steps")):
            assert np.array_equal(a, b_), f"{what} differs with split tiles ({lanes} lanes, {W}x{H} rows {rows})"
    # the multi-GPU share path
    cam = abi.default_camera()
    gpu.set_split(0)
    ref, rows = gpu.render_blocks(cam, params, 480, 270, 8, 1, 4)
    ref = ref.cpu().numpy()
    gpu.set_split(16, lanes, 1)
    for _ in range(2):
        got, _ = gpu.render_blocks(cam, params, 480, 270, 8, 1, 4)
    gpu.set_split(0)
    torch.cuda.synchronize()
    assert np.array_equal(ref[:rows], got.cpu().numpy()[:rows])


def test_latency_mode_bit_identical(pkg, gpu):
    """sr_set_latency_mode (the integrate kernel's 2-step fast-loop
    instantiation) changes how many steps one fast-loop iteration runs, never
    a pixel: float FragColor, RGBA8 and step counts equal the default
    kernel's (which the other tests hold to the oracle), alone and with split
    tiles."""
    import torch

    sc, abi = pkg.scenes, pkg.abi
    gpu.set_scene(sc.scene_default(textured=True))
    gpu.set_test_ray(abi.default_test_ray())
    params = abi.default_params(max_steps=2000, percent_black=-1.0)

    def frame(cam, W, H):
        f, b, s = gpu.render_debug(cam, params, W, H)
        torch.cuda.synchronize()
        return f.cpu().numpy().view(np.uint32), b.cpu().numpy(), s.cpu().numpy()

    for cam, W, H in ((abi.default_camera(), 480, 270), (sc.random_camera(11), 320, 200)):
        gpu.set_latency_mode(False)
        ref = frame(cam, W, H)
        gpu.set_latency_mode(True)
        got = frame(cam, W, H)
        gpu.set_split(24, 16, 1)
        frame(cam, W, H)  # learns the costs
        got_split = frame(cam, W, H)
        gpu.set_split(0)
        gpu.set_latency_mode(False)
        for a, b_, c_, what in zip(ref, got, got_split, ("float", "rgba8", "steps")):
            assert np.array_equal(a, b_), f"{what} differs in latency mode ({W}x{H})"
            assert np.array_equal(a, c_), f"{what} differs in latency mode with split tiles ({W}x{H})"


@pytest.mark.parametrize("split,mode", [(0, 0), (12, 0), (0, 2)])
def test_batch_equals_single_frames(pkg, gpu, split, mode):
    """sr_render_blocks_batch: B frames with different cameras (the flyby) in
    one launch, byte-identical to rendering each frame alone - a whole frame
    and block-cyclic shares, with and without split tiles, and in the
    half-width split mode with the noise mask."""
    import torch

    sc, abi = pkg.scenes, pkg.abi
    gpu.set_scene(sc.scene_default(textured=True))
    gpu.set_test_ray(abi.default_test_ray())
    if mode:
        params = abi.default_params(max_steps=1500, percent_black=0.6, raytrace_type=mode, curved_percentage=0.4)
    else:
        params = abi.default_params(max_steps=1500, percent_black=-1.0)
    W, H = 320, 184
    for B, (first, step) in ((5, (0, 1)), (3, (1, 4)), (16, (2, 8))):
        cams = [abi.camera_flyby((f + 0.5) / B, 30.0, 10.0) for f in range(B)]
        gpu.set_split(0)
        ref = []
        for c in cams:
            o, rows = gpu.render_blocks(c, params, W, H, 8, first, step)
            ref.append(o.cpu().numpy()[:rows])
        gpu.set_split(split, 4, 1)
        for _ in range(2):  # the second batch runs the learned order (and split tiles)
            out, rows = gpu.render_blocks_batch(cams, params, W, H, 8, first, step)
        torch.cuda.synchronize()
        gpu.set_split(0)
        got = out.cpu().numpy()
        assert len({r.tobytes() for r in ref}) == B  # every camera differs
        for f in range(B):
            assert np.array_equal(got[f, :rows], ref[f]), (B, first, step, f)


def test_block_list_rows_equal_full_frames(pkg, gpu):
    """sr_render_block_list: an explicit, unordered block list with -1 padding
    (dist.balanced_blocks' layout) renders, for B flyby frames in one launch,
    exactly the rows of each whole frame; padding rows stay untouched. Then
    the lists of every rank reassemble the frames (dist.assemble_lists)."""
    import torch

    sc, abi, D = pkg.scenes, pkg.abi, pkg.dist
    gpu.set_scene(sc.scene_default(textured=True))
    params = abi.default_params(max_steps=1500, percent_black=-1.0)
    W, H, B = 320, 180, 3
    cams = [abi.camera_flyby((f + 0.5) / B, 30.0, 10.0) for f in range(B)]
    full = [gpu.render(c, params, W, H).cpu().numpy() for c in cams]
    _, _, steps = gpu.render_debug(cams[0], params, W, H)
    torch.cuda.synchronize()
    blocks = [5, 0, 22, -1, 13, 7, -1]
    out = torch.full((B, len(blocks) * 8, W, 4), 77, dtype=torch.uint8, device="cuda")
    for _ in range(2):  # the second launch runs the learned order
        gpu.render_block_list(cams, params, W, H, 8, blocks, out=out)
    got = out.cpu().numpy()
    for f in range(B):
        for s, b in enumerate(blocks):
            rows = got[f, s * 8:(s + 1) * 8]
            n = 0 if b < 0 else min(8, H - b * 8)  # block 22 holds the frame's last 4 rows
            assert (rows[n:] == 77).all()
            if n:
                assert np.array_equal(rows[:n], full[f][b * 8:b * 8 + n]), (f, s, b)
    world = 3
    lists = D.balanced_blocks(D.wave_costs(steps, 8), world)
    tiles = np.stack([gpu.render_block_list(cams, params, W, H, 8, l).cpu().numpy() for l in lists])
    assert np.array_equal(D.assemble_lists(tiles, lists, H, 8), np.stack(full))


def test_wave_costs_map(pkg, gpu):
    """sr_wave_costs: per 8x8 wave, the longest ray's steps (the integrate
    kernel's count: at least render_debug's, which stops at the first hit the
    shade kernel finds opaque where the step loop logged it as possibly
    translucent and ran on) and the wave's budget events; deterministic, and the
    context's split setting is left as it was. dist.block_costs and
    balanced_blocks turn it into the ranks' lists."""
    import torch

    sc, abi, D = pkg.scenes, pkg.abi, pkg.dist
    gpu.set_scene(sc.scene_default(textured=True))
    params = abi.default_params(max_steps=2000, percent_black=-1.0)
    W, H = 328, 184  # partial wave columns at the right edge
    cam = abi.default_camera()
    gpu.set_split(16, 4, 1)
    a = gpu.wave_costs(cam, params, W, H).cpu().numpy()
    b = gpu.wave_costs(cam, params, W, H).cpu().numpy()
    assert np.array_equal(a, b)
    _, _, steps = gpu.render_debug(cam, params, W, H)
    torch.cuda.synchronize()
    s = steps.cpu().numpy()
    assert a.shape == ((H + 7) // 8, (W + 7) // 8, 2)
    pad = np.zeros((a.shape[0] * 8, a.shape[1] * 8), dtype=np.int64)
    pad[:H, :W] = s
    mx = pad.reshape(a.shape[0], 8, a.shape[1], 8).max(axis=(1, 3))
    assert (a[..., 0] >= mx).all() and (a[..., 0] == mx).mean() > 0.95
    assert (a[..., 1] >= 0).all() and a[..., 1].sum() > 0
    assert (a[..., 1][a[..., 0] == 0] == 0).all()
    costs = D.block_costs(a)
    assert costs.shape == (a.shape[0],) and (costs > 0).all()
    lists = D.balanced_blocks(costs, 4)
    assert sorted(x for l in lists for x in l if x >= 0) == list(range(a.shape[0]))
    # the split setting survives: a split render still equals the plain frame
    ref = gpu.render(cam, params, W, H).cpu().numpy()
    for _ in range(2):
        out = gpu.render(cam, params, W, H).cpu().numpy()
    assert np.array_equal(out, ref)
    gpu.set_split(0)


def test_rows_and_blocks_assemble_full_frame(pkg, gpu):
    import torch

    sc, abi = pkg.scenes, pkg.abi
    scene = sc.scene_default(textured=True)
    cam = abi.default_camera()
    params = abi.default_params(max_steps=500, percent_black=-1.0)
    gpu.set_scene(scene)
    W, H = 200, 113
    full = gpu.render(cam, params, W, H).cpu().numpy()
    part = gpu.render(cam, params, W, H, 37, 90).cpu().numpy()
    assert np.array_equal(part, full[37:90])
    for nranks in (2, 3, 8):
        frame = np.zeros_like(full)
        for rank in range(nranks):
            out, rows = gpu.render_blocks(cam, params, W, H, 8, rank, nranks)
            out = out.cpu().numpy()
            k = 0
            for b in range(rank, (H + 7) // 8, nranks):
                n = min(8, H - b * 8)
                frame[b * 8:b * 8 + n] = out[k:k + n]
                k += n
            assert k == rows
        torch.cuda.synchronize()
        assert np.array_equal(frame, full), nranks


def test_headline_frame_deterministic(pkg, gpu):
    """The metric's frame with the procedural golden textures: two launches
    byte-identical and the mean step count of SURVEY §8d (full-frame parity on
    the bench's own inputs is tests/test_gpu_frames.py)."""
    import torch

    sc, abi = pkg.scenes, pkg.abi
    gpu.set_scene(sc.scene_default(textured=True))
    gpu.set_test_ray(abi.default_test_ray())
    params = abi.default_params(max_steps=2000, percent_black=-1.0)
    _, b, s = gpu.render_debug(abi.default_camera(), params, 1920, 1080)
    b2 = gpu.render(abi.default_camera(), params, 1920, 1080)
    torch.cuda.synchronize()
    assert torch.equal(b, b2)
    # mean executed steps per pixel at N=2000 ~ 0.206 N
    assert 380 < float(s.float().mean()) < 440


@pytest.mark.parametrize("seed", range(8))
def test_random_scenes(pkg, gpu, oracle, oracle_tex, seed):
    """Stress scenes: 18-21 objects - more than the
    kernel's budget slots, so some are tested per chord - skewed frames
    (unbounded for culling), translucent and single-sided materials (logged
    hits, resumed rays), normal maps, planes in every other scene."""
    sc, abi = pkg.scenes, pkg.abi
    scene = sc.scene_random(seed, planes=seed % 2 == 0)
    cam = sc.random_camera(300 + seed)
    params = abi.default_params(max_steps=600, percent_black=-1.0)
    g = gpu_debug(gpu, scene, cam, params, 96, 54)
    o = oracle.render(scene, cam, params, 96, 54, oracle_tex)
    compare(g, o, f"random scene {seed}")


@pytest.mark.parametrize("seed", range(4))
def test_random_scenes_culling_exact(pkg, gpu, seed):
    """Culling, lazy chords and hit classification must not change a bit on
    the stress scenes either."""
    import torch

    sc, abi = pkg.scenes, pkg.abi
    gpu.set_scene(sc.scene_random(100 + seed, planes=seed % 2 == 1))
    gpu.set_test_ray(abi.default_test_ray())
    cam = sc.random_camera(400 + seed)
    params = abi.default_params(max_steps=1500, percent_black=-1.0)
    outs = []
    for cull in (True, False):
        gpu.set_culling(cull)
        f, b, s = gpu.render_debug(cam, params, 320, 180)
        torch.cuda.synchronize()
        outs.append((f.cpu().numpy().view(np.uint32), b.cpu().numpy(), s.cpu().numpy()))
    gpu.set_culling(True)
    for a, b in zip(outs[0], outs[1]):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("shear", [0.0, 0.3, -0.6])
@pytest.mark.parametrize("scale", [1.3, 0.7])
def test_skewed_frames_budgeted(pkg, gpu, oracle, oracle_tex, shear, scale):
    """Rectangles and boxes whose frames are not orthonormal (a column scaled,
    a shear between columns) are budgeted by the bounding sphere of their
    faces' parallelograms since round 6 (sr_api.cpp parallelogram_corners;
    they were tested on every chord and turned lazy chords off for the whole
    frame): the default scene with its rectangle and box so skewed, whole
    frames bit-exact against the oracle, and culling on vs off identical."""
    import torch

    sc, abi = pkg.scenes, pkg.abi
    scene = sc.scene_default(textured=True)
    A = np.eye(3)
    A[:, 0] *= scale
    A[:, 2] += shear * A[:, 1]
    cols = [float(np.float32(v)) for v in A.T.reshape(-1)]  # column-major axes
    for k in range(9):
        scene.rectangles[0].plane.transform.axes[k] = cols[k]
        scene.boxes[0].transform.axes[k] = cols[(k + 3) % 9]
    cam = sc.camera_look((0.0, 2.0, 15.0), (0.0, -2.0, -15.0), fov=70.0)
    params = abi.default_params(max_steps=1200, percent_black=-1.0)
    g = gpu_debug(gpu, scene, cam, params, 160, 90)
    o = oracle.render(scene, cam, params, 160, 90, oracle_tex)
    print(compare(g, o, f"skewed frames, scale {scale}, shear {shear}"))
    outs = []
    for cull in (True, False):
        gpu.set_culling(cull)
        f, b, st = gpu.render_debug(cam, params, 160, 90)
        torch.cuda.synchronize()
        outs.append((f.cpu().numpy().view(np.uint32), b.cpu().numpy(), st.cpu().numpy()))
    gpu.set_culling(True)
    for a, b_ in zip(outs[0], outs[1]):
        assert np.array_equal(a, b_)


def stacked_layers_scene(sc, abi, n_translucent=4, gap=0.5):
    """n_translucent translucent rectangles and an opaque one behind them,
    stacked across the default camera's view (z = 10, 10 - gap, ...): every
    ray logs four translucent hits (the hit log's capacity), stops as ST_MORE
    and is resumed by sr_resume_kernel a gap before the opaque layer."""
    import ctypes as C

    s = abi.Scene()
    abi.load().sr_scene_clear(C.byref(s))
    for m, col in ((0, (0.02, 0.04, 0.06, 0.3)), (1, (0.9, 0.2, 0.2, 1.0))):
        M = s.materials[m]
        for k in range(4):
            M.color[k] = col[k]
        M.ambient, M.diffuse, M.specular, M.shininess = 0.2, 0.8, 0.3, 16.0
        M.texture_index, M.normal_map_index, M.double_sided_normals = -1, -1, 1
    axes = sc._axes_from((0.0, 0.0, 1.0))  # normal +z, columns x and -y
    # three disks, then rectangles (three of each primitive at most)
    for k in range(n_translucent + 1):
        z = 10.0 - gap * k
        if k < 3:
            t, kind, idx = s.disks[k].plane.transform, abi.OBJECT_DISK, k
            pos = (0.0, 2.0, z)
            s.disks[k].radius = 12.0
        else:
            t, kind, idx = s.rectangles[k - 3].plane.transform, abi.OBJECT_RECTANGLE, k - 3
            pos = (-8.0, 10.0, z)  # a corner: x in [-8, 8], y in [-6, 10]
            s.rectangles[k - 3].width = s.rectangles[k - 3].height = 16.0
        for i in range(3):
            t.pos[i] = pos[i]
        for i in range(9):
            t.axes[i] = axes[i]
        o = s.objects[k]
        o.type, o.index, o.material_index = kind, idx, int(k == n_translucent)
    s.num_objects = n_translucent + 1
    s.num_lights = 1
    L = s.lights[0]
    for i in range(3):
        L.transform.pos[i] = (0.0, 5.0, 14.0)[i]
        L.color[i] = 1.0
    L.intensity, L.attenuation_constant, L.attenuation_linear, L.attenuation_quadratic = 5.0, 1.0, 0.09, 0.032
    return s


def test_resumed_rays_start_without_a_window(pkg, gpu, oracle, oracle_tex):
    """Rays resumed after a full hit log (sr_resume_kernel) start from a chord
    end, not from the orbit's tangent, so they get no directional start
    window (budget_init<false>). Round 6: the resume passed a NaN direction
    meant to disable the window, but fminf dropped the NaN and the planar
    slots got the window's caps: the layer right behind the fourth one was
    skipped unless a wave-mate's event re-anchored it first (three pixels of
    a four-frame stress batch, varying with the worklist's order). Here every
    ray resumes 0.5 before an opaque layer: whole frames bit-exact against
    the oracle, culling on and off identical, at two step counts."""
    import torch

    sc, abi = pkg.scenes, pkg.abi
    scene = stacked_layers_scene(sc, abi)
    cam = abi.default_camera()
    for N in (1000, 2000):
        params = abi.default_params(max_steps=N, percent_black=-1.0)
        g = gpu_debug(gpu, scene, cam, params, 160, 90)
        o = oracle.render(scene, cam, params, 160, 90, oracle_tex)
        # the case is the one described: most rays end on the opaque layer
        assert (o[0][..., 0] > o[0][..., 2]).mean() > 0.5
        print(compare(g, o, f"stacked layers, {N} steps"))
        gpu.set_culling(False)
        f, b, st = gpu.render_debug(cam, params, 160, 90)
        torch.cuda.synchronize()
        gpu.set_culling(True)
        assert np.array_equal(b.cpu().numpy(), g[0]) and np.array_equal(st.cpu().numpy(), g[2])


def test_ray_through_singularity(pkg, gpu, oracle, oracle_tex):
    """A ray that passes the r = 1 shell behind an alpha-0 texel (the chord's
    closest hit is the object, so the hole is not hit) falls on to the
    singularity: u passes 1e30, then +inf, where RK4 keeps u = u' = +inf, and
    the reference's next chord (zero length, NaN direction) ends the ray with
    a NaN colour at step 285. The fast loop must leave for that degenerate
    chord although the lane's ball holds the origin (geodesic.hip SR_U_NOWIN;
    round 6: the stress scene's pixel (322, 154) at 640x360 ran to max_steps
    once that scene's chords were lazy)."""
    sc, abi = pkg.scenes, pkg.abi
    params = abi.default_params(max_steps=1000, percent_black=-1.0)
    cam = abi.default_camera()
    g = gpu_debug(gpu, sc.scene_stress(), cam, params, 640, 360, row_begin=152, row_end=157)
    o = oracle.render(sc.scene_stress(), cam, params, 640, 360, oracle_tex, row_begin=152, row_end=157)
    assert o[2][154 - 152, 322] == 285  # the case is the one described
    assert np.isnan(o[1][154 - 152, 322]).any()
    print(compare(g, o, "ray through the singularity"))


def test_test_ray_far_view(pkg, gpu, oracle, oracle_tex):
    """A visible press-R polyline seen from far away: every chord must be
    tested against the test-ray cylinders even where no budget is spent."""
    sc, abi = pkg.scenes, pkg.abi
    cam0 = sc.camera_look((4.0, 1.0, 12.0), (-0.3, -0.05, -1.0))
    fwd = list(cam0.transform.axes[6:9])
    pts = abi.test_ray_points(list(cam0.transform.pos), fwd, 300, 2)
    tr = abi.default_test_ray()
    tr.visible = 1
    tr.num_curved_points = len(pts)
    for i, p in enumerate(pts):
        tr.curved_points[i][0], tr.curved_points[i][1], tr.curved_points[i][2] = p
    for k in range(3):
        tr.flat_origin[k] = cam0.transform.pos[k] + fwd[k]
        tr.flat_dir[k] = fwd[k]
    view = sc.camera_look((0.0, 25.0, 45.0), (0.0, -25.0, -45.0), fov=60.0)
    scene = sc.scene_black_hole_only()
    params = abi.default_params(max_steps=800, percent_black=-1.0)
    g = gpu_debug(gpu, scene, view, params, 96, 54, tr)
    o = oracle.render(scene, view, params, 96, 54, oracle_tex, tr)
    compare(g, o, "test ray far view")
    assert (g[0][..., :3] != o[0][..., :3]).sum() == 0
    gpu.set_test_ray(abi.default_test_ray())


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_test_ray_budget_random(pkg, gpu, oracle, oracle_tex, seed):
    """The test ray's budget (round 6, clearance_tr and the group mask) against
    the oracle's exhaustive loop: random press-R polylines seen from their own
    camera (every ray starts beside the polyline and the flat cylinder, and
    the pixels near the polyline's image travel along it) and from another
    random camera. Random directions give some segments the reference's
    ill-conditioned gram_schmidt frames (frame_norms' skewed bounds)."""
    sc, abi = pkg.scenes, pkg.abi
    cam0 = sc.random_camera(900 + seed)
    fwd = list(cam0.transform.axes[6:9])
    pts = abi.test_ray_points(list(cam0.transform.pos), fwd, 300 + 100 * seed, 2)[:abi.MAX_POINTS]
    tr = abi.default_test_ray()
    tr.visible = 1
    tr.num_curved_points = len(pts)
    for i, p in enumerate(pts):
        tr.curved_points[i][0], tr.curved_points[i][1], tr.curved_points[i][2] = p
    for k in range(3):
        tr.flat_origin[k] = cam0.transform.pos[k] + fwd[k]
        tr.flat_dir[k] = fwd[k]
    view = cam0 if seed % 2 == 0 else sc.random_camera(950 + seed)
    scene = sc.scene_default(textured=False)
    params = abi.default_params(max_steps=500, percent_black=-1.0)
    g = gpu_debug(gpu, scene, view, params, 96, 54, tr)
    o = oracle.render(scene, view, params, 96, 54, oracle_tex, tr)
    compare(g, o, f"test-ray budget, seed {seed}")
    # the overlay is on screen (flat: green, curved: red; frag:191-192)
    b = o[0][..., :3]
    assert (((b == (255, 0, 0)).all(-1)) | ((b == (0, 255, 0)).all(-1))).sum() > 0
    gpu.set_test_ray(abi.default_test_ray())


@pytest.mark.parametrize("kind", ["general", "large", "large_translucent"])
def test_test_ray_budget_instantiations(pkg, gpu, oracle, oracle_tex, kind):
    """The test-ray instantiations beyond the small one: an 8-object scene
    (the general 8-slot kernel with the test ray's row) and 21-object scenes
    (the large kernel), one with translucent materials so that rays stop with
    their hit log full and the test-ray resume kernel continues them."""
    sc, abi = pkg.scenes, pkg.abi
    if kind == "general":
        scene = sc.scene_random(7, n_objects=8, translucent=False, planes=False)
    elif kind == "large":
        scene = sc.scene_stress()
    else:
        scene = sc.scene_random(11, n_objects=21, translucent=True, planes=True)
    cam0 = sc.camera_look((1.0, 3.0, 16.0), (0.18, -0.1, -1.0))
    fwd = list(cam0.transform.axes[6:9])
    pts = abi.test_ray_points(list(cam0.transform.pos), fwd, 600, 2)[:abi.MAX_POINTS]
    tr = abi.default_test_ray()
    tr.visible = 1
    tr.num_curved_points = len(pts)
    for i, p in enumerate(pts):
        tr.curved_points[i][0], tr.curved_points[i][1], tr.curved_points[i][2] = p
    for k in range(3):
        tr.flat_origin[k] = cam0.transform.pos[k] + fwd[k]
        tr.flat_dir[k] = fwd[k]
    view = sc.camera_look((0.0, 2.0, 15.0), (0.0, -2.0, -15.0))
    params = abi.default_params(max_steps=400, percent_black=-1.0)
    g = gpu_debug(gpu, scene, view, params, 64, 36, tr)
    o = oracle.render(scene, view, params, 64, 36, oracle_tex, tr)
    compare(g, o, f"test-ray budget, {kind} instantiation")
    gpu.set_test_ray(abi.default_test_ray())


@pytest.mark.parametrize("name,pos,fwd,fov,textured", [
    ("close to the hole", (0.0, 0.4, 4.0), (0.0, -0.1, -1.0), 90.0, True),
    ("edge-on accretion disk", (9.0, 0.05, 0.0), (-1.0, 0.0, 0.0), 40.0, True),
    ("photon ring, untextured", (0.0, 3.0, 14.0), (0.0, -3.0, -14.0), 25.0, False),
])
def test_near_horizon_views(pkg, gpu, oracle, oracle_tex, name, pos, fwd, fov, textured):
    """Rays skimming the r = 1 shell and orbiting the photon sphere for up to
    2000 steps: the black hole's shell clearance, the budget look-ahead and
    the re-anchor shortcuts where budget events are densest."""
    sc, abi = pkg.scenes, pkg.abi
    scene = sc.scene_default(textured=textured)
    cam = sc.camera_look(pos, fwd, fov=fov)
    params = abi.default_params(max_steps=2000, percent_black=-1.0)
    g = gpu_debug(gpu, scene, cam, params, 96, 54)
    o = oracle.render(scene, cam, params, 96, 54, oracle_tex)
    compare(g, o, name)
    assert (g[2] != o[2]).sum() == 0, f"{name}: step counts differ"


def test_config2_full_frame(pkg, gpu, oracle, oracle_tex):
    """BASELINE config 2 (640x360, 1000 steps, default textured scene), the
    whole frame: RGBA8, float FragColor and step counts, GPU == oracle."""
    sc, abi = pkg.scenes, pkg.abi
    scene = sc.scene_default(textured=True)
    cam = abi.default_camera()
    params = abi.default_params(max_steps=1000, percent_black=-1.0)
    g = gpu_debug(gpu, scene, cam, params, 640, 360)
    o = oracle.render(scene, cam, params, 640, 360, oracle_tex)
    print(compare(g, o, "config 2"))
    assert (g[2] != o[2]).sum() == 0, "config 2: step counts differ"
    assert 180 < g[2].mean() < 230, g[2].mean()  # 206.5 mean steps per pixel


@pytest.mark.parametrize("name,pos,fov,u_f", [
    ("r = 120, headline size", (0.0, 12.0, 119.4), 12.0, 0.01),
    ("r = 300, headline size", (60.0, 40.0, 291.2), 5.0, 0.01),
    ("default camera, u_f = 0.1", None, 90.0, 0.1),
])
def test_reseed_headline_rows(pkg, gpu, oracle, oracle_tex, name, pos, fov, u_f):
    """The u < u_f reseed branch (frag:891-912: intersect the r = 1/u_f sphere,
    rebuild the orbital frame, phi not reset) at 1920x1080 / 2000 steps: the
    whole frame on the GPU, 12 rows through it bit-compared with the oracle,
    step counts included."""
    import torch

    sc, abi = pkg.scenes, pkg.abi
    scene = sc.scene_default(textured=True)
    cam = abi.default_camera() if pos is None else sc.camera_look(pos, tuple(-v for v in pos), fov=fov)
    params = abi.default_params(max_steps=2000, percent_black=-1.0, u_f=u_f)
    W, H = 1920, 1080
    gpu.set_scene(scene)
    gpu.set_test_ray(abi.default_test_ray())
    _, b, s = gpu.render_debug(cam, params, W, H)
    torch.cuda.synchronize()
    b, s = b.cpu().numpy(), s.cpu().numpy()
    rows = np.linspace(0, H - 1, 12).astype(int)
    # the rows through the black hole (its longest rays) too
    rows = sorted(set(rows.tolist()) | set(int(v) for v in np.argsort(s.max(axis=1))[-4:]))
    for y in rows:
        rb, _, rs = oracle.render(scene, cam, params, W, H, oracle_tex, None, int(y), int(y) + 1)
        assert not (rb[0] != b[y]).any(), f"{name}: row {y}"
        assert (rs[0] != s[y]).sum() == 0, f"{name}: row {y} step counts"


@pytest.mark.parametrize("max_steps,revs", [(2000, 2), (600, 1)])
def test_negative_u_exits(pkg, gpu, oracle, oracle_tex, max_steps, revs):
    """Rays that leave by u < 0 (frag:921-922: get_bg with the previous
    chord) rather than by the u_f reseed: with u_f = 1e-4 an escaping ray's u
    steps from above 1e-4 straight below 0, so every escaping lane takes the
    exit whose previous chord needs u after step i - 2, which the fast loop
    does not carry (integrate's recover_up replays the RK4 steps). With one
    revolution of the step schedule (frag:20) over 600 steps, rays near the
    photon ring also reach the end of the loop (the other replay). Whole
    320x180 frames, bit-exact with step counts."""
    sc, abi = pkg.scenes, pkg.abi
    scene = sc.scene_default(textured=True)
    cam = abi.default_camera()
    params = abi.default_params(max_steps=max_steps, percent_black=-1.0, u_f=1.0e-4, max_revolutions=revs)
    g = gpu_debug(gpu, scene, cam, params, 320, 180)
    o = oracle.render(scene, cam, params, 320, 180, oracle_tex)
    print(compare(g, o, f"u_f 1e-4, {max_steps} steps, {revs} revolutions"))  # pixels, float bits, steps
    if revs == 1:
        assert (o[2] == max_steps).sum() > 50  # rays that ran to the end of the loop


@pytest.mark.parametrize("max_steps,revs,closest", [(2000, 2, 10.0), (1000, 2, 4.0), (600, 2, 4.0), (300, 1, 6.0)])
def test_black_hole_crossings(pkg, gpu, oracle, oracle_tex, max_steps, revs, closest):
    """Rays falling into the hole (geodesic.hip SR_BH_WINDOW2 / SR_BH_CROSS):
    the inner window down to the frame's bound and crossings that end as
    ST_BH without an event. Step angles on both sides of SR_BH_S_DPHI (the
    steep lanes' 6e-5 bound at 2000 and 1000 steps over two revolutions, the
    1.5e-3 one at 600 and 300), flyby cameras 4-10 units from the hole so
    that much of the frame falls in. Whole 320x180 frames, bit-exact with
    step counts."""
    sc, abi = pkg.scenes, pkg.abi
    scene = sc.scene_default(textured=True)
    cam = abi.camera_flyby(0.5, 30.0, closest)
    params = abi.default_params(max_steps=max_steps, percent_black=-1.0, max_revolutions=revs)
    g = gpu_debug(gpu, scene, cam, params, 320, 180)
    o = oracle.render(scene, cam, params, 320, 180, oracle_tex)
    print(compare(g, o, f"{max_steps} steps, {revs} revolutions, closest {closest}"))
    assert (o[2] < max_steps).sum() > 0


def test_reference_assets_frame(pkg, oracle):
    """The reference's own textures through the ingest path (assets/textures:
    2k.jpg skybox, uv_checker.jpg + cubemap.png array, image_utils.cpp:7-117)
    into sr_set_background / sr_set_texture_array: a 480x270 / 1000-step
    frame and a flyby view, GPU == oracle on the same decoded texels."""
    import torch

    A, sc, abi = pkg.assets, pkg.scenes, pkg.abi
    if not A.available():
        pytest.skip("assets/textures missing")
    bg = A.skybox("2k")
    arr, sizes, mx = A.texture_array()
    scene = sc.scene_default(textured=True)
    assert [tuple(scene.texture_sizes[i]) for i in range(2)] == [tuple(float(v) for v in s) for s in sizes]
    r = pkg.Renderer(0)
    r.set_background(bg)
    r.set_texture_array(arr)
    r.set_scene(scene)
    tex = oracle.TextureSet(bg, arr)
    for label, cam in (("default camera", abi.default_camera()), ("flyby t = 0.4", abi.camera_flyby(0.4))):
        params = abi.default_params(max_steps=1000, percent_black=-1.0)
        f, b, s = r.render_debug(cam, params, 480, 270)
        torch.cuda.synchronize()
        o = oracle.render(scene, cam, params, 480, 270, tex)
        print(compare((b.cpu().numpy(), f.cpu().numpy(), s.cpu().numpy()), o, label))
    r.close()


def test_presentation_png_of_a_gpu_frame(pkg, gpu, tmp_path):
    """Presentation: a frame rendered on the GPU, copied to
    the host and written by sr_write_png decodes (PIL) to the same pixels,
    top row first (sr_render's rows are bottom-up, as GL leaves them)."""
    import torch

    PIL = pytest.importorskip("PIL.Image")
    sc, abi = pkg.scenes, pkg.abi
    gpu.set_scene(sc.scene_default(textured=True))
    gpu.set_test_ray(abi.default_test_ray())
    params = abi.default_params(max_steps=800, percent_black=-1.0)
    frame = gpu.render(abi.default_camera(), params, 200, 113)
    torch.cuda.synchronize()
    frame = frame.cpu().numpy()
    path = tmp_path / "frame.png"
    abi.write_png(path, frame)
    got = np.asarray(PIL.open(path).convert("RGBA"))
    assert got.shape == (113, 200, 4)
    assert np.array_equal(got, frame[::-1])


def test_two_contexts_alternating_shapes_in_flight(pkg, textures):
    """Render paths allocate in stream order (no device-wide synchronisation):
    two contexts on two streams with frames in flight, cycling through more
    frame shapes, step counts and block lists than a context's caches hold
    (LRU eviction, stream-ordered frees after the in-flight frames). Every
    frame equals, byte for byte, a fresh context's render of it."""
    import torch

    sc, abi = pkg.scenes, pkg.abi
    bg, arr = textures
    scene = sc.scene_default(textured=True)
    cam = abi.default_camera()

    def make():
        r = pkg.Renderer(0)
        r.set_scene(scene)
        r.set_background(bg)
        r.set_texture_array(arr)
        return r

    shapes = [(160, 90, 300), (200, 113, 500), (96, 54, 800), (320, 180, 400), (128, 72, 300), (64, 36, 200),
              (256, 144, 350), (144, 81, 450), (176, 99, 250), (112, 63, 600), (208, 117, 320)]
    lists = [[5, 0, 2, -1], [1, 3], [4, -1, 0], [2], [0, 1, 2, 3, 4], [3, -1], [4, 2], [1], [0, 4], [2, 3, 1],
             [5, 4, 3]]
    lw, lh, ln = 160, 48, 400
    ref = {}
    r0 = make()
    for W, H, N in shapes:
        ref[(W, H, N)] = r0.render(cam, abi.default_params(max_steps=N, percent_black=-1.0), W, H).cpu().numpy()
    full = r0.render(cam, abi.default_params(max_steps=ln, percent_black=-1.0), lw, lh).cpu().numpy()
    r0.close()
    ctxs, streams = [make(), make()], [torch.cuda.Stream(), torch.cuda.Stream()]
    got = []
    for rep in range(3):
        for i, (W, H, N) in enumerate(shapes):
            k = (i + rep) % 2
            with torch.cuda.stream(streams[k]):
                out = ctxs[k].render(cam, abi.default_params(max_steps=N, percent_black=-1.0), W, H, stream=streams[k])
            got.append(((W, H, N), out, streams[k]))
        for i, blocks in enumerate(lists):
            k = i % 2
            with torch.cuda.stream(streams[k]):
                out = ctxs[k].render_block_list([cam], abi.default_params(max_steps=ln, percent_black=-1.0), lw, lh,
                                                8, blocks, stream=streams[k])
            got.append((tuple(blocks), out, streams[k]))
    torch.cuda.synchronize()
    for key, out, _ in got:
        o = out.cpu().numpy()
        if key in ref:
            assert np.array_equal(o, ref[key]), key
        else:
            for s_, b in enumerate(key):
                if b >= 0:
                    n = min(8, lh - b * 8)
                    assert np.array_equal(o[0, s_ * 8:s_ * 8 + n], full[b * 8:b * 8 + n]), (key, b)
    for c in ctxs:
        c.close()


def test_one_context_alternating_streams(pkg, textures):
    """A context's launches on another stream than its last one wait for that
    stream first (sr_api.cpp launch: an event on the old stream): one context
    alternating two streams with no host synchronisation renders every frame
    equal to a fresh render of it, though the frames share its pixel state."""
    import torch

    sc, abi = pkg.scenes, pkg.abi
    bg, arr = textures
    scene = sc.scene_default(textured=True)
    cams = [sc.random_camera(700 + i) for i in range(6)]
    params = abi.default_params(max_steps=500, percent_black=-1.0)
    W, H = 160, 90
    r = pkg.Renderer(0)
    r.set_scene(scene)
    r.set_background(bg)
    r.set_texture_array(arr)
    ref = [r.render(c, params, W, H).cpu().numpy() for c in cams]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    got = []
    for rep in range(2):
        for i, c in enumerate(cams):
            s = streams[(i + rep) % 2]
            with torch.cuda.stream(s):
                got.append((i, r.render(c, params, W, H, stream=s)))
    torch.cuda.synchronize()
    for i, out in got:
        assert np.array_equal(out.cpu().numpy(), ref[i]), i
    assert r.diag_counters() == {"hit_not_opaque": 0, "free_errors": 0}
    r.close()


def test_zz_diag_counters_zero(gpu):
    """After every render of this module on the shared context (translucent,
    single-sided and textured materials, stress scenes, resumed rays): no
    pixel stopped at an opaque-classified hit whose shaded alpha was not 1
    (the step loop's classification is exact where it claims), and no
    stream-ordered free failed."""
    assert gpu.diag_counters() == {"hit_not_opaque": 0, "free_errors": 0}


@pytest.mark.parametrize("u_f", [1.0e-4, 0.01, 0.05])
def test_objects_near_orbital_planes(pkg, gpu, oracle, oracle_tex, u_f):
    """The orbital-plane exclusion (geodesic.hip budget_frame) with its
    bound S_max = (sqrt 3 + 3) / u_f + 1 (sr_dev_frame.xplane_s): a sphere and
    a box on the line through the camera and the hole lie near the pencil of
    orbital planes through that line, at the exclusion's margin, for small and
    large u_f (chords up to r = 2e4 with u_f = 1e-4, where the bound is
    effectively off; the near-radial escapes to u < u_f / 2 force the
    excluded slots). Whole 160x90 frames, bit-exact with step counts."""
    sc, abi = pkg.scenes, pkg.abi
    scene = sc.scene_default(textured=True)
    for k, v in enumerate((0.05, 1.02, 7.3)):
        scene.spheres[0].transform.pos[k] = v
    for k, v in enumerate((-0.4, -1.1, -8.2)):
        scene.boxes[0].transform.pos[k] = v
    cam = sc.camera_look((0.0, 2.0, 15.0), (0.0, -2.0, -15.0), fov=70.0)
    params = abi.default_params(max_steps=1200, percent_black=-1.0, u_f=u_f)
    g = gpu_debug(gpu, scene, cam, params, 160, 90)
    o = oracle.render(scene, cam, params, 160, 90, oracle_tex)
    print(compare(g, o, f"objects near orbital planes, u_f {u_f}"))


@pytest.mark.parametrize("u_f,max_steps,t,d,revs", [
    (0.01, 1200, 7.0, 2.9, 2), (0.01, 600, 7.0, 4.0, 2), (0.01, 1200, 4.0, 2.7, 2),
    (0.05, 1200, -8.0, 3.2, 2), (1.0e-4, 1200, 7.0, 3.0, 2),
    (0.01, 100, 7.0, 2.9, 2), (0.01, 100, 7.0, 3.4, 3), (0.01, 8000, 7.0, 2.9, 2), (0.01, 300, 4.0, 2.7, 1)])
def test_cylinder_near_orbital_planes(pkg, gpu, oracle, oracle_tex, u_f, max_steps, t, d, revs):
    """The cylinder's orbital-plane exclusion for low-energy orbits
    (geodesic.hip SR_XCYL, sr_api.cpp xcyl_need: about br + 0.3 at the
    default step angle and u_f = 0.01, +inf at u_f = 1e-4). Every orbital
    plane holds the line through the camera and the hole; the cylinder's
    base sits at t along it and d off it, so its bounding centre is at 0 ..
    d + 2 from the planes of the frame's rays, across the exclusion's
    threshold. Step angles over the range the exclusions are enabled for
    (sr_api.cpp clear_radius, SR_XLOW_DPHI_MAX; tests/test_low_energy_bounds.py
    proves the premises there): the app's MAX_STEPS 100 (src/main.cpp:68) at
    two and three revolutions (0.126, 0.188 rad), 300 steps at one, 600 and
    1200 at two, and config 5's 8000; whole 160x90 frames, bit-exact with
    step counts."""
    sc, abi = pkg.scenes, pkg.abi
    scene = sc.scene_default(textured=True)
    line = np.array([0.0, 2.0, 15.0]) / np.linalg.norm([0.0, 2.0, 15.0])
    pos = line * t + np.array([d, 0.0, 0.0])
    for k in range(3):
        scene.cylinders[0].transform.pos[k] = float(np.float32(pos[k]))
    cam = sc.camera_look((0.0, 2.0, 15.0), (0.0, -2.0, -15.0), fov=70.0)
    params = abi.default_params(max_steps=max_steps, percent_black=-1.0, u_f=u_f, max_revolutions=revs)
    g = gpu_debug(gpu, scene, cam, params, 160, 90)
    o = oracle.render(scene, cam, params, 160, 90, oracle_tex)
    print(compare(g, o, f"cylinder near orbital planes, u_f {u_f}, {max_steps} steps x {revs} revs, t {t}, d {d}"))


@pytest.mark.parametrize("u_f,max_steps,rs,rb,revs", [
    (0.01, 1200, 3.2, 4.0, 2), (0.01, 600, 4.5, 5.5, 2), (0.05, 1200, 2.6, 6.5, 2), (1.0e-4, 1200, 3.2, 4.0, 2),
    (0.01, 100, 3.2, 4.0, 2), (0.01, 100, 4.5, 5.5, 3), (0.01, 8000, 3.2, 4.0, 2), (0.01, 300, 2.6, 6.5, 1)])
def test_objects_near_periapsis(pkg, gpu, oracle, oracle_tex, u_f, max_steps, rs, rb, revs):
    """The periapsis exclusion (geodesic.hip SR_XPERI, sr_api.cpp xperi_e): a
    low-energy orbit never comes closer to the hole than its periapsis, so
    objects whose reachable chords all lie inside that sphere are excluded
    for it. A sphere and a box moved close to the hole (centres at rs and rb
    from it, beside the accretion disk within r = 5) put the exclusion's
    threshold energy inside the frame's spread of impact parameters. Step
    angles over the range the exclusion is enabled for (100 steps at two and
    three revolutions, 300 at one, 600 / 1200 at two, 8000; see
    test_cylinder_near_orbital_planes) and three u_f (1e-4: chords out to r =
    2e4, the bound's large-r clearing fails and nothing is excluded), whole
    160x90 frames, bit-exact with step counts."""
    sc, abi = pkg.scenes, pkg.abi
    scene = sc.scene_default(textured=True)
    for k, v in enumerate((rs * 0.8, 0.0, rs * 0.6)):
        scene.spheres[0].transform.pos[k] = v
    for k, v in enumerate((-rb * 0.6, 0.5, -rb * 0.8)):
        scene.boxes[0].transform.pos[k] = v
    cam = sc.camera_look((0.0, 2.0, 15.0), (0.0, -2.0, -15.0), fov=70.0)
    params = abi.default_params(max_steps=max_steps, percent_black=-1.0, u_f=u_f, max_revolutions=revs)
    g = gpu_debug(gpu, scene, cam, params, 160, 90)
    o = oracle.render(scene, cam, params, 160, 90, oracle_tex)
    print(compare(g, o, f"objects near periapsis, u_f {u_f}, {max_steps} steps x {revs} revs, sphere at {rs}, box at {rb}"))
