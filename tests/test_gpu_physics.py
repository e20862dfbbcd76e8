"""The capture threshold b_crit = 3*sqrt(3)/2 on the gfx950 kernel (1x1
frames through the C-ABI), mirroring tests/test_physics.py's oracle check."""
import numpy as np
import pytest

from test_physics import one_pixel

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("b,captured", [(2.0, True), (2.45, True), (2.55, True), (2.65, False), (3.0, False),
                                        (6.0, False)])
def test_capture_threshold_kernel(pkg, b, captured):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    sc, abi = pkg.scenes, pkg.abi
    with pkg.Renderer(0) as r:
        r.set_scene(sc.scene_black_hole_only())
        r.set_background(np.full((8, 16, 3), 200, dtype=np.uint8))
        cam = one_pixel(pkg, b)
        out = r.render(cam, abi.default_params(max_steps=4000, percent_black=-1.0), 1, 1)
        px = out.cpu().numpy()[0, 0].tolist()
    assert px == ([0, 0, 0, 255] if captured else [200, 200, 200, 255]), (b, px)
