#!/usr/bin/env python3
"""Parity of one libsr variant against the CPU oracle on the stress scenes
(tests/test_gpu_parity.py::test_random_scenes), printing every differing
pixel: python tools/variant_parity.py LIB [--seeds 0 1 2 3] [--no-cull]"""
import argparse
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--seeds", type=int, nargs="+", default=[0, 1, 2, 3, 4, 5, 6, 7])
    ap.add_argument("--no-cull", action="store_true")
    args = ap.parse_args()
    os.environ["SR_LIB"] = str(Path(args.lib).resolve())
    import torch

    import srpkg

    pkg = srpkg.load_package()
    oracle = srpkg.load_oracle()
    sc, abi = pkg.scenes, pkg.abi
    bg = sc.skybox(512, 256)  # tests/conftest.py textures (golden meta_skybox_shape)
    arr, _, _ = sc.default_texture_array()
    tex = oracle.TextureSet(bg, arr)
    r = pkg.Renderer(0)
    r.set_background(bg)
    r.set_texture_array(arr)
    r.set_culling(not args.no_cull)
    for seed in args.seeds:
        scene = sc.scene_random(seed, planes=seed % 2 == 0)
        cam = sc.random_camera(300 + seed)
        params = abi.default_params(max_steps=600, percent_black=-1.0)
        r.set_scene(scene)
        r.set_test_ray(abi.default_test_ray())
        f, b, s = r.render_debug(cam, params, 96, 54)
        torch.cuda.synchronize()
        b, s = b.cpu().numpy(), s.cpu().numpy()
        rb, _, rs = oracle.render(scene, cam, params, 96, 54, tex)
        bad = np.argwhere((b != rb).any(-1) | (s != rs))
        print(f"seed {seed}: {len(bad)} differing pixels")
        for y, x in bad[:10]:
            print(f"   ({x},{y}) gpu steps {s[y, x]} rgba {b[y, x]}  oracle steps {rs[y, x]} rgba {rb[y, x]}")
    # rays skimming the horizon and orbiting the photon sphere (2000 steps)
    for name, cam, w, h in [("headline camera", abi.default_camera(), 192, 108),
                            ("close to the hole", sc.camera_look((0.0, 0.4, 4.0), (0.0, -0.1, -1.0), fov=90.0), 96, 54),
                            ("edge-on disk", sc.camera_look((9.0, 0.05, 0.0), (-1.0, 0.0, 0.0), fov=40.0), 96, 54)]:
        scene = sc.scene_default(textured=True)
        params = abi.default_params(max_steps=2000, percent_black=-1.0)
        r.set_scene(scene)
        r.set_test_ray(abi.default_test_ray())
        f, b, s = r.render_debug(cam, params, w, h)
        torch.cuda.synchronize()
        b, s = b.cpu().numpy(), s.cpu().numpy()
        rb, _, rs = oracle.render(scene, cam, params, w, h, tex)
        bad = np.argwhere((b != rb).any(-1) | (s != rs))
        print(f"{name}: {len(bad)} differing pixels")
        for y, x in bad[:10]:
            print(f"   ({x},{y}) gpu steps {s[y, x]} rgba {b[y, x]}  oracle steps {rs[y, x]} rgba {rb[y, x]}")
    r.close()


if __name__ == "__main__":
    main()
