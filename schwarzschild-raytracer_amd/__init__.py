"""schwarzschild-raytracer_amd — MI355X-native drop-in for the reference's
per-pixel geodesic shader (Yachim/schwarzschild-raytracer,
assets/shaders/black_hole.frag).

Layout:
  csrc/kernels/geodesic.hip  the gfx950 kernel (one wave64 lane per ray)
  csrc/sr_api.cpp            the C-ABI of include/sr/sr.h
  csrc/host/scene.cpp        the reference-shaped C++ scene model (include/sr/scene.hpp)
  abi.py                     ctypes mirror of sr.h
  renderer.py                Renderer: device handle (torch for memory/streams)
  scenes.py                  scenes, cameras, stand-in textures
  assets.py                  the reference's own textures (assets/textures) decoded as stb_image does
  dist.py                    row-band tiling over ranks + RCCL gather

Import as a package via `load_package()` in bench.py / tests (the directory
name is not a Python identifier).
"""
from . import abi, assets, dist, scenes  # noqa: F401

__all__ = ["abi", "assets", "dist", "scenes", "Renderer"]


def __getattr__(name):
    if name == "Renderer":
        from .renderer import Renderer

        return Renderer
    raise AttributeError(name)
