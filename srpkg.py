"""Import helper: the package directory `schwarzschild-raytracer_amd/` is not a
Python identifier, so it is loaded under the module name
`schwarzschild_raytracer_amd`."""
from __future__ import annotations

import importlib.util
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent
PKG_DIR = ROOT / "schwarzschild-raytracer_amd"
NAME = "schwarzschild_raytracer_amd"


def load_package():
    if NAME in sys.modules:
        return sys.modules[NAME]
    spec = importlib.util.spec_from_file_location(NAME, PKG_DIR / "__init__.py", submodule_search_locations=[str(PKG_DIR)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    spec.loader.exec_module(mod)
    return mod


def load_oracle():
    """The CPU oracle binding (test infrastructure: tests/, smoke(), bench cpu_baseline)."""
    if str(ROOT) not in sys.path:
        sys.path.insert(0, str(ROOT))
    load_package()
    from oracle import oracle as o

    return o
