"""Builds tests/cpp/test_scene.cpp against include/sr/scene.hpp + libsr.so
with the host C++ compiler and runs it (host code only, no GPU)."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def test_cpp_scene_model(pkg, tmp_path):
    lib = pkg.abi.LIB_PATH
    assert lib.exists()
    cxx = shutil.which("g++") or shutil.which("c++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = tmp_path / "test_scene"
    cmd = [cxx, "-std=c++17", "-O1", "-ffp-contract=off", f"-I{ROOT / 'include'}", str(ROOT / "tests/cpp/test_scene.cpp"),
           str(lib), f"-Wl,-rpath,{lib.parent}", "-L/opt/rocm/lib", "-Wl,-rpath,/opt/rocm/lib", "-lamdhip64",
           "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    res = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert res.returncode == 0, res.stdout + res.stderr
    assert "ALL OK" in res.stdout
