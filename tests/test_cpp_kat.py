"""The C++ host mirror (include/sidecar/catalog.hpp) and its reference KATs
(tests/cpp/test_catalog_kat.cpp), linked against the CPU oracle (CPU suite) or the HIP engine."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "test_catalog_kat.cpp")
OUT = os.path.join(ROOT, "tests", "cpp", "build")


def build_and_run(libdir, libname, tag):
    os.makedirs(OUT, exist_ok=True)
    exe = os.path.join(OUT, f"test_catalog_kat_{tag}")
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-I", os.path.join(ROOT, "include"), SRC, "-o", exe,
                    f"-L{libdir}", f"-l{libname}", f"-Wl,-rpath,{libdir}"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_cpp_mirror_kats_oracle(oracle_lib):
    out = build_and_run(os.path.join(ROOT, "oracle"), "oracle_gx", "oracle")
    assert "backend=oracle-cpu" in out and "failures=0" in out


@pytest.mark.gpu
def test_cpp_mirror_kats_gpu(gx_lib):
    out = build_and_run(os.path.join(ROOT, "sidecar_amd"), "gx", "gpu")
    assert "backend=hip-gfx950" in out and "failures=0" in out
