"""Builds the HIP engine in-tree: sidecar_amd/libgx.so for gfx950 (hipcc, no JIT cache)."""
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = [os.path.join(HERE, "csrc", "gx_engine.hip"), os.path.join(HERE, "csrc", "gx_sort.hip")]
DEPS = SRC + sorted(glob.glob(os.path.join(HERE, "csrc", "*.hpp"))) + [os.path.join(ROOT, "include", "gx.h")]
OUT = os.path.join(HERE, "libgx.so")
ARCH = os.environ.get("GX_OFFLOAD_ARCH", "gfx950")


def needs_build():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(p) > t for p in DEPS)


def build(force=False, verbose=True):
    if not force and not needs_build():
        return OUT
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-function", "-o", OUT + ".tmp"] + SRC
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
