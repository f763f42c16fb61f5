"""Builds the HIP engine in-tree: sidecar_amd/libgx.so for gfx950 (hipcc, no JIT cache)."""
import glob
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = [os.path.join(HERE, "csrc", "gx_engine.hip"), os.path.join(HERE, "csrc", "gx_sort.hip")]
DEPS = SRC + sorted(glob.glob(os.path.join(HERE, "csrc", "*.hpp"))) + [os.path.join(ROOT, "include", "gx.h")]
OUT = os.path.join(HERE, "libgx.so")
ARCH = os.environ.get("GX_OFFLOAD_ARCH", "gfx950")


STAMP = OUT + ".sha256"  # the sources a build compiled (travels with the .so; git-ignored)


def source_hash():
    """sha256 over the engine's sources and headers, path and content, in a fixed order."""
    h = hashlib.sha256()
    for p in DEPS:
        h.update(os.path.relpath(p, ROOT).encode())
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def built_hash():
    try:
        with open(STAMP) as f:
            return f.read().strip()
    except OSError:
        return None


def needs_build():
    """The library is missing or was built from other sources than these (a content hash, not
    mtimes: a source edited while a build ran, or a checkout, can carry an older mtime)."""
    return not os.path.exists(OUT) or built_hash() != source_hash()


def build(force=False, verbose=True):
    if not force and not needs_build():
        return OUT
    h = source_hash()  # the sources as this build reads them
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-function", "-o", OUT + ".tmp"] + SRC
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    if source_hash() == h:  # a source edited during the build leaves the stamp stale: rebuilt next time
        with open(STAMP, "w") as f:
            f.write(h + "\n")
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
