"""Loads the CPU oracle (oracle/liboracle_gx.so) — test infrastructure only.

Builds it with the committed Makefile if the shared object is missing (gcc is present both in
the build container and on the GPU box)."""
import os
import subprocess

from sidecar_amd.abi import load_library

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liboracle_gx.so")
ORACLE_OMP_SO = os.path.join(ORACLE_DIR, "liboracle_gx_omp.so")  # multi-threaded CPU baseline


def build_oracle():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def load_oracle(omp=False):
    """The serial oracle (the checker), or with omp=True the same source built with its per-host
    phase loops on OpenMP threads (bench.py's multi-threaded cpu_baseline)."""
    so = ORACLE_OMP_SO if omp else ORACLE_SO
    src = os.path.join(ORACLE_DIR, "gx_oracle.c")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        build_oracle()
    lib = load_library(so)
    assert lib.gx_backend().decode() == "oracle-cpu"
    return lib
