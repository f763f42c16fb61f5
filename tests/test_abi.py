"""The C-ABI library loads and exports every symbol include/gx.h declares (no GPU calls)."""
import os
import re

import pytest

from sidecar_amd.abi import ABI_FUNCS, LIBGX_PATH, load_library

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "gx.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char \*)\s*(gx_\w+)\s*\(", src, re.M)))


def test_header_matches_binding():
    assert declared_symbols() == sorted(ABI_FUNCS)


def test_libgx_exports_every_symbol():
    if not os.path.exists(LIBGX_PATH):
        from sidecar_amd.build import build
        build()
    lib = load_library(LIBGX_PATH)
    for name in declared_symbols():
        assert hasattr(lib, name), name
    assert lib.gx_abi_version() == 11
    assert lib.gx_backend().decode() == "hip-gfx950"


def test_oracle_exports_every_symbol(oracle_lib):
    for name in declared_symbols():
        assert hasattr(oracle_lib, name), name
    assert oracle_lib.gx_backend().decode() == "oracle-cpu"


def test_params_default_identical(oracle_lib):
    from sidecar_amd.abi import default_params
    if not os.path.exists(LIBGX_PATH):
        pytest.skip("libgx not built")
    a = default_params(oracle_lib)
    b = default_params(load_library(LIBGX_PATH))
    for f, _ in a._fields_:
        x, y = getattr(a, f), getattr(b, f)
        if hasattr(x, "_length_"):  # ctypes array
            x, y = list(x), list(y)
        assert x == y, f


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 9, 10, 63, 64, 99, 100, 999, 1000, 4096, 16384, 32768, 65534])
def test_fd_defaults_identical(oracle_lib, n):
    """memberlist's size-derived parameters (retransmitLimit, Lifeguard suspicion timeouts) agree
    between the product and the oracle, and follow util.go / suspicion.go."""
    import ctypes as C
    import math
    from sidecar_amd.abi import GxParams
    if not os.path.exists(LIBGX_PATH):
        pytest.skip("libgx not built")
    got = []
    for lib in (oracle_lib, load_library(LIBGX_PATH)):
        p = GxParams()
        lib.gx_params_default(C.byref(p))
        p.n_hosts = n
        assert lib.gx_fd_defaults(C.byref(p)) == 0
        got.append((p.fd_retransmit_limit, p.fd_suspicion_k, list(p.fd_suspicion_rounds)))
    assert got[0] == got[1]
    limit, k, rounds = got[0]
    assert limit == min(32, 4 * math.ceil(math.log10(n + 1)))
    assert k == (0 if n - 2 < 2 else 2)
    tmin_ms = 4 * int(max(1.0, math.log10(max(1, n))) * 1000) * 1000 // 1000  # ProbeInterval 1 s
    assert rounds[0] == math.ceil((tmin_ms if k < 1 else 6 * tmin_ms) / 200)
    if k:
        assert rounds[k] == math.ceil(tmin_ms / 200)  # k confirmations: the minimum
        assert rounds[0] >= rounds[1] >= rounds[2]


def test_libgx_is_built_from_these_sources():
    """The in-tree library the GPU tiers load was compiled from the sources in the tree (build.py's
    content stamp, written by the build that produced it): a stale binary cannot pass for HEAD."""
    from sidecar_amd import build
    if build.needs_build():
        build.build()
    assert build.built_hash() == build.source_hash()
