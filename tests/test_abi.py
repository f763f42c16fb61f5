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
    assert lib.gx_abi_version() == 1
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
        assert getattr(a, f) == getattr(b, f), f
