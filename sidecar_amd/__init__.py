"""sidecar_amd — MI355X-native gossip-convergence engine for Sidecar's catalog merge path.

The compute path is the HIP library ``sidecar_amd/libgx.so`` (gfx950) behind the C-ABI in
``include/gx.h``. ``Engine`` is a thin Python handle over that ABI; ``catalog`` mirrors the
reference's ``catalog.ServicesState`` / memberlist delegate method names on top of it.
"""
from .abi import (ABSENT, ALIVE, DRAINING, TOMBSTONE, UNHEALTHY, UNKNOWN, Engine, GxError,  # noqa: F401
                  default_params, load_product)

__all__ = ["Engine", "GxError", "default_params", "load_product", "ALIVE", "TOMBSTONE", "UNHEALTHY",
           "UNKNOWN", "DRAINING", "ABSENT"]
