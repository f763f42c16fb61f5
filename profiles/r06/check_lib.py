"""Parity spot-check of an alternative engine build against the oracle (round-model scenarios of
tests/test_gpu_parity.py and tests/test_gpu_lock.py, bit for bit), before timing it.
    python profiles/r06/check_lib.py path/to/libgx_variant.so"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from sidecar_amd.abi import Engine, default_params, load_library  # noqa: E402
from tests.oracle_lib import load_oracle  # noqa: E402
from tests.parity import assert_same  # noqa: E402
from tests.test_gpu_lock import SCENARIOS as LOCK  # noqa: E402
from tests.test_gpu_parity import SCENARIOS as PAR  # noqa: E402

lib, orc = load_library(sys.argv[1]), load_oracle()
scen = dict(PAR)
scen.update(LOCK)
for name, kw in sorted(scen.items()):
    g = Engine(default_params(lib, **kw), lib=lib)
    o = Engine(default_params(orc, **kw), lib=orc)
    for chunk in (1, 4, 10, 35, 50):
        g.run_rounds(chunk)
        o.run_rounds(chunk)
        assert_same(g, o, f"{name} round {g.round}")
    g.close()
    o.close()
    print("ok", name, flush=True)
print("all ok")
