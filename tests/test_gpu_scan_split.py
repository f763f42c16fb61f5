"""The worklist expiry scan with rows split over blocks (k_scan_split + k_scan_join, round 6) against
the oracle, bit for bit: rows of 64K and 256K slots (2 and 8 chunks), aged records so that every
tick expires some, churn, push-pull, and the lock on and off."""
import pytest

from sidecar_amd.abi import INIT_WARM, Engine, default_params
from tests.oracle_lib import load_oracle
from tests.parity import assert_same

pytestmark = pytest.mark.gpu

CASES = {
    "r64k_s16": dict(n_hosts=4096, n_services=16),
    "r64k_s64_lock_off": dict(n_hosts=1024, n_services=64, lock_model=0),
    "r256k_s64": dict(n_hosts=4096, n_services=64),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_scan_split_parity(gx_lib, name):
    omp = load_oracle(omp=True)
    kw = dict(CASES[name], init_mode=INIT_WARM, aged_ppm=200000, aged_max_ns=100 * 10**9, churn_ppm=20000,
              ae_period_rounds=10, queue_cap=4096)
    g = Engine(default_params(gx_lib, **kw), lib=gx_lib)
    o = Engine(default_params(omp, **kw), lib=omp)
    for chunk in (11, 20, 30):
        g.run_rounds(chunk)
        o.run_rounds(chunk)
        assert_same(g, o, f"{name} round {g.round}")
    st = g.stats()
    assert st["expired"] > 0 and st["scan_slots"] > 0
