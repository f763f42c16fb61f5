"""EachServiceSorted / SortedServices / ByService (catalog/view.go:14-58, services_state.go:726-748)
on the device against the oracle, on catalogs the round model built (ties in Updated are common:
a storm tombstones whole servers at one instant)."""
import numpy as np
import pytest

from sidecar_amd.abi import INIT_WARM, Engine, default_params

pytestmark = pytest.mark.gpu


def _tup(x):
    return (x.host, x.svc, x.updated_ns, x.status)


@pytest.mark.parametrize("kw", [
    dict(n_hosts=64, n_services=8, init_mode=INIT_WARM, partition_start=0, partition_end=20, storm_round=3,
         ae_period_rounds=10, churn_ppm=50000, queue_cap=4096),
    dict(n_hosts=300, n_services=5, init_mode=1, ae_period_rounds=7, churn_ppm=80000, aged_ppm=50000),
])
def test_sorted_readers_match_oracle(gx_lib, oracle_lib, kw):
    g = Engine(default_params(gx_lib, **kw), lib=gx_lib)
    o = Engine(default_params(oracle_lib, **kw), lib=oracle_lib)
    g.run_rounds(40)
    o.run_rounds(40)
    rnd = np.random.default_rng(7)
    names = [f"svc-{int(x)}" for x in rnd.integers(0, 7, size=g.H * g.S)]
    g.set_service_names(names)
    o.set_service_names(names)
    for v in (0, 1, g.H // 2, g.H - 1):
        a, b = g.each_service_sorted(v), o.each_service_sorted(v)
        assert [_tup(x) for x in a] == [_tup(x) for x in b], v
        assert len(a) == len(g.local_state(v))
        for owner in (0, v, g.H - 1):
            assert [_tup(x) for x in g.each_service_sorted(v, owner)] == [_tup(x) for x in o.each_service_sorted(v, owner)]
        ga, gb = g.by_service(v), o.by_service(v)
        assert [(k, _tup(x)) for k, x in ga] == [(k, _tup(x)) for k, x in gb], v
