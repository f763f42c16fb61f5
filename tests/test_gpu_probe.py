"""Probe-traffic piggybacking (gx.h probe_piggyback, k_probe) and staggered push-pull timers (push_pull_stagger)
on the HIP engine against the oracle,
bit for bit: views, bookkeeping, queue digests, server times and every counter (false_expiries
included), with the lock on and off, GossipMessages, byte mode, departures and the partition."""
import pytest

from sidecar_amd.abi import INIT_OWN, INIT_WARM, Engine, default_params
from tests.parity import assert_same

pytestmark = pytest.mark.gpu

SCENARIOS = {
    "probe_cfg1_own": dict(n_hosts=64, n_services=8, init_mode=INIT_OWN, ae_period_rounds=10, queue_cap=4096),
    "probe_storm_partition": dict(n_hosts=96, n_services=4, init_mode=INIT_WARM, partition_start=0, partition_end=20,
                                  storm_round=4, ae_period_rounds=10, queue_cap=4096),
    "probe_storm_lock_off": dict(n_hosts=96, n_services=4, init_mode=INIT_WARM, partition_start=0, partition_end=20,
                                 storm_round=4, ae_period_rounds=10, queue_cap=4096, lock_model=0),
    "probe_gm15_churn": dict(n_hosts=64, n_services=8, init_mode=INIT_OWN, gossip_messages=15, churn_ppm=50000,
                             ae_period_rounds=10, queue_cap=2048),
    "probe_bytes": dict(n_hosts=64, n_services=8, init_mode=INIT_WARM, limit_bytes=1398, overhead_bytes=3,
                        churn_ppm=50000, ae_period_rounds=10, queue_cap=4096),
    "probe_depart_aged": dict(n_hosts=80, n_services=4, init_mode=INIT_WARM, aged_ppm=200000,
                              aged_max_ns=100 * 10**9, depart_round=6, depart_ppm=100000, ae_period_rounds=10,
                              queue_cap=4096),
    "probe_pp_initiate": dict(n_hosts=64, n_services=8, init_mode=INIT_OWN, push_pull_mode=1, ae_period_rounds=5,
                              churn_ppm=30000, queue_cap=4096),
    "probe_tiny_h3": dict(n_hosts=3, n_services=2, init_mode=INIT_OWN, ae_period_rounds=3),
    # memberlist's staggered push-pull timers (gx.h push_pull_stagger), with and without the probes
    "pp_stagger": dict(n_hosts=64, n_services=8, init_mode=INIT_WARM, push_pull_mode=1, push_pull_stagger=1,
                       ae_period_rounds=20, churn_ppm=30000, queue_cap=4096, probe=0),
    "pp_stagger_probe_gm15_storm": dict(n_hosts=96, n_services=4, init_mode=INIT_WARM, push_pull_mode=1,
                                        push_pull_stagger=1, ae_period_rounds=10, gossip_messages=15,
                                        partition_start=0, partition_end=20, storm_round=4, queue_cap=4096),
}


@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_probe_parity(oracle_lib, gx_lib, name):
    kw = dict(SCENARIOS[name])
    kw["probe_piggyback"] = kw.pop("probe", 1)
    g = Engine(default_params(gx_lib, **kw), lib=gx_lib)
    o = Engine(default_params(oracle_lib, **kw), lib=oracle_lib)
    for chunk in (1, 4, 10, 35, 50, 150):
        g.run_rounds(chunk)
        o.run_rounds(chunk)
        assert_same(g, o, f"{name} round {g.round}")
    st = g.stats()
    assert st["packets"] > 0
    if name == "probe_depart_aged":
        assert 0 < st["false_expiries"] < st["expired"]
