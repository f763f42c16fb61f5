"""The two memberlist scheduling knobs of the round model (the memberlist fork is
absent, so these readings are parity unpinned and checked here for their defining properties):

* GossipMessages (config/config.go:46, main.go:257-259; README.md:180 "How many times to gather
  messages per round", default 15): up to N GetBroadcasts gathers per gossip target and round, each
  its own packet; a target's gathering ends at an empty result.
* per-node push-pull initiation (memberlist's pushPull timer per node, PushPullInterval
  config/config.go:45): every live host starts one exchange per push-pull round with a random peer.
"""
import numpy as np
import pytest

from sidecar_amd.abi import INIT_OWN, INIT_WARM, Engine, default_params, load_library
from tests.oracle_lib import load_oracle


def _eng(lib, **kw):
    return Engine(default_params(lib, **kw), lib=lib)


def test_gossip_messages_one_is_the_default(oracle_lib):
    kw = dict(n_hosts=48, n_services=6, init_mode=INIT_OWN, churn_ppm=40000, ae_period_rounds=10)
    a, b = _eng(oracle_lib, **kw), _eng(oracle_lib, gossip_messages=1, **kw)
    a.run_rounds(60)
    b.run_rounds(60)
    assert a.stats() == b.stats()
    assert np.array_equal(a.read_views(), b.read_views())


def test_gossip_messages_drains_queues_faster(oracle_lib):
    """A cold start (every owner announces its records): with 15 gathers per target a host's queued
    batches leave up to 15x faster, so more records are sent per round and the catalog agrees
    sooner; every record sent is still merged exactly once."""
    kw = dict(n_hosts=64, n_services=8, init_mode=INIT_OWN, queue_cap=4096)
    one, many = _eng(oracle_lib, **kw), _eng(oracle_lib, gossip_messages=15, **kw)
    conv = {}
    for name, e in (("one", one), ("many", many)):
        for _ in range(40):
            e.run_rounds(5)
            if e.converged()[0]:
                break
        conv[name] = e.stats()["last_change_round"]
        st = e.stats()
        assert st["gossip_merges"] == st["records_sent"]
    s1, s15 = one.stats(), many.stats()
    assert s15["packets"] > s1["packets"]
    assert conv["many"] <= conv["one"]


def test_gossip_messages_validation(oracle_lib):
    from sidecar_amd.abi import GxError
    for bad in (dict(gossip_messages=17), dict(inbox_slots=257)):
        with pytest.raises(GxError):
            _eng(oracle_lib, n_hosts=16, n_services=2, **bad)
    # GossipMessages runs with the failure detector too (each gather takes memberlist's queue first)
    e = _eng(oracle_lib, n_hosts=16, n_services=2, gossip_messages=2, fd_enable=1)
    e.run_rounds(3)


def test_push_pull_initiate_every_host_starts_one(oracle_lib):
    """Per AE round every live host initiates exactly one exchange, so H exchanges per round
    (the matching has H/2) and a host takes part in 1 + (times drawn) of them."""
    H = 64
    kw = dict(n_hosts=H, n_services=4, init_mode=INIT_WARM, ae_period_rounds=5)
    m, i = _eng(oracle_lib, **kw), _eng(oracle_lib, push_pull_mode=1, **kw)
    m.run_rounds(11)  # AE rounds 0, 5, 10
    i.run_rounds(11)
    assert m.stats()["ae_exchanges"] == 3 * (H // 2)
    assert i.stats()["ae_exchanges"] == 3 * H
    assert i.stats()["ae_slots"] == 3 * H * 2 * H * 4


def test_push_pull_initiate_departed_hosts_do_not_exchange(oracle_lib):
    H = 80
    kw = dict(n_hosts=H, n_services=4, init_mode=INIT_WARM, ae_period_rounds=4, push_pull_mode=1,
              depart_round=2, depart_ppm=100000)
    e = _eng(oracle_lib, **kw)
    e.run_rounds(5)  # AE rounds 0 (all up) and 4 (crashed hosts out)
    st = e.stats()
    assert H < st["ae_exchanges"] < 2 * H


def test_push_pull_initiate_validation(oracle_lib):
    from sidecar_amd.abi import GxError
    for bad in (dict(push_pull_mode=2), dict(push_pull_mode=1, fd_enable=1),
                dict(push_pull_mode=1, n_shards=2, shard_id=0)):
        with pytest.raises(GxError):
            _eng(oracle_lib, n_hosts=16, n_services=2, **bad)


def test_round_end_bounded(oracle_lib):
    """Rounds are 32-bit in jobs and sleepers (gx.h GX_MAX_ROUND): the sharded stepping path refuses
    to pass the bound like gx_set_round and gx_run_rounds do."""
    from sidecar_amd.abi import Engine, GxError, default_params
    e = Engine(default_params(oracle_lib, n_hosts=4, n_services=2), lib=oracle_lib)
    e.set_round((1 << 31) - 2)
    e.round_end()
    assert e.round == (1 << 31) - 1
    with pytest.raises(GxError):
        e.round_end()
