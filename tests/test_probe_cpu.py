"""Probe-traffic piggybacking (gx.h probe_piggyback) and the false_expiries counter on the CPU
oracle. memberlist's sendMsg hands the delegate's GetBroadcasts every outgoing UDP message (the
absent fork's net.go; parity unpinned), so besides gossip() a host's probe ping and its ack to the
host that pinged it each carry one GetBroadcasts result. These tests pin the knob's defining
properties; tests/test_gpu_probe.py compares the HIP engine with the oracle bit for bit."""
import numpy as np
import pytest

from sidecar_amd.abi import INIT_OWN, INIT_WARM, Engine, GxError, default_params


def _eng(lib, **kw):
    return Engine(default_params(lib, **kw), lib=lib)


def test_probe_off_is_the_default(oracle_lib):
    kw = dict(n_hosts=48, n_services=6, init_mode=INIT_OWN, churn_ppm=40000, ae_period_rounds=10)
    a, b = _eng(oracle_lib, **kw), _eng(oracle_lib, probe_piggyback=0, **kw)
    a.run_rounds(60)
    b.run_rounds(60)
    assert a.stats() == b.stats()
    assert np.array_equal(a.read_views(), b.read_views())


@pytest.mark.parametrize("bad", [dict(probe_piggyback=2), dict(probe_piggyback=1, fd_enable=1),
                                 dict(probe_piggyback=1, n_shards=2, shard_id=0),
                                 dict(probe_piggyback=1, fd_probe_rounds=0)])
def test_probe_rejects_unsupported_modes(oracle_lib, bad):
    with pytest.raises(GxError):
        _eng(oracle_lib, n_hosts=16, n_services=4, **bad)


def test_probe_calls_add_packets_and_spread_sooner(oracle_lib):
    """A cold start with probe traffic: two more GetBroadcasts calls per host and probe interval,
    so more batches leave per round; every record sent is still merged once (gossip_merges counts
    the records sent to live receivers)."""
    kw = dict(n_hosts=64, n_services=8, init_mode=INIT_OWN, queue_cap=4096, lock_model=0)
    off, on = _eng(oracle_lib, **kw), _eng(oracle_lib, probe_piggyback=1, **kw)
    off.run_rounds(40)
    on.run_rounds(40)
    a, b = off.stats(), on.stats()
    assert b["dequeues"] > a["dequeues"] and b["packets"] > a["packets"]
    # ~2 calls per host per 5 rounds on top of 3 per round: at most 2/15 more dequeues
    assert b["dequeues"] <= a["dequeues"] * (1 + 2 / 15) * 1.25
    assert b["gossip_merges"] == b["records_sent"] and b["lost_packets"] == 0


def test_probe_pings_across_the_partition_are_lost(oracle_lib):
    """Probe targets come from all hosts, not the sampling side: during a partition a ping to the
    other half is lost after GetBroadcasts took its records (records sent, never merged), and gets
    no ack; after the heal nothing is lost."""
    kw = dict(n_hosts=64, n_services=4, init_mode=INIT_WARM, churn_ppm=100000, partition_start=0,
              partition_end=40, queue_cap=4096, lock_model=0)
    e = _eng(oracle_lib, probe_piggyback=1, **kw)
    e.run_rounds(40)
    st = e.stats()
    assert st["lost_packets"] > 0 and st["records_sent"] > st["gossip_merges"]
    e.run_rounds(40)
    st2 = e.stats()
    assert st2["lost_packets"] == st["lost_packets"]
    assert st2["records_sent"] - st["records_sent"] == st2["gossip_merges"] - st["gossip_merges"]


def test_false_expiries_count_live_owners(oracle_lib):
    """false_expiries counts the alive-lifespan expiries of records whose owner has not departed:
    all of `expired` without departures, fewer with them."""
    kw = dict(n_hosts=48, n_services=4, init_mode=INIT_WARM, aged_ppm=300000, aged_max_ns=100 * 10**9,
              ae_period_rounds=10, queue_cap=4096)
    e = _eng(oracle_lib, **kw)
    e.run_rounds(60)
    st = e.stats()
    assert st["expired"] > 0 and st["false_expiries"] == st["expired"]
    d = _eng(oracle_lib, depart_round=1, depart_ppm=300000, **kw)
    d.run_rounds(600)
    sd = d.stats()
    assert 0 < sd["false_expiries"] < sd["expired"]


@pytest.mark.parametrize("bad", [dict(push_pull_stagger=2), dict(push_pull_stagger=1),
                                 dict(push_pull_stagger=1, push_pull_mode=1, ae_period_rounds=0)])
def test_push_pull_stagger_rejects_unsupported_modes(oracle_lib, bad):
    kw = dict(n_hosts=16, n_services=4, ae_period_rounds=10)
    kw.update(bad)
    with pytest.raises(GxError):
        _eng(oracle_lib, **kw)


def test_push_pull_stagger_spreads_the_exchanges(oracle_lib):
    """memberlist's staggered push-pull timers (gx.h push_pull_stagger): every host still initiates
    once per interval, but in the rounds of its own phase, so exchanges happen in most rounds and the
    total over whole intervals equals the aligned model's."""
    kw = dict(n_hosts=64, n_services=4, init_mode=INIT_WARM, push_pull_mode=1, ae_period_rounds=10, queue_cap=4096,
              lock_model=0)
    al, st = _eng(oracle_lib, **kw), _eng(oracle_lib, push_pull_stagger=1, **kw)
    rounds_with = 0
    for _ in range(40):
        a0 = st.stats()["ae_exchanges"]
        st.run_rounds(1)
        rounds_with += st.stats()["ae_exchanges"] > a0
    al.run_rounds(40)
    assert al.stats()["ae_exchanges"] == st.stats()["ae_exchanges"] == 4 * 64
    assert rounds_with >= 30
