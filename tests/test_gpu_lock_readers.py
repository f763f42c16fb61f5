"""Push-pull exchanges with a read-locked side (gx.h lock_readers, k_ae_ro / k_defer_drain) on the
HIP engine against the oracle, bit for bit: views, host states (lock words with the write-lock and
waiting-merge bits), queue digests, server times and every counter (ae_deferred and ae_defer_lost
included). Go's sync.RWMutex admits LocalState's RLock (services_delegate.go:148) while only
BroadcastServices' read lock (services_state.go:535) holds the lock and no writer waits; the
read-locked side's merge waits behind the lock (services_state.go:367-373 -> UpdateService
:138-140). The schedules are small clusters at fanout 1 with one-record packets and short looper
intervals, where a locked host's pipeline often stays empty (on the BASELINE schedules such
exchanges are rare: DESIGN.md §3d); lock_defer_slots 1 and 2 make pool slots collide."""
import pytest

from sidecar_amd.abi import INIT_OWN, Engine, default_params
from tests.parity import assert_same

pytestmark = pytest.mark.gpu

BASE = dict(n_hosts=32, n_services=4, fanout=1, packet_cap=1, init_mode=INIT_OWN, churn_ppm=100000,
            alive_interval_rounds=2, tombstone_interval_rounds=7, ae_period_rounds=1, queue_cap=4096,
            storm_round=5, lock_readers=1)

SCENARIOS = {
    "matching": {},
    "matching_pool2": dict(lock_defer_slots=2),
    "initiate": dict(push_pull_mode=1),
    "initiate_pool1": dict(push_pull_mode=1, lock_defer_slots=1),
    "fd": dict(fd_enable=1),
    "odd_rows": dict(n_hosts=33, n_services=3),
    "gm4": dict(gossip_messages=4),
    "h128": dict(n_hosts=128),
    "pp2_cap4": dict(ae_period_rounds=2, packet_cap=4),
}


def _pair(oracle_lib, gx_lib, **kw):
    g = Engine(default_params(gx_lib, **kw), lib=gx_lib)
    o = Engine(default_params(oracle_lib, **kw), lib=oracle_lib)
    return g, o


@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_lock_readers_parity(oracle_lib, gx_lib, name):
    kw = dict(BASE)
    kw.update(SCENARIOS[name])
    g, o = _pair(oracle_lib, gx_lib, **kw)
    for chunk in (1, 4, 10, 35, 50, 100, 100):
        g.run_rounds(chunk)
        o.run_rounds(chunk)
        assert_same(g, o, f"{name} round {g.round}")
    st = g.stats()
    assert st["ae_deferred"] > 0, st
    if kw.get("lock_defer_slots", 0) in (1, 2):
        assert st["ae_defer_lost"] > 0, st


def test_lock_readers_events_parity(oracle_lib, gx_lib):
    """A waiting merge's ChangeEvents come at the receive phase of the host's first unlocked round,
    before its pipeline's and that round's packets'."""
    kw = dict(BASE)
    kw.update(gossip_messages=4)
    g, o = _pair(oracle_lib, gx_lib, **kw)
    views = [(v, 1, 4096) for v in range(0, 32, 3)]
    for v, lid, cap in views:
        g.add_listener(v, lid, cap)
        o.add_listener(v, lid, cap)
    n_ev = 0
    for chunk in (1, 9, 40, 100, 150):
        g.run_rounds(chunk)
        o.run_rounds(chunk)
        assert_same(g, o, f"events round {g.round}")
        for v, lid, cap in views:
            ge = [x.tup() for x in g.drain_listener(v, lid, cap)]
            oe = [x.tup() for x in o.drain_listener(v, lid, cap)]
            assert ge == oe, f"view {v} round {g.round}"
            n_ev += len(ge)
    assert n_ev > 0 and g.stats()["ae_deferred"] > 0


def test_lock_readers_off_is_round5(oracle_lib, gx_lib):
    """lock_readers = 0 (the default) is the round-5 model: every exchange with a locked side fails."""
    kw = dict(BASE)
    kw["lock_readers"] = 0
    g, o = _pair(oracle_lib, gx_lib, **kw)
    g.run_rounds(120)
    o.run_rounds(120)
    assert_same(g, o, "lock_readers 0")
    st = g.stats()
    assert st["ae_deferred"] == 0 and st["ae_defer_lost"] == 0 and st["ae_locked"] > 0
